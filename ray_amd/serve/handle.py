"""DeploymentHandle / DeploymentResponse and the replica router (reference:
python/ray/serve/handle.py, _private/router.py, _private/replica_scheduler/pow_2_scheduler.py).

Routing: power-of-two-choices on the number of requests this handle has in
flight to each replica (no extra RPC on the hot path). Replica-set changes arrive by
long poll (one ``_LongPoller`` thread per process blocks in the controller's
``long_poll`` and installs new versions as they are published; reference
serve/_private/long_poll.py:173); an explicit refresh happens only before the first
update or after a replica failure. A ``_MetricsPusher`` thread reports the requests each
handle holds back to the controller's autoscaler."""

from __future__ import annotations

import asyncio
import random
import threading
import time

import ray_amd as ray


class _Router:
    def __init__(self, app_name, deployment_name):
        self.app = app_name
        self.dep = deployment_name
        self.version = -1
        self.replicas = []  # [(rid, handle)]
        self.inflight = {}
        self.max_ongoing = 100
        self.max_queued = -1
        self.queued = 0  # requests of this handle waiting for a replica slot
        self.lock = threading.Lock()
        self.slot_freed = threading.Condition(self.lock)
        self.pending = []  # [(future, send, model_id)] waiting for a slot, FIFO
        self.dispatching = False
        self.last_refresh = 0.0
        self.stale = False
        self.affinity = {}  # multiplexed model id -> replica that loaded it
        # replicas a request of this handle saw die: skipped until the controller's replica
        # set no longer lists them (its health check has not noticed the death yet)
        self.dead = set()

    def _controller(self):
        from ray_amd.serve.api import _get_controller

        return _get_controller()

    def refresh(self, force=False):
        now = time.time()
        if not force and not self.stale and self.replicas and (
                now - self.last_refresh < 1.0 or _poller.alive):
            return
        info = ray.get(self._controller().get_replicas.remote(self.app, self.dep))
        self.last_refresh = now
        self.stale = False
        if info is None:
            raise RuntimeError(f"deployment {self.dep} of app {self.app} does not exist")
        self._install(info)

    def _install(self, info):
        version, reps, mo, mq = info
        with self.lock:
            listed = {rid for rid, _ in reps}
            self.dead &= listed  # the controller dropped them: forget
            reps = [x for x in reps if x[0] not in self.dead]
            if version != self.version or len(reps) != len(self.replicas):
                self.version = version
                self.replicas = reps
                self.inflight = {rid: self.inflight.get(rid, 0) for rid, _ in reps}
            self.max_ongoing = mo
            self.max_queued = mq
            self.slot_freed.notify_all()

    async def arefresh(self, force=False):
        now = time.time()
        if not force and not self.stale and self.replicas and (
                now - self.last_refresh < 1.0 or _poller.alive):
            return
        info = await self._controller().get_replicas.remote(self.app, self.dep)
        self.last_refresh = now
        self.stale = False
        if info is None:
            raise RuntimeError(f"deployment {self.dep} of app {self.app} does not exist")
        self._install(info)

    def _admit(self):
        """Count this request as queued, or raise BackPressureError when the handle's
        queue is full (reference: max_queued_requests in the replica scheduler)."""
        waiting = self.queued + len(self.pending)
        if self.max_queued != -1 and waiting >= self.max_queued:
            from ray_amd.serve.exceptions import BackPressureError

            raise BackPressureError(num_queued_requests=waiting,
                                    max_queued_requests=self.max_queued)
        self.queued += 1

    def assign(self, send, model_id=""):
        """Non-blocking routing for DeploymentHandle.remote: ``(rid, send(h))`` when a
        replica has a free slot, else a Future of it that the dispatcher thread fulfils
        in arrival order as slots free up (or fails with BackPressureError)."""
        import concurrent.futures

        self.choose_wait_for_replicas()
        with self.lock:
            got = None if self.pending else self._pick(model_id)
            if got is None:
                fut = concurrent.futures.Future()
                try:
                    self._admit()
                    self.queued -= 1  # counted as pending instead
                except Exception as e:  # noqa: BLE001  (BackPressureError)
                    fut.set_exception(e)
                    return fut
                self.pending.append((fut, send, model_id))
                if not self.dispatching:
                    self.dispatching = True
                    threading.Thread(target=self._dispatch, daemon=True,
                                     name=f"serve-dispatch-{self.dep}").start()
                return fut
        slot = _Slot(self, got[0])
        try:
            ref = send(got[1])
        except BaseException:
            slot.release()
            raise
        _watch(slot, ref)
        return slot, ref

    def cancel_pending(self, fut) -> bool:
        with self.lock:
            for i, item in enumerate(self.pending):
                if item[0] is fut:
                    del self.pending[i]
                    fut.cancel()
                    return True
        return False

    def _dispatch(self):
        while True:
            ready = []
            with self.lock:
                if not self.pending:
                    self.dispatching = False
                    return
                self.slot_freed.wait(0.05)
                while self.pending:
                    got = self._pick(self.pending[0][2])
                    if got is None:
                        break
                    ready.append((self.pending.pop(0), got))
            for (fut, send, _), (rid, h) in ready:
                slot = _Slot(self, rid)
                try:
                    ref = send(h)
                except BaseException as e:  # noqa: BLE001
                    slot.release()
                    fut.set_exception(e)
                    continue
                _watch(slot, ref)
                fut.set_result((slot, ref))
            try:
                self.refresh()
            except RuntimeError as e:  # the deployment was deleted: fail what still waits
                with self.lock:
                    waiting, self.pending = self.pending, []
                for fut, _, _ in waiting:
                    fut.set_exception(e)
            except Exception:  # noqa: BLE001  (controller briefly unreachable: retry)
                pass

    def choose_wait_for_replicas(self):
        deadline = time.time() + 30
        while True:
            self.refresh()
            with self.lock:
                if self.replicas:
                    return
            if time.time() > deadline:
                raise RuntimeError(f"no replicas available for {self.dep}")
            time.sleep(0.05)
            self.refresh(force=True)

    async def achoose(self, model_id=""):
        """choose() for event loops: refreshes are awaited and a request waiting for a
        replica slot yields to the loop instead of blocking it."""
        deadline = time.time() + 30
        await self.arefresh()
        while not self.replicas:
            if time.time() > deadline:
                raise RuntimeError(f"no replicas available for {self.dep}")
            await asyncio.sleep(0.05)
            await self.arefresh(force=True)
        with self.lock:
            got = self._pick(model_id)
            if got is not None:
                return got
            self._admit()
        try:
            while True:
                await asyncio.sleep(0.002)
                await self.arefresh()
                with self.lock:
                    got = self._pick(model_id)
                if got is not None:
                    return got
        finally:
            with self.lock:
                self.queued -= 1

    def choose(self, model_id=""):
        self.choose_wait_for_replicas()
        with self.lock:
            got = self._pick(model_id)
            if got is not None:
                return got
            self._admit()
        try:
            while True:
                with self.lock:
                    self.slot_freed.wait(0.1)
                    got = self._pick(model_id)
                if got is not None:
                    return got
                self.refresh()
        finally:
            with self.lock:
                self.queued -= 1

    def _pick(self, model_id=""):
        """Caller holds self.lock. A replica below max_ongoing_requests, or None when all
        are at capacity (the request then waits at the handle, as in the reference)."""
        reps = [x for x in self.replicas if self.inflight.get(x[0], 0) < self.max_ongoing]
        if not reps:
            return None
        # multiplexed requests stick to the replica that already loaded the model
        # while it is below max_ongoing_requests (reference: replica_scheduler
        # multiplexed-model matching before power-of-two choices)
        prev = self.affinity.get(model_id) if model_id else None
        hit = next((x for x in reps if x[0] == prev), None)
        if hit is not None:
            rid, h = hit
        elif len(reps) == 1:
            rid, h = reps[0]
        else:
            a, b = random.sample(reps, 2)
            rid, h = a if self.inflight.get(a[0], 0) <= self.inflight.get(b[0], 0) else b
        if model_id:
            self.affinity[model_id] = rid
        self.inflight[rid] = self.inflight.get(rid, 0) + 1
        return rid, h

    def mark_dead(self, rid):
        """A request on replica ``rid`` failed with an actor death: stop routing to it
        before the controller's health check removes it from the replica set."""
        with self.lock:
            self.dead.add(rid)
            self.replicas = [x for x in self.replicas if x[0] != rid]
            self.inflight.pop(rid, None)
            self.slot_freed.notify_all()

    def done(self, rid):
        with self.lock:
            self._done_locked(rid)

    def _done_locked(self, rid):
        if rid in self.inflight:
            self.inflight[rid] = max(0, self.inflight[rid] - 1)
        self.slot_freed.notify()


_routers: dict = {}
_rlock = threading.Lock()


def _router(app, dep):
    with _rlock:
        r = _routers.get((app, dep))
        if r is None:
            r = _routers[(app, dep)] = _Router(app, dep)
    _poller.ensure()
    _pusher.ensure()
    return r


class _Daemon:
    name = "serve-daemon"

    def __init__(self):
        self.thread = None
        self.lock = threading.Lock()
        self.alive = False

    def ensure(self):
        with self.lock:
            if self.thread is None or not self.thread.is_alive():
                self.thread = threading.Thread(target=self._run_safe, daemon=True,
                                               name=self.name)
                self.thread.start()

    def _run_safe(self):
        try:
            self._run()
        finally:
            self.alive = False

    def _controller(self):
        from ray_amd.serve.api import _get_controller

        return _get_controller()


class _LongPoller(_Daemon):
    """Blocks in ServeController.long_poll with the versions this process holds and
    installs every change it returns (the push half of the routing-table protocol)."""

    name = "serve-long-poll"

    def _run(self):
        while ray.is_initialized():
            with _rlock:
                routers = dict(_routers)
            if not routers:
                self.alive = False
                time.sleep(0.1)
                continue
            snap = {f"{a}/{d}": r.version for (a, d), r in routers.items()}
            try:
                res = ray.get(self._controller().long_poll.remote(snap, 5.0), timeout=30)
            except Exception:  # noqa: BLE001  (controller restarting / serve shut down)
                self.alive = False
                time.sleep(0.2)
                continue
            self.alive = True
            now = time.time()
            for key, info in res.items():
                a, _, d = key.partition("/")
                r = routers.get((a, d))
                if r is None:
                    continue
                if info is None:  # deployment deleted
                    with r.lock:
                        r.version, r.replicas = -1, []
                        r.slot_freed.notify_all()
                else:
                    r._install(info)
                    r.last_refresh = now


class _MetricsPusher(_Daemon):
    """Every 0.25 s, reports each handle's held-back requests (queued for a replica
    slot) to the controller, which adds them to the replicas' ongoing requests when it
    autoscales over look_back_period_s."""

    name = "serve-handle-metrics"
    PERIOD_S = 0.25

    def _run(self):
        import os

        last = {}
        while ray.is_initialized():
            time.sleep(self.PERIOD_S)
            with _rlock:
                routers = dict(_routers)
            for (a, d), r in routers.items():
                q = r.queued + len(r.pending)
                if q or last.get((a, d)):
                    try:
                        self._controller().record_handle_metrics.remote(
                            a, d, f"{os.getpid()}:{id(r)}", q)
                    except Exception:  # noqa: BLE001
                        continue
                last[(a, d)] = q
            self.alive = True


_poller = _LongPoller()
_pusher = _MetricsPusher()


def invalidate(app, drop=True):
    """After a delete (drop=True) forget this process's routers of `app`; after a redeploy
    (drop=False) make their next use re-read the replica set (the long poll delivers it
    too, but the caller of serve.run must not route by a set older than its own deploy)."""
    with _rlock:
        for key in [k for k in _routers if k[0] == app]:
            if drop:
                del _routers[key]
            else:
                _routers[key].stale = True


def _is_replica_death(e) -> bool:
    from ray_amd.exceptions import RayActorError

    return isinstance(e, RayActorError)


class _Slot:
    """One request's claim on a replica's max_ongoing_requests budget; released exactly
    once, by whichever comes first: the reply landing or the caller finishing."""

    __slots__ = ("router", "rid", "released")

    def __init__(self, router, rid):
        self.router, self.rid, self.released = router, rid, False

    def release(self):
        # reply-landed callbacks (I/O thread) race the caller's own finish: decide under
        # the router lock so a slot is returned exactly once
        with self.router.lock:
            if self.released:
                return
            self.released = True
            self.router._done_locked(self.rid)


def _watch(slot: _Slot, ref) -> None:
    """Release the slot when the reply lands, whether or not the caller ever reads it
    (fire-and-forget requests must not hold max_ongoing_requests slots)."""
    cw = ref._cw
    if cw is None or cw._on_ready(ref._id, lambda _oid, ref=ref: slot.release()):
        slot.release()


class DeploymentResponse:
    """Reply of one handle call. The request may still wait at the handle for a replica
    slot (every replica at ``max_ongoing_requests``): ``pending`` then resolves to
    ``(slot, ref)`` once the router's dispatcher sends it, or raises BackPressureError
    (``max_queued_requests`` exceeded) / is cancelled.

    ``resend`` re-issues the request on a freshly chosen replica when the replica died
    before answering (killed, crashed, or a redeploy / scale-down raced the cached routing
    table; reference: the router retries requests whose replica became unavailable). The
    dead replica is excluded from this handle's routing at once, and up to MAX_RETRIES
    resends are made."""

    MAX_RETRIES = 3

    def __init__(self, ref, router, slot=None, resend=None, pending=None):
        self._ref = ref
        self._router = router
        self._slot = slot
        self._resend = resend
        self._pending = pending
        self._retries = 0

    def _retry(self):
        """The assigned replica died: stop routing to it, resend; None when out of
        retries (the caller re-raises)."""
        if self._resend is None or self._retries >= self.MAX_RETRIES:
            return None
        self._retries += 1
        if self._slot is not None:
            self._router.mark_dead(self._slot.rid)
        return self._resend

    def _assigned(self, timeout_s=None):
        if self._pending is not None:
            import concurrent.futures

            try:
                self._slot, self._ref = self._pending.result(timeout_s)
            except concurrent.futures.TimeoutError:
                raise ray.exceptions.GetTimeoutError(
                    "request still queued at the handle") from None
            except concurrent.futures.CancelledError:
                from ray_amd.serve.exceptions import RequestCancelledError

                raise RequestCancelledError("request cancelled while queued") from None
            self._pending = None
        return self._ref

    def _finish(self):
        if self._slot is not None:
            self._slot.release()

    def _adopt(self, again):
        self._finish()
        again._assigned()
        self._ref, self._slot = again._ref, again._slot

    def _give_up(self, e):
        # a timed-out wait leaves the request in flight: its slot is released by _watch
        # when the reply lands, not here (releasing now would over-admit the replica)
        if not isinstance(e, ray.exceptions.GetTimeoutError):
            self._finish()

    def result(self, timeout_s: float | None = None):
        while True:
            try:
                out = ray.get(self._assigned(timeout_s), timeout=timeout_s)
            except Exception as e:  # noqa: BLE001
                resend = self._retry() if _is_replica_death(e) else None
                if resend is None:
                    self._give_up(e)
                    raise
                self._router.refresh(force=True)
                again = resend()
                # releases the dead replica's slot; the retried request keeps its own
                # slot until its reply lands (_watch) or this loop returns / raises
                self._adopt(again)
                continue
            self._finish()
            return out

    def __await__(self):
        async def _w():
            if self._pending is not None:
                await asyncio.wrap_future(self._pending)
            while True:
                try:
                    out = await self._assigned()
                except Exception as e:  # noqa: BLE001
                    resend = self._retry() if _is_replica_death(e) else None
                    if resend is None:
                        self._give_up(e)
                        raise
                    await self._router.arefresh(force=True)
                    again = resend()
                    if again._pending is not None:
                        await asyncio.wrap_future(again._pending)
                    self._adopt(again)
                    continue
                self._finish()
                return out

        return _w().__await__()

    def _to_object_ref(self):
        return self._assigned()

    async def _to_object_ref_async(self):
        if self._pending is not None:
            await asyncio.wrap_future(self._pending)
        return self._assigned()

    def cancel(self):
        if self._pending is not None and self._router.cancel_pending(self._pending):
            return
        ray.cancel(self._assigned())

    def __reduce__(self):
        # passing a response to another deployment passes the underlying object
        return (_resolve, (self._assigned(),))


def _resolve(ref):
    return ref


class DeploymentResponseGenerator:
    """Streaming response (``handle.options(stream=True)``): iterate (sync or async) to
    receive each item the deployment's generator yields, as it is produced."""

    def __init__(self, gen, router, rid):
        self._gen = gen
        self._router = router
        self._rid = rid
        self._done = False

    def _finish(self):
        if not self._done:
            self._done = True
            self._router.done(self._rid)

    def __iter__(self):
        return self

    def __next__(self):
        try:
            ref = next(self._gen)
        except StopIteration:
            self._finish()
            raise
        return ray.get(ref)

    def __aiter__(self):
        return self

    async def __anext__(self):
        try:
            ref = await self._gen.__anext__()
        except StopAsyncIteration:
            self._finish()
            raise
        return await ref

    def cancel(self):
        self._finish()

    def __del__(self):
        try:
            self._finish()
        except Exception:  # noqa: BLE001
            pass


class DeploymentHandle:
    def __init__(self, deployment_name: str, app_name: str = "default", *, method_name=None,
                 multiplexed_model_id: str = "", stream: bool = False):
        self.deployment_name = deployment_name
        self.app_name = app_name
        self._method = method_name
        self._mux = multiplexed_model_id
        self._stream = stream

    def options(self, *, method_name=None, multiplexed_model_id=None, stream=None,
                use_new_handle_api=None, **kw):
        return DeploymentHandle(self.deployment_name, self.app_name,
                                method_name=method_name or self._method,
                                multiplexed_model_id=multiplexed_model_id if
                                multiplexed_model_id is not None else self._mux,
                                stream=self._stream if stream is None else stream)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return self.options(method_name=name)

    def remote(self, *args, **kwargs):
        r = _router(self.app_name, self.deployment_name)
        args = tuple(a._to_object_ref() if isinstance(a, DeploymentResponse) else a
                     for a in args)
        kwargs = {k: (v._to_object_ref() if isinstance(v, DeploymentResponse) else v)
                  for k, v in kwargs.items()}
        if self._stream:
            rid, h = r.choose(self._mux)
            gen = h.handle_request_streaming.remote(self._method or "__call__", args, kwargs,
                                                    self._mux)
            return DeploymentResponseGenerator(gen, r, rid)
        return self._send(r, args, kwargs, resend=lambda: self._send(r, args, kwargs))

    def _send(self, r, args, kwargs, resend=None):
        method, mux = self._method or "__call__", self._mux

        def send(h):
            return h.handle_request.remote(method, args, kwargs, mux)

        got = r.assign(send, mux)
        if isinstance(got, tuple):
            slot, ref = got
            return DeploymentResponse(ref, r, slot, resend=resend)
        return DeploymentResponse(None, r, resend=resend, pending=got)

    def __reduce__(self):
        return (DeploymentHandle, (self.deployment_name, self.app_name),
                {"_method": self._method, "_mux": self._mux, "_stream": self._stream})

    def __setstate__(self, st):
        self.__dict__.update(st)

    def __repr__(self):
        return f"DeploymentHandle(deployment='{self.deployment_name}', app='{self.app_name}')"


asyncio  # noqa: B018
