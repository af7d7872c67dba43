"""DeploymentHandle / DeploymentResponse and the replica router (reference:
python/ray/serve/handle.py, _private/router.py, _private/replica_scheduler/pow_2_scheduler.py).

Routing: power-of-two-choices on the number of requests this handle has in
flight to each replica (no extra RPC on the hot path); the replica set is
refreshed from the controller when its version changes or a replica fails."""

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
        self.lock = threading.Lock()
        self.last_refresh = 0.0
        self.affinity = {}  # multiplexed model id -> replica that loaded it

    def _controller(self):
        from ray_amd.serve.api import _get_controller

        return _get_controller()

    def refresh(self, force=False):
        now = time.time()
        if not force and self.replicas and now - self.last_refresh < 1.0:
            return
        info = ray.get(self._controller().get_replicas.remote(self.app, self.dep))
        self.last_refresh = now
        if info is None:
            raise RuntimeError(f"deployment {self.dep} of app {self.app} does not exist")
        version, reps, mo = info
        with self.lock:
            if version != self.version:
                self.version = version
                self.replicas = reps
                self.inflight = {rid: self.inflight.get(rid, 0) for rid, _ in reps}
            self.max_ongoing = mo

    async def arefresh(self, force=False):
        now = time.time()
        if not force and self.replicas and now - self.last_refresh < 1.0:
            return
        info = await self._controller().get_replicas.remote(self.app, self.dep)
        self.last_refresh = now
        if info is None:
            raise RuntimeError(f"deployment {self.dep} of app {self.app} does not exist")
        version, reps, mo = info
        with self.lock:
            if version != self.version:
                self.version = version
                self.replicas = reps
                self.inflight = {rid: self.inflight.get(rid, 0) for rid, _ in reps}
            self.max_ongoing = mo

    async def achoose(self, model_id=""):
        """choose() for event loops: the replica-set refresh is awaited, never blocks."""
        deadline = time.time() + 30
        await self.arefresh()
        while not self.replicas:
            if time.time() > deadline:
                raise RuntimeError(f"no replicas available for {self.dep}")
            await asyncio.sleep(0.05)
            await self.arefresh(force=True)
        return self._pick(model_id)

    def choose(self, model_id=""):
        deadline = time.time() + 30
        while True:
            self.refresh()
            with self.lock:
                reps = list(self.replicas)
            if reps:
                break
            if time.time() > deadline:
                raise RuntimeError(f"no replicas available for {self.dep}")
            time.sleep(0.05)
            self.refresh(force=True)
        return self._pick(model_id)

    def _pick(self, model_id=""):
        with self.lock:
            reps = list(self.replicas)
            # multiplexed requests stick to the replica that already loaded the model
            # while it is below max_ongoing_requests (reference: replica_scheduler
            # multiplexed-model matching before power-of-two choices)
            prev = self.affinity.get(model_id) if model_id else None
            hit = next((x for x in reps if x[0] == prev), None)
            if hit is not None and self.inflight.get(prev, 0) < self.max_ongoing:
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

    def done(self, rid):
        with self.lock:
            if rid in self.inflight:
                self.inflight[rid] = max(0, self.inflight[rid] - 1)


_routers: dict = {}
_rlock = threading.Lock()


def _router(app, dep):
    with _rlock:
        r = _routers.get((app, dep))
        if r is None:
            r = _routers[(app, dep)] = _Router(app, dep)
        return r


def invalidate(app):
    """Drop this process's cached replica sets of `app` (after a redeploy / delete)."""
    with _rlock:
        for key in [k for k in _routers if k[0] == app]:
            del _routers[key]


def _is_replica_death(e) -> bool:
    from ray_amd.exceptions import RayActorError

    return isinstance(e, RayActorError)


class DeploymentResponse:
    """``resend`` re-issues the request on a freshly chosen replica: used once when the
    replica died before answering (a redeploy / scale-down raced the cached routing
    table; reference: the router retries requests whose replica became unavailable)."""

    def __init__(self, ref, router, rid, resend=None):
        self._ref = ref
        self._router = router
        self._rid = rid
        self._done = False
        self._resend = resend

    def _finish(self):
        if not self._done:
            self._done = True
            self._router.done(self._rid)

    def _retry(self):
        self._finish()
        self._router.refresh(force=True)
        again, self._resend = self._resend(), None
        self._ref, self._rid, self._done = again._ref, again._rid, False

    def result(self, timeout_s: float | None = None):
        while True:
            try:
                return ray.get(self._ref, timeout=timeout_s)
            except Exception as e:  # noqa: BLE001
                if self._resend is None or not _is_replica_death(e):
                    raise
                self._retry()
            finally:
                self._finish()

    def __await__(self):
        async def _w():
            while True:
                try:
                    return await self._ref
                except Exception as e:  # noqa: BLE001
                    if self._resend is None or not _is_replica_death(e):
                        raise
                    self._finish()
                    await self._router.arefresh(force=True)
                    again, self._resend = self._resend(), None
                    self._ref, self._rid, self._done = again._ref, again._rid, False
                finally:
                    self._finish()

        return _w().__await__()

    def _to_object_ref(self):
        return self._ref

    async def _to_object_ref_async(self):
        return self._ref

    def cancel(self):
        ray.cancel(self._ref)

    def __reduce__(self):
        # passing a response to another deployment passes the underlying object
        return (_resolve, (self._ref,))


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
        rid, h = r.choose(self._mux)
        args = tuple(a._ref if isinstance(a, DeploymentResponse) else a for a in args)
        kwargs = {k: (v._ref if isinstance(v, DeploymentResponse) else v)
                  for k, v in kwargs.items()}
        if self._stream:
            gen = h.handle_request_streaming.remote(self._method or "__call__", args, kwargs,
                                                    self._mux)
            return DeploymentResponseGenerator(gen, r, rid)
        ref = h.handle_request.remote(self._method or "__call__", args, kwargs, self._mux)
        return DeploymentResponse(ref, r, rid, resend=lambda: self._send(r, args, kwargs))

    def _send(self, r, args, kwargs):
        rid, h = r.choose(self._mux)
        ref = h.handle_request.remote(self._method or "__call__", args, kwargs, self._mux)
        return DeploymentResponse(ref, r, rid)

    def __reduce__(self):
        return (DeploymentHandle, (self.deployment_name, self.app_name),
                {"_method": self._method, "_mux": self._mux, "_stream": self._stream})

    def __setstate__(self, st):
        self.__dict__.update(st)

    def __repr__(self):
        return f"DeploymentHandle(deployment='{self.deployment_name}', app='{self.app_name}')"


asyncio  # noqa: B018
