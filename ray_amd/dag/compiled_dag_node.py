"""Compiled (accelerated) DAGs over mutable shared-memory channels.

Reference behaviour: python/ray/dag/compiled_dag_node.py (``CompiledDAG``,
``build_compiled_dag_from_ray_dag``, ``do_exec_tasks``), python/ray/experimental/
compiled_dag_ref.py (``CompiledDAGRef``/``CompiledDAGFuture``) and
python/ray/dag/dag_node.py:``experimental_compile``.

``dag.experimental_compile()`` turns a static graph of actor-method nodes into:
  * one channel (``ray_amd.experimental.channel.Channel``) per producer — the driver's
    input and every method node's output — with one reader slot per consumer;
  * one persistent execution loop per actor, started once through ``__ray_call__`` on a
    daemon thread of that actor: read the input channels, run the bound methods in the
    graph's topological order, write the output channels. No task submission, lease,
    object-table entry or RPC happens per execution;
  * ``execute()`` writes the input channel and returns ``CompiledDAGRef``s that read
    the output channels in order (results of earlier executions are buffered, so refs
    may be resolved in any order).
Errors raised by a method are written to its output channel and propagate through
downstream nodes to the driver (the DAG stays usable). ``teardown()`` closes the
channels, which ends every loop. Tensors of nodes marked with
``.with_tensor_transport()`` move through the node's HBM arena (D2D copy, zero-copy
reader view) rather than host memory. Channels are node-local shared memory: every
actor of a compiled DAG must run on the driver's node.
"""

from __future__ import annotations

import asyncio
import os
import threading
import time
import uuid
import weakref

from ray_amd.exceptions import (RayCgraphCapacityExceeded, RayChannelError,
                                RayChannelTimeoutError, RayTaskError)
from ray_amd.experimental.channel import Channel

_KIND_ERROR = 1
_SLICE = 0.05  # seconds between liveness checks while blocked


# ============================================================================ actor side
class _Slot:
    """Placeholder for a channel-fed argument: ``inputs[idx]`` passed through ``ext``."""

    __slots__ = ("idx", "ext")

    def __init__(self, idx, ext=None):
        self.idx = idx
        self.ext = ext


def _extract(v, ext):
    if ext is None:
        return v
    kind, key = ext
    if kind == "input":  # the InputNode itself: same rule as InputNode.execute
        a, k = v
        if len(a) == 1 and not k:
            return a[0]
        if not a and k:
            return k
        return a
    a, k = v
    if isinstance(key, int):
        return a[key]
    if key in k:
        return k[key]
    whole = _extract(v, ("input", None))
    return getattr(whole, key) if kind == "attr" else whole[key]


def _fill(t, vals):
    if isinstance(t, _Slot):
        return _extract(vals[t.idx], t.ext)
    if isinstance(t, list):
        return [_fill(x, vals) for x in t]
    if isinstance(t, tuple):
        return tuple(_fill(x, vals) for x in t)
    if isinstance(t, dict):
        return {k: _fill(x, vals) for k, x in t.items()}
    return t


class _ExecTask:
    """One bound method of an actor's loop."""

    def __init__(self, method, args, kwargs, inputs, out):
        self.method = method
        self.args = args
        self.kwargs = kwargs
        self.inputs = inputs  # [(Channel, reader_index)]
        self.out = out  # Channel


_loops: dict = {}


def _start_loop(inst, dag_id, tasks):
    for t in tasks:  # attach every endpoint now so a missing file fails the compile
        for ch, _ in t.inputs:
            ch._chan()
        t.out._chan()
    th = threading.Thread(target=_run_loop, args=(inst, tasks), daemon=True,
                          name=f"cdag-{dag_id[:8]}")
    _loops[dag_id] = th
    th.start()
    return os.uname().nodename


def _stop_loop(inst, dag_id, timeout=10.0):
    th = _loops.pop(dag_id, None)
    if th is not None:
        th.join(timeout)
        return not th.is_alive()
    return True


def _run_coro(coro):
    from ray_amd._private import worker as W

    loop = getattr(W.global_worker.core, "async_loop", None)
    if loop is not None:
        return asyncio.run_coroutine_threadsafe(coro, loop).result()
    return asyncio.run(coro)


def _run_loop(inst, tasks):
    import inspect

    try:
        while True:
            for t in tasks:
                vals, err = [], None
                for ch, r in t.inputs:
                    kind, v = ch.read_raw(r)
                    if kind == _KIND_ERROR and err is None:
                        err = v
                    vals.append(v)
                if err is not None:  # an upstream node failed: forward its error
                    t.out.write(err, _error=True)
                    continue
                try:
                    res = getattr(inst, t.method)(*_fill(t.args, vals), **_fill(t.kwargs, vals))
                    if inspect.isawaitable(res):
                        res = _run_coro(res)
                except Exception as e:  # noqa: BLE001
                    t.out.write(RayTaskError.from_exception(e, t.method, pid=os.getpid()),
                                _error=True)
                    continue
                t.out.write(res)
    except RayChannelError:
        pass  # a channel was closed: teardown
    finally:
        for t in tasks:
            t.out.close()


# ============================================================================ driver side
class CompiledDAGRef:
    """Result of one ``CompiledDAG.execute``; resolve with ``ray.get(ref)`` or
    ``ref.get()``. Each ref can be resolved once."""

    def __init__(self, dag, exec_index, out_index):
        self._dag = dag
        self._exec_index = exec_index
        self._out_index = out_index
        self._got = False

    def get(self, timeout=None):
        if self._got:
            raise ValueError("ray.get() can only be called once on a CompiledDAGRef")
        self._got = True
        return self._dag._get(self._exec_index, self._out_index, timeout)

    def __repr__(self):
        return f"CompiledDAGRef(execution={self._exec_index}, output={self._out_index})"

    def __del__(self):
        if not self._got:
            try:
                self._dag._discard(self._exec_index, self._out_index)
            except Exception:  # noqa: BLE001
                pass


class CompiledDAGFuture:
    """``await``-able result of ``execute_async``."""

    def __init__(self, ref: CompiledDAGRef):
        self._ref = ref

    def __await__(self):
        loop = asyncio.get_running_loop()
        return loop.run_in_executor(None, self._ref.get).__await__()


class CompiledDAG:
    def __init__(self, root, *, buffer_size_bytes: int | None = None,
                 max_inflight_executions: int | None = None, submit_timeout=None,
                 get_timeout=None, enable_asyncio: bool = False):
        self._root = root
        self._buffer = int(buffer_size_bytes or 1 << 20)
        self._max_inflight = int(max_inflight_executions or 10)
        self._submit_timeout = submit_timeout if submit_timeout is not None else 30.0
        self._get_timeout = get_timeout
        self._enable_asyncio = enable_asyncio
        self._dag_id = uuid.uuid4().hex
        self._torn_down = False
        self._lock = threading.RLock()
        self._next_exec = 0
        self._results: dict = {}  # (exec, out) -> (kind, value)
        self._discarded: set = set()
        self._got: set = set()
        self._build()
        self._finalizer = weakref.finalize(self, _teardown_channels, self._channels)

    # ---------------------------------------------------------------- compile
    def _build(self):
        from ray_amd.dag import (ClassMethodNode, ClassNode, DAGNode, FunctionNode,
                                 InputAttributeNode, InputNode, MultiOutputNode)

        root = self._root
        outs = list(root._bound_args[0]) if isinstance(root, MultiOutputNode) else [root]
        self._multi = isinstance(root, MultiOutputNode)
        order, seen = [], set()
        actors_cache: dict = {}

        def visit(n):
            if n._stable_uuid in seen:
                return
            seen.add(n._stable_uuid)
            if isinstance(n, FunctionNode):
                raise ValueError("Compiled DAGs support only actor method nodes; got a task "
                                 f"node ({n._fn}). Wrap the function in an actor method.")
            for c in n._children():
                if not isinstance(c, ClassNode):
                    visit(c)
            if isinstance(n, ClassMethodNode):
                order.append(n)
            elif not isinstance(n, (InputNode, InputAttributeNode, MultiOutputNode)):
                raise ValueError(f"unsupported node in a compiled DAG: {type(n).__name__}")

        for o in outs:
            if not isinstance(o, ClassMethodNode):
                raise ValueError("every output of a compiled DAG must be an actor method node")
            visit(o)

        def handle_of(n):
            a = n._actor
            if isinstance(a, ClassNode):
                if a._stable_uuid not in actors_cache:
                    actors_cache[a._stable_uuid] = a._exec({}, ((), {}))
                return actors_cache[a._stable_uuid]
            return a

        # readers per producer: producer key -> [consumer uuid]; "input" is the driver input
        consumers: dict = {"input": []}
        node_inputs: dict = {}
        templates: dict = {}
        for n in order:
            ins = []  # distinct producer keys, in first-use order

            def slot(v):
                if isinstance(v, (InputNode, InputAttributeNode)):
                    key = "input"
                    if isinstance(v, InputNode):
                        ext = ("input", None)
                    else:
                        ext = ("attr" if v._attr else "item", v._key)
                elif isinstance(v, ClassMethodNode):
                    key, ext = v._stable_uuid, None
                elif isinstance(v, DAGNode):
                    raise ValueError(f"unsupported argument node {type(v).__name__}")
                else:
                    if isinstance(v, list):
                        return [slot(x) for x in v]
                    if isinstance(v, tuple):
                        return tuple(slot(x) for x in v)
                    if isinstance(v, dict):
                        return {k: slot(x) for k, x in v.items()}
                    return v
                if key not in ins:
                    ins.append(key)
                return _Slot(ins.index(key), ext)

            args = [slot(a) for a in n._bound_args]
            kwargs = {k: slot(v) for k, v in n._bound_kwargs.items()}
            if not ins:  # a source node with constant arguments: triggered by the input
                ins.append("input")
            templates[n._stable_uuid] = (args, kwargs)
            node_inputs[n._stable_uuid] = ins
            for k in ins:
                consumers.setdefault(k, []).append(n._stable_uuid)
        out_keys = []
        for o in outs:
            if o._stable_uuid not in out_keys:
                out_keys.append(o._stable_uuid)
        self._out_pos = [out_keys.index(o._stable_uuid) for o in outs]

        # channels: one per producer; the driver is an extra reader of each output node
        chans = {}
        for key in ["input"] + [n._stable_uuid for n in order]:
            readers = list(consumers.get(key, []))
            if key in out_keys:
                readers.append("driver")
            if not readers:
                raise ValueError("a node's result is never consumed (make it an output)")
            gpu = False
            if key != "input":
                node = next(n for n in order if n._stable_uuid == key)
                gpu = getattr(node, "_tensor_transport", None) not in (None, "shm", "cpu")
            chans[key] = (Channel(len(readers), self._buffer, gpu=gpu), readers)
        self._channels = [c for c, _ in chans.values()]
        self._input = chans["input"][0]
        self._outputs = []
        for k in out_keys:
            ch, readers = chans[k]
            self._outputs.append((ch, readers.index("driver")))
        self._out_counts = [0] * len(self._outputs)

        # per-actor loops in global topological order
        per_actor: dict = {}
        handles: dict = {}
        for n in order:
            h = handle_of(n)
            handles[h._actor_id] = h
            inputs = []
            for k in node_inputs[n._stable_uuid]:
                ch, readers = chans[k]
                inputs.append((ch, readers.index(n._stable_uuid)))
            args, kwargs = templates[n._stable_uuid]
            per_actor.setdefault(h._actor_id, []).append(
                _ExecTask(n._method, args, kwargs, inputs, chans[n._stable_uuid][0]))
        self._handles = handles
        import ray_amd as ray

        here = os.uname().nodename
        try:
            nodes = ray.get([handles[a].__ray_call__.remote(_start_loop, self._dag_id, ts)
                             for a, ts in per_actor.items()])
        except Exception as e:
            _teardown_channels(self._channels)
            raise RayChannelError(
                "failed to start the compiled DAG's actor loops (channels are node-local "
                f"shared memory: every actor must run on the driver's node): {e}") from e
        if any(nd != here for nd in nodes):
            _teardown_channels(self._channels)
            raise RayChannelError("compiled DAG actors must run on the driver's node")

    # ---------------------------------------------------------------- execution
    def _check_alive(self):
        from ray_amd._private import protocol as P
        from ray_amd._private import worker as W

        cw = W.global_worker.core
        if cw is None:
            return
        for aid in self._handles:
            ac = cw.actors.get(aid)
            if ac is not None and ac.state == P.DEAD:
                self.teardown()
                from ray_amd.exceptions import ActorDiedError

                raise ActorDiedError(aid.hex(), "an actor of the compiled DAG died; the DAG "
                                     "was torn down")

    def _inflight(self):
        return self._next_exec * len(self._outputs) - len(self._got) - len(self._discarded)

    def execute(self, *args, **kwargs):
        with self._lock:
            if self._torn_down:
                raise RayChannelError("the compiled DAG was torn down")
            if self._inflight() >= self._max_inflight * len(self._outputs):
                raise RayCgraphCapacityExceeded(
                    f"more than {self._max_inflight} executions are in flight; ray.get() "
                    "earlier results first (or raise _max_inflight_executions)")
            from ray_amd._private import serialization as ser

            data = ser.serialize((args, kwargs)).to_bytes()
            deadline = time.monotonic() + self._submit_timeout
            while True:
                try:
                    self._input.write_bytes(data, timeout=_SLICE)
                    break
                except RayChannelTimeoutError:
                    # the pipeline is full: pull finished results into the buffer
                    self._drain()
                    self._check_alive()
                    if time.monotonic() > deadline:
                        raise RayChannelTimeoutError(
                            f"execute() could not submit within {self._submit_timeout}s")
            i = self._next_exec
            self._next_exec += 1
        refs = [CompiledDAGRef(self, i, p) for p in self._out_pos]
        return refs if self._multi else refs[0]

    def execute_async(self, *args, **kwargs):
        r = self.execute(*args, **kwargs)
        if isinstance(r, list):
            return [CompiledDAGFuture(x) for x in r]
        return CompiledDAGFuture(r)

    def _store(self, j, kv):
        key = (self._out_counts[j], j)
        self._out_counts[j] += 1
        if key in self._discarded:
            self._discarded.discard(key)
            self._got.add(key)
        else:
            self._results[key] = kv

    def _drain(self):
        for j, (ch, r) in enumerate(self._outputs):
            while self._out_counts[j] < self._next_exec:
                try:
                    kv = ch.read_raw(r, timeout=0)
                except RayChannelTimeoutError:
                    break
                self._store(j, kv)

    def _get(self, i, pos, timeout):
        j = pos
        timeout = timeout if timeout is not None else self._get_timeout
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._lock:
            while (i, j) not in self._results:
                if self._torn_down:
                    raise RayChannelError("the compiled DAG was torn down")
                ch, r = self._outputs[j]
                try:
                    kv = ch.read_raw(r, timeout=_SLICE)
                except RayChannelTimeoutError:
                    # the producer may be blocked writing ANOTHER output channel that
                    # holds an unread value: buffer every ready output so it can go on
                    # (refs may be resolved in any order)
                    self._drain()
                    self._check_alive()
                    if (i, j) in self._results:
                        break
                    if deadline is not None and time.monotonic() > deadline:
                        raise RayChannelTimeoutError(
                            f"result of execution {i} not ready after {timeout}s") from None
                    continue
                self._store(j, kv)
            kind, value = self._results.pop((i, j))
            self._got.add((i, j))
        if kind == _KIND_ERROR:
            if isinstance(value, RayTaskError):
                raise value.as_instanceof_cause()
            raise value
        return value

    def _discard(self, i, pos):
        with self._lock:
            if (i, pos) in self._results:
                self._results.pop((i, pos))
                self._got.add((i, pos))
            else:
                self._discarded.add((i, pos))

    # ---------------------------------------------------------------- teardown
    def teardown(self):
        with self._lock:
            if self._torn_down:
                return
            self._torn_down = True
        for ch in self._channels:
            ch.close()
        import ray_amd as ray

        try:
            ray.get([h.__ray_call__.remote(_stop_loop, self._dag_id)
                     for h in self._handles.values()], timeout=15)
        except Exception:  # noqa: BLE001  (dead actors: nothing to stop)
            pass
        self._finalizer()

    def __del__(self):
        try:
            if not self._torn_down:
                self.teardown()
        except Exception:  # noqa: BLE001
            pass

    def visualize(self) -> str:
        """Text rendering of the compiled schedule: actor -> ordered method list."""
        lines = []
        for aid, h in self._handles.items():
            lines.append(f"{h._class_name}({aid.hex()[:8]})")
        return "\n".join(lines)


def _teardown_channels(chans):
    for ch in chans:
        try:
            ch.destroy()
        except Exception:  # noqa: BLE001
            pass
