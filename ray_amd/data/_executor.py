"""Streaming executor with resource budgets and backpressure.

Reference behaviour: python/ray/data/_internal/execution/streaming_executor.py
(scheduling loop on its own thread), streaming_executor_state.py
(``select_operator_to_run``), resource_manager.py (``ReservationOpResourceAllocator``:
a reserved share of the global limits per operator plus a shared pool),
backpressure_policy/ (concurrency cap, resource budget), operators/
{task_pool_map_operator,actor_pool_map_operator}.py (autoscaling actor pools) and
logical/rules/operator_fusion.py.

Structure:
  * a ``Plan`` (source + stages) becomes a chain of physical operators; runs of task
    stages are FUSED into one remote task per block (read -> map -> filter -> ...);
  * one scheduling thread per execution: harvest finished tasks (``ray.wait`` over every
    operator's in-flight metadata refs), hand outputs downstream, then launch work
    downstream-first, each launch gated by the backpressure policies;
  * the ``ResourceManager`` accounts per operator: CPU/GPU of running tasks and live
    actors, and object-store bytes of outputs that are produced but not yet consumed
    (queued for the next operator or for the consumer) plus the estimated output of
    in-flight tasks. Each operator gets ``reservation_ratio / n_ops`` of the limits
    reserved and competes for the rest; when the consumer is slow the last operator's
    queued bytes hit its budget and the pressure propagates upstream;
  * actor-pool operators autoscale between ``min_size`` and ``max_size``: a new actor
    starts when every live actor is saturated and inputs are waiting (and the budget
    allows its resources); idle actors above ``min_size`` are released once their
    input is exhausted.
Outputs are yielded in input order.
"""

from __future__ import annotations

import collections
import os
import threading
import weakref
import time

import ray_amd as ray

from . import block as B


def _meta(b):
    return {"num_rows": B.num_rows(b), "size_bytes": B.size_bytes(b), "schema": B.schema_of(b)}


def _nbytes(m):
    return int(m.get("size_bytes", 0)) if isinstance(m, dict) else 0


@ray.remote
def _split_block(blk, k):
    """Cut an oversized block into k row ranges (DataContext.target_max_block_size)."""
    n = B.num_rows(blk)
    bounds = [n * i // k for i in range(k + 1)]
    out = []
    for i in range(k):
        b = B.slice_block(blk, bounds[i], bounds[i + 1])
        out += [b]
    return tuple(out) if k > 1 else out[0]


def _target_block_size():
    from . import DataContext

    return int(getattr(DataContext.get_current(), "target_max_block_size", 0) or 0)


def _apply(fns, blk):
    for f in fns:
        blk = f(blk)
        if blk is None:
            blk = {}
    return blk


@ray.remote(num_returns=2)
def _read_and_map(read_fn, fns):
    blk = read_fn()
    if not isinstance(blk, dict):
        blk = B.from_batch(blk)
    blk = _apply(fns, blk)
    return blk, _meta(blk)


@ray.remote(num_returns=2)
def _map_block(blk, fns):
    blk = _apply(fns, blk)
    return blk, _meta(blk)


class _MapWorker:
    """Actor hosting a stateful (class-based) UDF for an actor-pool stage."""

    def __init__(self, make_fn):
        self.fn = make_fn()

    def process(self, blk, pre, post):
        blk = _apply(pre, blk)
        blk = self.fn(blk)
        blk = _apply(post, blk)
        return blk, _meta(blk)

    def ready(self):
        return True


class Stage:
    def __init__(self, kind, fns=None, make_fn=None, resources=None, pool=(1, 1),
                 max_tasks_in_flight_per_actor=2, name="Map", concurrency=None):
        self.kind = kind  # "task" | "actor"
        self.fns = list(fns or [])
        self.make_fn = make_fn
        self.resources = dict(resources or {})
        self.pool = pool
        self.max_tasks_in_flight_per_actor = max_tasks_in_flight_per_actor
        self.name = name
        self.concurrency = concurrency  # task stages: cap on concurrent tasks

    def fusable_with(self, other):
        return self.kind == "task" and other.kind == "task" and \
            self.resources == other.resources and self.concurrency == other.concurrency


class Plan:
    def __init__(self, source, stages=None, source_meta=None):
        # source: ("read", [callables]) | ("refs", [block refs]) | ("lazy", fn -> refs)
        #       | ("stream", fn -> iterator of (block ref, meta or meta ref)): pulled
        #         incrementally by a feeder thread (union / zip / shuffle outputs)
        self.source = source
        self.stages = list(stages or [])
        self.source_meta = source_meta
        self._cache = None  # materialized (refs, metas)
        self.last_stats = None

    def num_blocks_hint(self):
        """Upstream block count known without executing anything (read tasks, given refs,
        a materialized cache), or None. Stages may split blocks, so it is a hint."""
        if self._cache is not None:
            return len(self._cache[0])
        kind, val = self.source[0], self.source[1]
        if kind in ("read", "refs") and isinstance(val, (list, tuple)):
            return len(val)
        return None

    def with_stage(self, st: Stage) -> "Plan":
        stages = list(self.stages)
        if stages and stages[-1].fusable_with(st):
            last = stages[-1]
            stages[-1] = Stage("task", last.fns + st.fns, resources=last.resources,
                               name=f"{last.name}->{st.name}", concurrency=last.concurrency)
        else:
            stages.append(st)
        return Plan(self.source, stages, self.source_meta)


# ============================================================================ resources
class ExecutionResources:
    """cpu / gpu slots and object-store bytes (None = unlimited)."""

    __slots__ = ("cpu", "gpu", "object_store_memory")

    def __init__(self, cpu=None, gpu=None, object_store_memory=None):
        self.cpu = cpu
        self.gpu = gpu
        self.object_store_memory = object_store_memory

    def __repr__(self):
        return (f"ExecutionResources(cpu={self.cpu}, gpu={self.gpu}, "
                f"object_store_memory={self.object_store_memory})")


class ExecutionOptions:
    def __init__(self, resource_limits: ExecutionResources | None = None,
                 preserve_order: bool = True, reservation_ratio: float = 0.5,
                 max_tasks_in_flight: int | None = None, verbose_progress: bool = False):
        self.resource_limits = resource_limits or ExecutionResources()
        self.preserve_order = preserve_order
        self.reservation_ratio = reservation_ratio
        self.max_tasks_in_flight = max_tasks_in_flight
        self.verbose_progress = verbose_progress


# ray_remote_args of map-like operators passed through to the tasks / actors they launch
PASS_THROUGH_REMOTE_ARGS = ("memory", "max_retries", "retry_exceptions", "scheduling_strategy",
                            "runtime_env", "accelerator_type", "label_selector",
                            "max_restarts", "max_task_retries")


def _task_opts(res, actor=False):
    o = {}
    if "num_cpus" in res:
        o["num_cpus"] = res["num_cpus"]
    if res.get("num_gpus"):
        o["num_gpus"] = res["num_gpus"]
    if res.get("resources"):
        o["resources"] = res["resources"]
    for k in PASS_THROUGH_REMOTE_ARGS:
        if res.get(k) is None:
            continue
        if actor and k in ("max_retries", "retry_exceptions"):
            continue
        if not actor and k in ("max_restarts", "max_task_retries"):
            continue
        o[k] = res[k]
    return o


def default_parallelism():
    try:
        return max(2, int(ray.cluster_resources().get("CPU", os.cpu_count() or 2)))
    except Exception:
        return os.cpu_count() or 2


def _cluster_limits(opts: ExecutionOptions) -> ExecutionResources:
    lim = opts.resource_limits
    try:
        cr = ray.cluster_resources()
    except Exception:  # noqa: BLE001
        cr = {}
    cpu = lim.cpu if lim.cpu is not None else float(cr.get("CPU", os.cpu_count() or 2))
    gpu = lim.gpu if lim.gpu is not None else float(cr.get("GPU", 0.0))
    mem = lim.object_store_memory
    if mem is None:
        store = cr.get("object_store_memory")
        mem = int(0.5 * store) if store else 2 << 30
    return ExecutionResources(cpu, gpu, mem)


# ============================================================================ operators
class _Op:
    """Common runtime state of a physical operator."""

    def __init__(self, name, res, cap):
        self.name = name
        self.res = res
        self.cpu = float(res.get("num_cpus", 1) or 0)
        self.gpu = float(res.get("num_gpus", 0) or 0)
        self.cap = cap  # concurrency cap (backpressure policy 1)
        self.inq = collections.deque()  # (ref, meta, seq, nbytes) waiting to be processed
        self.inflight = {}  # meta ref -> (seq, block ref, extra)
        self.reorder = {}  # seq -> (block ref, meta dict)
        self.next_seq = 0
        self.outq = collections.deque()  # (ref, meta, seq) ready for downstream
        self.upstream_done = False
        self.out_bytes = 0  # bytes in reorder + outq
        self.inq_bytes = 0  # bytes of queued inputs (charged to the upstream operator)
        self.downstream = None
        self.out_count = 0
        self.out_total_bytes = 0
        self.stats = {"tasks": 0, "rows": 0, "bytes": 0, "wall_s": 0.0, "backpressured_s": 0.0}
        self._bp_since = None

    # --- usage ---------------------------------------------------------------
    def avg_out_bytes(self):
        return self.out_total_bytes / self.out_count if self.out_count else 0

    def mem_usage(self):
        """Produced-but-unconsumed bytes: own queued outputs, outputs waiting in the next
        operator's input queue, and the estimated output of running tasks."""
        ds = self.downstream.inq_bytes if self.downstream is not None else 0
        return self.out_bytes + ds + len(self.inflight) * self.avg_out_bytes()

    def push_input(self, item):
        self.inq.append(item)
        self.inq_bytes += item[3]

    def pop_input(self):
        item = self.inq.popleft()
        self.inq_bytes -= item[3]
        return item

    def cpu_usage(self):
        return self.cpu * len(self.inflight)

    def gpu_usage(self):
        return self.gpu * len(self.inflight)

    def pending_inputs(self):
        return len(self.inq)

    def done(self):
        return self.upstream_done and not self.inq and not self.inflight and \
            not self.reorder and not self.outq

    # --- completions -----------------------------------------------------------
    def on_complete(self, m):
        seq, b, extra = self.inflight.pop(m)
        meta = ray.get(m)
        nb = _nbytes(meta)
        self.out_count += 1
        self.out_total_bytes += nb
        self.out_bytes += nb
        self.stats["tasks"] += 1
        self.stats["rows"] += meta.get("num_rows", 0) if meta else 0
        self.stats["bytes"] += nb
        self.reorder[seq] = self._maybe_split(b, meta)
        while self.next_seq in self.reorder:
            for b2, m2 in self.reorder.pop(self.next_seq):
                self.outq.append((b2, m2, self.next_seq))
            self.next_seq += 1
        return extra

    def _maybe_split(self, b, meta):
        """Dynamic block splitting (reference: map_operator.py:53 with
        DataContext.target_max_block_size): an output block larger than the target is cut
        into ceil(size / target) row ranges by one task; their metas follow from the row
        counts, so the scheduling thread never waits for the split."""
        target = _target_block_size()
        nb = _nbytes(meta)
        rows = meta.get("num_rows", 0) if isinstance(meta, dict) else 0
        if not target or nb <= target or rows < 2:
            return [(b, meta)]
        k = int(min(rows, -(-nb // target)))
        refs = _split_block.options(num_returns=k).remote(b, k)
        refs = refs if isinstance(refs, list) else [refs]
        bounds = [rows * i // k for i in range(k + 1)]
        out = []
        for i, r in enumerate(refs):
            n = bounds[i + 1] - bounds[i]
            out.append((r, {"num_rows": n, "size_bytes": int(nb * n / rows),
                            "schema": meta.get("schema")}))
        self.stats["splits"] = self.stats.get("splits", 0) + 1
        return out

    def take_output(self):
        b, m, seq = self.outq.popleft()
        self.out_bytes -= _nbytes(m)
        return b, m, seq

    def can_launch_more(self):
        return bool(self.inq) and len(self.inflight) < self.cap

    def launch(self):
        raise NotImplementedError

    def shutdown(self):
        pass


class _TaskOp(_Op):
    """Fused read/map tasks (a task pool)."""

    def __init__(self, name, fns, res, cap, read=False):
        super().__init__(name, res, cap)
        self.fns = fns
        self.read = read
        self.opts = _task_opts(res)

    def launch(self):
        item, _meta_in, seq, _nb = self.pop_input()
        if self.read:
            b, m = _read_and_map.options(**self.opts).remote(item, self.fns)
        else:
            b, m = _map_block.options(**self.opts).remote(item, self.fns)
        self.inflight[m] = (seq, b, None)
        return m


class _PassOp(_Op):
    """Input of a streamed source with no task stage: blocks pass straight through (no
    task), so union / zip / shuffle outputs stream to the consumer as they arrive."""

    def __init__(self, name):
        super().__init__(name, {"num_cpus": 0}, 1 << 30)

    def launch(self):
        item, meta, seq, nb = self.pop_input()
        self.out_count += 1
        self.out_total_bytes += nb
        self.out_bytes += nb
        self.outq.append((item, meta, seq))
        return None


class _ActorPoolOp(_Op):
    """Stateful UDF on an autoscaling actor pool."""

    def __init__(self, st: Stage):
        lo, hi = st.pool
        self.min_size = max(1, int(lo or 1))
        self.max_size = max(self.min_size, int(hi or self.min_size))
        self.per = max(1, int(st.max_tasks_in_flight_per_actor))
        super().__init__(st.name, st.resources or {"num_cpus": 1}, self.max_size * self.per)
        self.fns = st.fns
        self.make_fn = st.make_fn
        self.cls = ray.remote(_MapWorker)
        self.opts = _task_opts(self.res, actor=True)
        self.actors = {}  # idx -> handle (ready)
        self.starting = {}  # ready ref -> (idx, handle)
        self.load = {}
        self._next_idx = 0
        self.stats.update({"actors_started": 0, "actors_released": 0, "max_actors": 0})
        for _ in range(self.min_size):
            self._start_actor()

    def _start_actor(self):
        h = self.cls.options(**self.opts).remote(self.make_fn)
        i = self._next_idx
        self._next_idx += 1
        self.starting[h.ready.remote()] = (i, h)
        self.stats["actors_started"] += 1

    def n_actors(self):
        return len(self.actors) + len(self.starting)

    # actors hold their resources whether busy or not
    def cpu_usage(self):
        return self.cpu * self.n_actors()

    def gpu_usage(self):
        return self.gpu * self.n_actors()

    def on_actor_ready(self, r):
        i, h = self.starting.pop(r)
        ray.get(r)
        self.actors[i] = h
        self.load[i] = 0
        self.stats["max_actors"] = max(self.stats["max_actors"], len(self.actors))

    def can_launch_more(self):
        return bool(self.inq) and any(n < self.per for n in self.load.values())

    def launch(self):
        i = min((j for j, n in self.load.items() if n < self.per), key=lambda j: self.load[j])
        ref, _m, seq, _nb = self.pop_input()
        b, m = self.actors[i].process.options(num_returns=2).remote(ref, [], self.fns)
        self.load[i] += 1
        self.inflight[m] = (seq, b, i)
        return m

    def on_complete(self, m):
        i = super().on_complete(m)
        if i in self.load:
            self.load[i] -= 1
        return i

    def want_scale_up(self):
        return (self.inq and not self.starting and self.n_actors() < self.max_size and
                all(n >= self.per for n in self.load.values()))

    def scale_down_idle(self):
        if not (self.upstream_done and not self.inq):
            return
        keep = 0 if not self.inflight else self.min_size
        for i in [j for j, n in self.load.items() if n == 0]:
            if len(self.actors) <= keep:
                break
            h = self.actors.pop(i)
            self.load.pop(i)
            self.stats["actors_released"] += 1
            try:
                ray.kill(h)
            except Exception:  # noqa: BLE001
                pass

    def shutdown(self):
        for h in list(self.actors.values()) + [h for _, h in self.starting.values()]:
            try:
                ray.kill(h)
            except Exception:  # noqa: BLE001
                pass
        self.actors.clear()
        self.starting.clear()
        self.load.clear()


class ResourceManager:
    """Global limits, per-operator reservations and the shared remainder (reference:
    resource_manager.py ReservationOpResourceAllocator)."""

    def __init__(self, ops, limits: ExecutionResources, reservation_ratio: float):
        self.ops = ops
        self.limits = limits
        n = max(1, len(ops))
        self.reserved_mem = limits.object_store_memory * reservation_ratio / n
        self.shared_mem = limits.object_store_memory * (1 - reservation_ratio)

    def total_cpu(self):
        return sum(o.cpu_usage() for o in self.ops)

    def total_gpu(self):
        return sum(o.gpu_usage() for o in self.ops)

    def mem_budget_left(self, op):
        """Bytes `op` may still add: its reservation plus what is left of the shared pool
        after every operator's overflow beyond its own reservation."""
        over = sum(max(0.0, o.mem_usage() - self.reserved_mem) for o in self.ops)
        shared_left = max(0.0, self.shared_mem - over)
        mine = max(0.0, self.reserved_mem - op.mem_usage())
        return mine + shared_left

    def can_launch(self, op, actor=False):
        # backpressure policy 2: CPU/GPU slots (a task of an actor op uses the actor's)
        if not actor:
            if op.cpu and self.total_cpu() + op.cpu > self.limits.cpu + 1e-9:
                return False
            if op.gpu and self.total_gpu() + op.gpu > self.limits.gpu + 1e-9:
                return False
        # backpressure policy 3: object store budget (estimated output of one more task)
        est = op.avg_out_bytes()
        return est <= self.mem_budget_left(op) or not op.inflight

    def can_add_actor(self, op):
        if op.cpu and self.total_cpu() + op.cpu > self.limits.cpu + 1e-9:
            return False
        if op.gpu and self.total_gpu() + op.gpu > self.limits.gpu + 1e-9:
            return False
        return True


# ============================================================================ execution
_ACTIVE: "weakref.WeakSet[StreamingExecutor]" = weakref.WeakSet()


def stop_all(timeout: float = 5.0) -> None:
    """Stop every running executor of this process and wait for their scheduling threads
    (``ray_amd.shutdown`` calls this first: an abandoned iterator's executor must not keep
    calling into a cluster that is going away, or auto-initialise a new one)."""
    execs = list(_ACTIVE)
    for ex in execs:
        ex._stop = True
        with ex._cv:
            ex._cv.notify_all()
    for ex in execs:
        t = ex._thread
        if t is not None and t is not threading.current_thread():
            t.join(timeout=timeout)


class StreamingExecutor:
    """Runs one plan on a scheduling thread; iterate to receive (block_ref, meta)."""

    def __init__(self, plan: Plan, options: ExecutionOptions | None = None):
        _ACTIVE.add(self)
        self.plan = plan
        self.options = options or _default_options()
        self._cv = threading.Condition()
        self._out = collections.deque()
        self._out_bytes = 0  # bytes of blocks handed to the consumer but not yet read
        self._finished = False
        self._error = None
        self._stop = False
        self._thread = None
        self.ops = []
        self.stats = {}

    # --- plan -> operators --------------------------------------------------------
    def _build(self):
        plan = self.plan
        cap_default = self.options.max_tasks_in_flight or max(4, 2 * default_parallelism())
        kind, src = plan.source
        self._stream = None
        if kind == "lazy":
            refs, metas = src()
            kind, src, src_meta = "refs", refs, metas
        elif kind == "stream":
            self._stream = src
            src, src_meta = [], None
        else:
            src_meta = plan.source_meta
        stages = list(plan.stages)
        first_fns, first_res, first_cap = [], {"num_cpus": 1}, cap_default
        if stages and stages[0].kind == "task":
            first_fns = stages[0].fns
            first_res = stages[0].resources or first_res
            first_cap = stages[0].concurrency or cap_default
            first_name = stages[0].name
            stages = stages[1:]
        else:
            first_name = "Read" if kind == "read" else "Input"
        ops = []
        if kind == "stream":
            ops.append(_TaskOp(first_name, first_fns, first_res, first_cap) if first_fns
                       else _PassOp("Input"))
            self._source = []
        elif kind == "refs" and not first_fns:
            self._source = [(r, (src_meta[i] if src_meta else None), i)
                            for i, r in enumerate(src)]
        else:
            name = ("Read->" + first_name) if kind == "read" and first_fns else first_name
            ops.append(_TaskOp(name, first_fns, first_res, first_cap, read=(kind == "read")))
            self._source = [(item, None, i) for i, item in enumerate(src)]
        for st in stages:
            if st.kind == "task":
                ops.append(_TaskOp(st.name, st.fns, st.resources or {"num_cpus": 1},
                                   st.concurrency or cap_default))
            else:
                ops.append(_ActorPoolOp(st))
        for a, b in zip(ops, ops[1:]):
            a.downstream = b
        self.ops = ops
        self.rm = ResourceManager(ops, _cluster_limits(self.options),
                                  self.options.reservation_ratio)
        if ops and self._stream is None:
            for item, meta, seq in self._source:
                ops[0].inq.append((item, meta, seq, 0))
            ops[0].upstream_done = True

    # --- thread ---------------------------------------------------------------------
    def start(self):
        self._build()
        if not self.ops:  # plain refs, nothing to run
            for r, m, _ in self._source:
                self._out.append((r, m))
            self._finished = True
            return self
        self._t0 = time.perf_counter()
        if self._stream is not None:
            self._feed = collections.deque()
            self._feed_done = False
            self._feed_error = None
            self._feeder = threading.Thread(target=self._feed_run, daemon=True,
                                            name="data-feed")
            self._feeder.start()
        self._thread = threading.Thread(target=self._run, daemon=True, name="data-exec")
        self._thread.start()
        return self

    def _feed_run(self):
        """Pull the streamed source; stay at most a few blocks ahead of the first op."""
        seq = 0
        try:
            for item, meta in self._stream():
                with self._cv:
                    while not self._stop and len(self._feed) + len(self.ops[0].inq) > \
                            max(8, 2 * min(self.ops[0].cap, 64)):
                        self._cv.wait(0.05)
                    if self._stop:
                        return
                    self._feed.append((item, meta, seq, _nbytes(meta)))
                    seq += 1
        except BaseException as e:  # noqa: BLE001
            self._feed_error = e
        finally:
            with self._cv:
                self._feed_done = True
                self._cv.notify_all()

    def _drain_feed(self):
        if self._stream is None:
            return False
        moved = False
        with self._cv:
            while self._feed:
                self.ops[0].push_input(self._feed.popleft())
                moved = True
            if self._feed_done and not self._feed and not self.ops[0].upstream_done:
                if self._feed_error is not None:
                    raise self._feed_error
                self.ops[0].upstream_done = True
                moved = True
            if moved:
                self._cv.notify_all()
        return moved

    def _run(self):
        try:
            self._loop()
        except BaseException as e:  # noqa: BLE001
            self._error = e
        finally:
            for op in self.ops:
                op.shutdown()
            self._collect_stats()
            with self._cv:
                self._finished = True
                self._cv.notify_all()

    def _loop(self):
        ops = self.ops
        last = ops[-1]
        while not self._stop:
            progressed = self._drain_feed()
            # 1. hand outputs downstream / to the consumer
            for k, op in enumerate(ops):
                while op.outq:
                    b, m, seq = op.take_output()
                    if k + 1 < len(ops):
                        ops[k + 1].push_input((b, m, seq, _nbytes(m)))
                    else:
                        with self._cv:
                            self._out.append((b, m))
                            self._out_bytes += _nbytes(m)
                            self._cv.notify_all()
                    progressed = True
                if k + 1 < len(ops) and op.done():
                    ops[k + 1].upstream_done = True
            # 2. launch, downstream first (drains memory before producing more)
            for op in reversed(ops):
                if isinstance(op, _ActorPoolOp):
                    if op.want_scale_up() and self.rm.can_add_actor(op):
                        op._start_actor()
                    op.scale_down_idle()
                launched = 0
                while op.can_launch_more() and self.rm.can_launch(
                        op, actor=isinstance(op, _ActorPoolOp)) and \
                        self._consumer_ok(op, last):
                    op.launch()
                    launched += 1
                if launched:
                    progressed = True
                    op._bp_since = None
                elif op.inq and op._bp_since is None:
                    op._bp_since = time.perf_counter()
            if all(op.done() for op in ops):
                return
            # 3. wait for a completion (task or actor start)
            waits = {}
            for op in ops:
                for m in op.inflight:
                    waits[m] = op
                if isinstance(op, _ActorPoolOp):
                    for r in op.starting:
                        waits[r] = op
            if not waits:
                if not progressed:
                    with self._cv:  # blocked on the consumer / the feeder: wait for it
                        self._cv.wait(0.05)
                continue
            ready, _ = ray.wait(list(waits), num_returns=1, timeout=0.05 if not progressed
                                else 0)
            ready2, _ = ray.wait(list(waits), num_returns=len(waits), timeout=0) \
                if ready else ([], None)
            for r in set(ready) | set(ready2):
                op = waits[r]
                if isinstance(op, _ActorPoolOp) and r in op.starting:
                    op.on_actor_ready(r)
                else:
                    op.on_complete(r)
            for op in ops:
                if op._bp_since is not None and not op.inq:
                    op.stats["backpressured_s"] += time.perf_counter() - op._bp_since
                    op._bp_since = None

    def _consumer_ok(self, op, last):
        """The consumer not keeping up: stop the last operator once its unread output
        exceeds its memory reservation (and the shared pool)."""
        if op is not last or not last.inflight and not self._out:
            return True
        pending = self._out_bytes + last.mem_usage()
        return pending <= self.rm.reserved_mem + self.rm.shared_mem

    def _collect_stats(self):
        wall = time.perf_counter() - getattr(self, "_t0", time.perf_counter())
        self.stats = {op.name: dict(op.stats) for op in self.ops}
        self.stats["_wall_s"] = wall
        self.plan.last_stats = self.stats

    # --- consumer side --------------------------------------------------------------
    def __iter__(self):
        try:
            while True:
                with self._cv:
                    while not self._out and not self._finished:
                        self._cv.wait(1.0)
                    if self._out:
                        item = self._out.popleft()
                        m = item[1]
                        self._out_bytes -= _nbytes(m)
                        self._cv.notify_all()
                    elif self._error is not None:
                        raise self._error
                    else:
                        return
                yield item
        finally:
            self.shutdown()

    def shutdown(self):
        self._stop = True
        with self._cv:
            self._cv.notify_all()
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join(timeout=30)


def _default_options():
    from . import DataContext

    o = DataContext.get_current().execution_options
    return o if isinstance(o, ExecutionOptions) else ExecutionOptions()


def execute(plan: Plan, max_in_flight: int | None = None,
            options: ExecutionOptions | None = None):
    """Yields (block_ref, meta) in order."""
    if plan._cache is not None:
        for r, m in zip(*plan._cache):
            yield r, m
        return
    opts = options or _default_options()
    if max_in_flight is not None:
        opts = ExecutionOptions(opts.resource_limits, opts.preserve_order,
                                opts.reservation_ratio, max_in_flight, opts.verbose_progress)
    ex = StreamingExecutor(plan, opts).start()
    for ref, meta in ex:
        if meta is not None and not isinstance(meta, dict):
            meta = ray.get(meta)
        yield ref, meta


def execute_started(plan: Plan, options: ExecutionOptions | None = None):
    """Like execute(), but the plan starts running NOW (before the first next()): a
    consumer of several inputs (union) starts them all at once without blocking."""
    if plan._cache is not None:
        return iter(list(zip(*plan._cache)))
    ex = StreamingExecutor(plan, options or _default_options()).start()

    def gen():
        for ref, meta in ex:
            if meta is not None and not isinstance(meta, dict):
                meta = ray.get(meta)
            yield ref, meta

    return gen()


def materialize(plan: Plan):
    if plan._cache is None:
        refs, metas = [], []
        for r, m in execute(plan):
            refs.append(r)
            metas.append(m)
        plan._cache = (refs, metas)
    return plan._cache


def format_stats(stats: dict | None) -> str:
    if not stats:
        return ""
    lines = []
    for name, s in stats.items():
        if name.startswith("_"):
            continue
        extra = ""
        if "max_actors" in s:
            extra = (f", actors started {s['actors_started']} (peak {s['max_actors']}), "
                     f"released {s['actors_released']}")
        lines.append(f"Operator {name}: {s['tasks']} tasks, {s['rows']} rows, "
                     f"{s['bytes']} bytes, backpressured {s['backpressured_s']:.3f}s{extra}")
    lines.append(f"Total wall time: {stats.get('_wall_s', 0):.3f}s")
    return "\n".join(lines)
