"""Streaming executor (reference: python/ray/data/_internal/execution/streaming_executor.py,
operators/{map_operator,actor_pool_map_operator,task_pool_map_operator}.py,
logical/rules/operator_fusion.py).

A plan is a source (read tasks or existing block refs) followed by stages. Runs of
task-based transforms are FUSED into the read task (one remote task per input
block: read → map → filter → map_batches ...). Actor-pool stages (stateful UDFs,
e.g. a model or a HIP preprocessing kernel on a GPU) run on a pool of long-lived
actors. Backpressure: each stage keeps at most ``max_in_flight`` tasks; outputs
are yielded in input order, so consumers (iter_batches, Train ingest) start as
soon as the first block is ready while upstream keeps producing.
"""

from __future__ import annotations

import collections
import itertools
import os

import ray_amd as ray

from . import block as B


def _meta(b):
    return {"num_rows": B.num_rows(b), "size_bytes": B.size_bytes(b), "schema": B.schema_of(b)}


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
                 max_tasks_in_flight_per_actor=2, name="Map"):
        self.kind = kind  # "task" | "actor"
        self.fns = list(fns or [])
        self.make_fn = make_fn
        self.resources = dict(resources or {})
        self.pool = pool
        self.max_tasks_in_flight_per_actor = max_tasks_in_flight_per_actor
        self.name = name

    def fusable_with(self, other):
        return self.kind == "task" and other.kind == "task" and \
            self.resources == other.resources


class Plan:
    def __init__(self, source, stages=None, source_meta=None):
        # source: ("read", [callables]) | ("refs", [block refs]) | ("lazy", fn -> refs)
        self.source = source
        self.stages = list(stages or [])
        self.source_meta = source_meta
        self._cache = None  # materialized (refs, metas)

    def with_stage(self, st: Stage) -> "Plan":
        stages = list(self.stages)
        if stages and stages[-1].fusable_with(st):
            last = stages[-1]
            stages[-1] = Stage("task", last.fns + st.fns, resources=last.resources,
                               name=f"{last.name}->{st.name}")
        else:
            stages.append(st)
        return Plan(self.source, stages, self.source_meta)


def _task_opts(res):
    o = {}
    if "num_cpus" in res:
        o["num_cpus"] = res["num_cpus"]
    if res.get("num_gpus"):
        o["num_gpus"] = res["num_gpus"]
    if res.get("resources"):
        o["resources"] = res["resources"]
    return o


def default_parallelism():
    try:
        return max(2, int(ray.cluster_resources().get("CPU", os.cpu_count() or 2)))
    except Exception:
        return os.cpu_count() or 2


def execute(plan: Plan, max_in_flight: int | None = None):
    """Yields (block_ref, meta) in order."""
    if plan._cache is not None:
        for r, m in zip(*plan._cache):
            yield r, m
        return
    cap = max_in_flight or max(4, 2 * default_parallelism())
    kind, src = plan.source
    if kind == "lazy":
        refs, metas = src()
        kind, src = "refs", refs
        src_meta = metas
    else:
        src_meta = plan.source_meta
    stages = list(plan.stages)
    # stage 0 fuses the read (or the first task stage) when it is a task stage
    first_fns = []
    first_res = {"num_cpus": 1}
    if stages and stages[0].kind == "task":
        first_fns = stages[0].fns
        first_res = stages[0].resources or first_res
        stages = stages[1:]
    if kind == "refs" and not first_fns:
        upstream = ((r, (src_meta[i] if src_meta else None), i) for i, r in enumerate(src))
    else:
        upstream = _run_first(kind, src, first_fns, first_res, cap)
    for st in stages:
        if st.kind == "task":
            upstream = _run_task_stage(upstream, st, cap)
        else:
            upstream = _run_actor_stage(upstream, st)
    for ref, meta, _ in upstream:
        if meta is not None and not isinstance(meta, dict):
            meta = ray.get(meta)
        yield ref, meta


def _run_first(kind, src, fns, res, cap):
    opts = _task_opts(res)
    items = iter(enumerate(src))
    inflight = collections.OrderedDict()
    done = {}
    next_out = 0
    exhausted = False
    while True:
        while not exhausted and len(inflight) + len(done) < cap:
            try:
                i, item = next(items)
            except StopIteration:
                exhausted = True
                break
            if kind == "read":
                b, m = _read_and_map.options(**opts).remote(item, fns)
            else:
                b, m = _map_block.options(**opts).remote(item, fns)
            inflight[m] = (i, b)
        if next_out in done:
            b, m = done.pop(next_out)
            yield b, m, next_out
            next_out += 1
            continue
        if not inflight:
            if exhausted and not done:
                return
            continue
        ready, _ = ray.wait(list(inflight), num_returns=1)
        for m in ready:
            i, b = inflight.pop(m)
            done[i] = (b, m)


def _run_task_stage(upstream, st, cap):
    opts = _task_opts(st.resources or {"num_cpus": 1})
    inflight = collections.OrderedDict()
    done = {}
    next_out = 0
    up = iter(upstream)
    exhausted = False
    while True:
        while not exhausted and len(inflight) + len(done) < cap:
            try:
                ref, _m, seq = next(up)
            except StopIteration:
                exhausted = True
                break
            b, m = _map_block.options(**opts).remote(ref, st.fns)
            inflight[m] = (seq, b)
        if next_out in done:
            b, m = done.pop(next_out)
            yield b, m, next_out
            next_out += 1
            continue
        if not inflight:
            if exhausted and not done:
                return
            continue
        ready, _ = ray.wait(list(inflight), num_returns=1)
        for m in ready:
            seq, b = inflight.pop(m)
            done[seq] = (b, m)


def _run_actor_stage(upstream, st):
    opts = _task_opts(st.resources or {"num_cpus": 1})
    lo, hi = st.pool
    cls = ray.remote(_MapWorker)
    actors = [cls.options(**opts).remote(st.make_fn) for _ in range(max(1, hi))]
    ray.get([a.ready.remote() for a in actors])
    load = {i: 0 for i in range(len(actors))}
    per = st.max_tasks_in_flight_per_actor
    inflight = {}
    done = {}
    next_out = 0
    up = iter(upstream)
    exhausted = False
    try:
        while True:
            while not exhausted:
                free = [i for i, n in load.items() if n < per]
                if not free:
                    break
                try:
                    ref, _m, seq = next(up)
                except StopIteration:
                    exhausted = True
                    break
                i = min(free, key=lambda j: load[j])
                b, m = actors[i].process.options(num_returns=2).remote(ref, [], st.fns)
                load[i] += 1
                inflight[m] = (seq, b, i)
            if next_out in done:
                b, m = done.pop(next_out)
                yield b, m, next_out
                next_out += 1
                continue
            if not inflight:
                if exhausted and not done:
                    return
                continue
            ready, _ = ray.wait(list(inflight), num_returns=1)
            for m in ready:
                seq, b, i = inflight.pop(m)
                load[i] -= 1
                done[seq] = (b, m)
    finally:
        for a in actors:
            try:
                ray.kill(a)
            except Exception:
                pass


def materialize(plan: Plan):
    if plan._cache is None:
        refs, metas = [], []
        for r, m in execute(plan):
            refs.append(r)
            metas.append(m)
        plan._cache = (refs, metas)
    return plan._cache


itertools  # noqa: B018
