"""`ray microbenchmark` equivalent (reference: python/ray/_private/ray_perf.py).

    python -m ray_amd._private.ray_perf [--quick] [--json out.json]
"""

from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing
import time

import numpy as np

import ray_amd as ray


def timeit(name, fn, multiplier=1, duration=2.0, warmup=0.3):
    t0 = time.time()
    while time.time() - t0 < warmup:
        fn()
    n = 0
    t0 = time.time()
    while time.time() - t0 < duration:
        fn()
        n += 1
    dt = time.time() - t0
    rate = n * multiplier / dt
    print(f"{name:48s} {rate:12.1f} /s", flush=True)
    return (name, rate)


@ray.remote
def create_object_containing_ref():
    return [ray.put(1) for _ in range(10000)]


@ray.remote(num_cpus=0)
class Actor:
    def small_value(self):
        return b"ok"

    def small_value_arg(self, x):
        return b"ok"

    def small_value_batch(self, n):
        ray.get([small_value.remote() for _ in range(n)])


@ray.remote
class AsyncActor:
    async def small_value(self):
        return b"ok"

    async def small_value_with_arg(self, x):
        return b"ok"


@ray.remote(num_cpus=0)
class Client:
    def __init__(self, servers):
        self.servers = servers if isinstance(servers, list) else [servers]

    def small_value_batch(self, n):
        res = []
        for s in self.servers:
            res.extend([s.small_value.remote() for _ in range(n)])
        ray.get(res)

    def small_value_batch_arg(self, n):
        x = ray.put(0)
        res = []
        for s in self.servers:
            res.extend([s.small_value_arg.remote(x) for _ in range(n)])
        ray.get(res)


@ray.remote(num_cpus=0)
class PutClient:
    def put_small(self, n):
        for _ in range(n):
            ray.put(0)

    def put_large(self, mb):
        arr = np.zeros(mb * 1024 * 1024 // 8, dtype=np.int64)
        for _ in range(10):
            ray.put(arr)

    def tasks(self, n):
        ray.get([small_value.remote() for _ in range(n)])


@ray.remote(num_cpus=0)
class DagStage:
    def f(self, x):
        return x


@ray.remote
def small_value():
    return b"ok"


def main(quick=False, num_cpus=None):
    results = []
    d = 1.0 if quick else 2.0
    ray.init(num_cpus=num_cpus)
    value = ray.put(0)
    results.append(timeit("single client get calls (Plasma Store)", lambda: ray.get(value),
                          duration=d))
    results.append(timeit("single client put calls (Plasma Store)", lambda: ray.put(0),
                          duration=d))
    arr = np.zeros(100 * 1024 * 1024, dtype=np.int64)
    results.append(timeit("single client put gigabytes", lambda: ray.put(arr), 8 * 0.1,
                          duration=d))

    def batch():
        ray.get([small_value.remote() for _ in range(1000)])

    results.append(timeit("single client tasks and get batch", batch, duration=d))
    n_clients = max(2, min(8, multiprocessing.cpu_count() // 2))
    clients = [PutClient.remote() for _ in range(n_clients)]
    ray.get([c.put_small.remote(1) for c in clients])
    results.append(timeit("multi client put calls (Plasma Store)",
                          lambda: ray.get([c.put_small.remote(1000) for c in clients]),
                          1000 * n_clients, duration=d))
    results.append(timeit("multi client put gigabytes",
                          lambda: ray.get([c.put_large.remote(80) for c in clients]),
                          n_clients * 10 * 80 / 1024, duration=d))

    # the object (a list of 10k refs, created once by a task) is built outside the timed
    # loop, as in the reference case: only the get (deserialising 10k refs) is timed
    obj_containing_ref = create_object_containing_ref.remote()
    ray.get(obj_containing_ref)

    def get_containing_object_ref():
        ray.get(obj_containing_ref)

    results.append(timeit("single client get object containing 10k refs",
                          get_containing_object_ref, duration=d))
    results.append(timeit("single client tasks sync", lambda: ray.get(small_value.remote()),
                          duration=d))
    results.append(timeit("single client tasks async", batch, 1000, duration=d))
    results.append(timeit("multi client tasks async",
                          lambda: ray.get([c.tasks.remote(1000) for c in clients]),
                          1000 * n_clients, duration=d))

    def wait_multiple_refs():
        not_ready = [small_value.remote() for _ in range(1000)]
        for _ in range(1000):
            _, not_ready = ray.wait(not_ready)

    results.append(timeit("single client wait 1k refs", wait_multiple_refs, duration=d))
    a = Actor.remote()
    results.append(timeit("1:1 actor calls sync", lambda: ray.get(a.small_value.remote()),
                          duration=d))
    a = Actor.remote()
    results.append(timeit("1:1 actor calls async",
                          lambda: ray.get([a.small_value.remote() for _ in range(1000)]), 1000,
                          duration=d))
    a = Actor.options(max_concurrency=16).remote()
    results.append(timeit("1:1 actor calls concurrent",
                          lambda: ray.get([a.small_value.remote() for _ in range(1000)]), 1000,
                          duration=d))
    n_cpu = max(1, multiprocessing.cpu_count() // 2)
    n = 2000
    actors = [Actor.remote() for _ in range(n_cpu)]
    client = Client.remote(actors)
    results.append(timeit("1:n actor calls async",
                          lambda: ray.get(client.small_value_batch.remote(n)), n * n_cpu,
                          duration=d))
    m = max(2, n_cpu // 2)
    servers = [Actor.remote() for _ in range(m)]
    nn_clients = [Client.remote(s) for s in servers]
    results.append(timeit("n:n actor calls async",
                          lambda: ray.get([c.small_value_batch.remote(1000)
                                           for c in nn_clients]), 1000 * m, duration=d))
    results.append(timeit("n:n actor calls with arg async",
                          lambda: ray.get([c.small_value_batch_arg.remote(1000)
                                           for c in nn_clients]), 1000 * m, duration=d))
    from ray_amd.dag import InputNode

    s1, s2 = DagStage.remote(), DagStage.remote()
    with InputNode() as inp:
        dag1 = s1.f.bind(inp)
    cd = dag1.experimental_compile()
    results.append(timeit("compiled DAG 1:1 actor calls sync",
                          lambda: ray.get(cd.execute(b"ok")), duration=d))
    cd.teardown()
    with InputNode() as inp:
        dag2 = s2.f.bind(s1.f.bind(inp))
    cd = dag2.experimental_compile()
    results.append(timeit("compiled DAG 2-actor chain sync",
                          lambda: ray.get(cd.execute(b"ok")), duration=d))
    cd.teardown()
    results.append(timeit("2-actor .remote() chain sync",
                          lambda: ray.get(s2.f.remote(s1.f.remote(b"ok"))), duration=d))
    aa = AsyncActor.remote()
    results.append(timeit("1:1 async-actor calls sync", lambda: ray.get(aa.small_value.remote()),
                          duration=d))
    results.append(timeit("1:1 async-actor calls async",
                          lambda: ray.get([aa.small_value.remote() for _ in range(1000)]), 1000,
                          duration=d))
    from ray_amd.util.placement_group import placement_group, remove_placement_group

    def pg_cycle():
        pgs = [placement_group([{"CPU": 0.001}]) for _ in range(20)]
        for pg in pgs:
            pg.wait(30)
        for pg in pgs:
            remove_placement_group(pg)

    results.append(timeit("placement group create/removal", pg_cycle, 20, duration=d))
    ray.shutdown()
    return results


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = main(a.quick)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({k: v for k, v in res}, f, indent=1)
    asyncio  # noqa: B018
