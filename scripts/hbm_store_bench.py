"""HBM object store put/get throughput on one MI355X (profiles/hbm_store_bench.json).

put  = ray.put(cuda tensor): D2D copy into the arena + async seal (producer not blocked)
get  = ray.get in the same process: zero-copy DLPack view (pin + wrap)
xget = ray.get in another actor process on the same GPU: IPC-mapped zero-copy view
"""

import json
import time

import torch

import ray_amd as ray
from ray_amd._private import gpu_object_store as gos


@ray.remote(num_gpus=0.5)
class Reader:
    def touch(self, refs):
        t0 = time.perf_counter()
        t = ray.get(refs[0])
        s = float(t.view(-1)[:1].float().sum())
        return time.perf_counter() - t0, s


def main():
    ray.init(num_cpus=4, num_gpus=1)
    out = {}
    rd = Reader.remote()
    ray.get(rd.touch.remote([ray.put(torch.ones(16, device="cuda"))]))
    for mb in (16, 256, 1024):
        n = mb << 20
        t = torch.empty(n, dtype=torch.uint8, device="cuda").fill_(1)
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        refs = [ray.put(t) for _ in range(reps)]
        t_put_host = (time.perf_counter() - t0) / reps
        gos.flush()
        t_put = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for r in refs:
            v = ray.get(r)
        t_get = (time.perf_counter() - t0) / reps
        del v
        xs = [ray.get(rd.touch.remote([r]))[0] for r in refs]
        out[f"{mb}MiB"] = {
            "put_return_ms": round(t_put_host * 1e3, 3),
            "put_sealed_GBps": round(n / t_put / 1e9, 1),
            "get_same_process_ms": round(t_get * 1e3, 3),
            "get_other_process_ms": round(min(xs) * 1e3, 3),
        }
        del refs
    out["stats"] = dict(gos.stats)
    print(json.dumps(out), flush=True)
    ray.shutdown()


if __name__ == "__main__":
    main()
