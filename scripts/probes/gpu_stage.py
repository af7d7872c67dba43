"""Per-block cost of the data bench's GPU stage (actor: uint8 block from the shm store ->
HIP normalize -> bf16 block into the HBM store) and of device-block puts/gets."""
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import ray_amd as ray  # noqa: E402
from ray_amd.data import bench as db  # noqa: E402
from ray_amd.data.preprocessors import _GPUNormalizeUDF  # noqa: E402

ray.init(num_cpus=16, num_gpus=1)
print("store bytes", ray.cluster_resources().get("object_store_memory"), flush=True)
dev = torch.device("cuda", 0)
y = torch.randn(256, 3, 224, 224, device=dev).to(torch.bfloat16)


def tm(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e3, 3)


print("driver put(device dict) ms", tm(lambda: ray.put({"image": y, "label": np.zeros(256)})),
      flush=True)
r = ray.put({"image": y, "label": np.zeros(256)})
print("driver get(device dict) ms", tm(lambda: ray.get(r)), flush=True)


@ray.remote(num_gpus=0.5)
class Stage:
    def __init__(self):
        self.u = _GPUNormalizeUDF("image", db.MEAN, db.STD, "bf16", None, True)

    def process(self, blk):
        return self.u(blk)

    def profile(self, refs):
        pr = cProfile.Profile()
        pr.enable()
        t0 = time.perf_counter()
        for r in refs:
            out = self.u(ray.get(r))
            x = ray.put(out)
            del x
        dt = (time.perf_counter() - t0) / len(refs) * 1e3
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
        return dt, s.getvalue()


a = Stage.remote()
blocks = [ray.put(db._make_images({"id": np.arange(256) + 256 * i})) for i in range(24)]
ray.get(a.process.remote(blocks[0]))
t0 = time.perf_counter()
ray.get([a.process.remote(b) for b in blocks[:8]])
print("actor process, 8 calls pipelined, ms/call",
      round((time.perf_counter() - t0) / 8 * 1e3, 2), flush=True)
t0 = time.perf_counter()
for b in blocks[8:16]:
    ray.get(a.process.remote(b))
print("actor process, sequential, ms/call", round((time.perf_counter() - t0) / 8 * 1e3, 2),
      flush=True)
dt, prof = ray.get(a.profile.remote(blocks[16:]))
print("in-actor get+udf+put ms", round(dt, 2))
print(prof, flush=True)
ray.shutdown()
