"""Where does the data-ingest bench spend its time? Times each stage in isolation:
H2D of a 256x224x224x3 uint8 block (pageable / pinned), the GPU-normalize UDF, the CPU
read stage alone through the streaming executor, and the full pipeline."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from ray_amd.data import bench as db  # noqa: E402


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


blk = db._make_images({"id": np.arange(256)})["image"]
print("block MB", blk.nbytes / 2**20, flush=True)
dev = torch.device("cuda", 0)
print("pageable H2D ms", t(lambda: torch.from_numpy(blk).to(dev, non_blocking=True)), flush=True)
pin = torch.empty(blk.shape, dtype=torch.uint8, pin_memory=True)
print("memcpy->pinned ms", t(lambda: pin.copy_(torch.from_numpy(blk))), flush=True)
print("pinned H2D ms", t(lambda: pin.to(dev, non_blocking=True)), flush=True)
print("make_images ms", t(lambda: db._make_images({"id": np.arange(256) + 7})), flush=True)
from ray_amd.data.preprocessors import _GPUNormalizeUDF  # noqa: E402

u = _GPUNormalizeUDF("image", db.MEAN, db.STD, "bf16", None, True)
b = {"image": blk, "label": np.zeros(256, np.int64)}
print("udf ms", t(lambda: u(b)), flush=True)

import ray_amd as ray  # noqa: E402
import ray_amd.data as rd  # noqa: E402

ray.init(num_cpus=16, num_gpus=1)
N = 80 * 256
for name, gpu in (("read-only", False), ("read+gpu", True)):
    ds = rd.range(N, override_num_blocks=80).map_batches(db._make_images, batch_size=256)
    if gpu:
        from ray_amd.data.preprocessors import GPUImageNormalize
        ds = GPUImageNormalize(out_dtype="bf16", batch_size=256, num_gpus=0.5,
                               keep_on_device=True).transform(ds)
    it = iter(ds.iter_batches(batch_size=256, batch_format="numpy"))
    for _ in range(5):
        next(it)
    t0 = time.perf_counter()
    n = 0
    for b in it:
        n += len(b["label"])
    dt = time.perf_counter() - t0
    print(name, "img/s", round(n / dt, 1), "ms/blk", round(dt / (n / 256) * 1e3, 2), flush=True)
ray.shutdown()
