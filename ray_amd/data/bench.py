"""Ray Data → GPU ingest bench (BASELINE.json config 4, single-GPU slice).

Pipeline (``--data-path hbm``, the config-4 path): CPU read tasks synthesise uint8
224x224x3 images (stand-in for decode, seeded per block) → ``map_batches`` on a GPU
actor pool running the HIP ``image_normalize`` kernel (uint8 NHWC → bf16 NCHW) with
the output kept on the device → blocks travel through the HBM object store (hipIpc,
zero-copy on the same GPU) → ``iter_torch_batches(device="cuda")`` hands them to the
trainer with no H2D at all.

``--data-path h2d``: the consumer-side variant: uint8 blocks stay in host shared memory,
``iter_torch_batches`` moves them with the pinned ping-pong H2D (4x fewer bytes than
fp32) and the consumer runs ``image_normalize``.

Metric: normalised bf16 images per second delivered to the consumer."""

from __future__ import annotations

import json
import os
import time

import numpy as np

MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)


def _make_images(batch):
    ids = batch["id"]
    rng = np.random.default_rng(int(ids[0]))
    return {"image": rng.integers(0, 256, size=(len(ids), 224, 224, 3), dtype=np.uint8),
            "label": (ids % 1000).astype(np.int64)}


def bench_data(args):
    import torch

    import ray_amd as ray
    import ray_amd.data as rd
    from ray_amd.data.preprocessors import GPUImageNormalize
    from ray_amd.ops import functional as rf

    bs = 256
    path = getattr(args, "data_path", "hbm")
    total = (args.warmup + args.steps) * bs
    ray.init(num_cpus=min(16, os.cpu_count() or 1), num_gpus=1, ignore_reinit_error=True)
    ds = rd.range(total, override_num_blocks=max(8, total // bs)).map_batches(
        _make_images, batch_size=bs)
    if path == "hbm":
        ds = GPUImageNormalize(out_dtype="bf16", batch_size=bs, num_gpus=0.5,
                               keep_on_device=True).transform(ds)
    dev = torch.device("cuda", 0)
    it = iter(ds.iter_torch_batches(batch_size=bs, device=dev, drop_last=True))

    def step():
        b = next(it)
        x = b["image"]
        if path == "h2d":
            x = rf.image_normalize(x, MEAN, STD, torch.bfloat16)
        return x

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in range(args.steps):
        n += step().shape[0]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pipe = ("read(uint8 224x224x3) -> map_batches(GPU actor, HIP image_normalize, bf16 "
            "NCHW kept on device) -> HBM object store (hipIpc) -> iter_torch_batches(cuda)"
            if path == "hbm" else
            "read(uint8 224x224x3) -> iter_torch_batches(cuda, pinned ping-pong H2D) -> "
            "HIP image_normalize(bf16 NCHW)")
    print(json.dumps({
        "metric": "ray_data_gpu_ingest_images_per_sec", "value": round(n / dt, 1),
        "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1000, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"pipeline": pipe, "batch_size": bs, "data_path": path}}), flush=True)
    ray.shutdown()
