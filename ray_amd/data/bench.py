"""Ray Data → GPU ingest bench (BASELINE.json config 4, single-GPU slice).

CPU read tasks synthesise uint8 224x224x3 images (stand-in for decode, seeded per
block) → streaming executor → ``iter_torch_batches(device="cuda")`` (pinned-memory
ping-pong H2D of the uint8 bytes, 4x less PCIe traffic than fp32) → HIP
``image_normalize`` to bf16 NCHW on the consuming GPU. Metric: normalised images per
second available to the trainer."""

from __future__ import annotations

import json
import os
import time

import numpy as np


def _make_images(batch):
    ids = batch["id"]
    rng = np.random.default_rng(int(ids[0]))
    return {"image": rng.integers(0, 256, size=(len(ids), 224, 224, 3), dtype=np.uint8),
            "label": (ids % 1000).astype(np.int64)}


def bench_data(args):
    import torch

    import ray_amd as ray
    import ray_amd.data as rd
    from ray_amd.ops import functional as rf

    bs = 256
    total = (args.warmup + args.steps) * bs
    ray.init(num_cpus=min(16, os.cpu_count() or 1), ignore_reinit_error=True)
    ds = rd.range(total, override_num_blocks=max(8, total // bs)).map_batches(
        _make_images, batch_size=bs)
    dev = torch.device("cuda", 0)
    it = iter(ds.iter_torch_batches(batch_size=bs, device=dev, drop_last=True))
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    for _ in range(args.warmup):
        b = next(it)
        rf.image_normalize(b["image"], mean, std, torch.bfloat16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in range(args.steps):
        b = next(it)
        y = rf.image_normalize(b["image"], mean, std, torch.bfloat16)
        n += y.shape[0]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({
        "metric": "ray_data_gpu_ingest_images_per_sec", "value": round(n / dt, 1),
        "unit": "images/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1000, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"pipeline": "read(uint8 224x224x3) -> iter_torch_batches(cuda) -> "
                               "HIP image_normalize(bf16 NCHW)", "batch_size": bs}}), flush=True)
    ray.shutdown()
