"""Ray Data → GPU ingest bench (BASELINE.json config 4; ``--gpus N``: N TorchTrainer
workers, see ``bench_data_trainer``).

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


_POOL = None


def _gpu_actors() -> int:
    """Preprocessing actors per GPU (RAY_AMD_DATA_GPU_ACTORS, default 2). One actor per
    block runs ray.get of the 38.5 MB uint8 block, the H2D copy, the normalise kernel and
    the HBM-store put serially; in the TorchTrainer timeline (profiles/r4) one actor's
    `process` was busy 95 % of the timed window. Two actors overlap those phases:
    112.7k vs 60.4k images/s through TorchTrainer, 100.9k vs 59.7k direct (r4f)."""
    return max(1, int(os.environ.get("RAY_AMD_DATA_GPU_ACTORS", "2")))


def _make_images(batch):
    """Synthetic uint8 images: a per-process pool of random images (generated once), each
    block a rotation of it by its first id — a memcpy-speed stand-in for decode, so the
    bench measures the ingest pipeline (object store, GPU preprocessing, H2D / HBM hand-off)
    rather than numpy's random-number generator (which capped a 16-CPU box near 85k
    images/s)."""
    global _POOL
    ids = batch["id"]
    if _POOL is None:
        _POOL = np.random.default_rng(0).integers(0, 256, size=(512, 224, 224, 3),
                                                  dtype=np.uint8)
    start = int(ids[0]) % len(_POOL)
    idx = (start + np.arange(len(ids))) % len(_POOL)
    return {"image": _POOL[idx], "label": (ids % 1000).astype(np.int64)}


def _ingest_loop(config):
    """TorchTrainer worker: consume this worker's dataset shard as device batches; every
    rank times its own loop, rank 0 reports the job total (sum of images, max time)."""
    import torch
    import torch.distributed as dist

    from ray_amd import train
    from ray_amd.ops import functional as rf
    from ray_amd.train.torch import get_device

    dev = get_device()
    bs, warmup, steps, path = (config[k] for k in ("bs", "warmup", "steps", "path"))
    shard = train.get_dataset_shard("train")
    it = iter(shard.iter_torch_batches(batch_size=bs, device=dev, drop_last=True))

    def step():
        x = next(it)["image"]
        if path == "h2d":
            x = rf.image_normalize(x, MEAN, STD, torch.bfloat16)
        return x.shape[0]

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    dist.barrier()
    prof = None
    if os.environ.get("RAY_AMD_DATA_PROFILE") == "1":  # cProfile of the timed loop
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    w0 = time.time()
    t0 = time.perf_counter()
    n = sum(step() for _ in range(steps))
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    w1 = time.time()
    if prof is not None:
        import io
        import pstats
        import sys

        prof.disable()
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(30)
        print(buf.getvalue(), file=sys.stderr, flush=True)
    t = torch.tensor([float(n), dt], device=dev, dtype=torch.float64)
    allt = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(allt, t)
    train.report({"images": sum(float(x[0]) for x in allt),
                  "seconds": max(float(x[1]) for x in allt),
                  "window": [w0, w1],  # wall-clock bounds of rank 0's timed loop
                  "rccl_world_size": dist.get_world_size()})


def bench_data_trainer(args, n_gpus: int):
    """Config 4 at N GPUs: N TorchTrainer workers (RCCL group) each ingesting its
    streaming_split shard of the GPU-preprocessed dataset. Preprocessing actors and
    trainers share the GPUs (0.5 each), so device blocks move GPU-to-GPU through the HBM
    store (same-GPU zero-copy or xGMI peer copies)."""
    import ray_amd as ray
    import ray_amd.data as rd
    from ray_amd.data.preprocessors import GPUImageNormalize
    from ray_amd.train import RunConfig, ScalingConfig
    from ray_amd.train.torch import TorchTrainer

    bs = 256
    path = getattr(args, "data_path", "hbm")
    total = (args.warmup + args.steps) * bs * n_gpus + n_gpus * bs  # + one spare per rank
    ray.init(num_cpus=max(16, 4 * n_gpus), num_gpus=n_gpus, ignore_reinit_error=True)
    try:
        ds = rd.range(total, override_num_blocks=max(8, total // bs)).map_batches(
            _make_images, batch_size=bs)
        if path == "hbm":
            na = _gpu_actors() * n_gpus
            ds = GPUImageNormalize(out_dtype="bf16", batch_size=bs, num_gpus=0.5 / _gpu_actors(),
                                   concurrency=na, keep_on_device=True).transform(ds)
        trainer = TorchTrainer(
            _ingest_loop, train_loop_config={"bs": bs, "warmup": args.warmup,
                                             "steps": args.steps, "path": path},
            scaling_config=ScalingConfig(num_workers=n_gpus, use_gpu=True,
                                         resources_per_worker={"GPU": 0.5}),
            datasets={"train": ds},
            run_config=RunConfig(name="bench_data", storage_path="/tmp/ray_amd_bench"))
        m = trainer.fit().metrics
        tl = os.environ.get("RAY_AMD_DATA_TIMELINE")
        if tl:  # task timeline of the whole run + the timed window (scripts/data_timeline.py)
            trace = ray.timeline()
            with open(tl, "w") as f:
                json.dump({"window": m.get("window"), "cpus": max(16, 4 * n_gpus),
                           "trace": trace}, f)
    finally:
        ray.shutdown()
    dt = m["seconds"]
    print(json.dumps({
        "metric": "ray_data_gpu_ingest_images_per_sec", "value": round(m["images"] / dt, 1),
        "unit": "images/s", "n_gpus": n_gpus, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1000, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic uint8 images (pre-generated pool, per-block rotation)",
        "config": {"pipeline": "read -> map_batches(GPU actors, HIP image_normalize, bf16 on "
                               "device) -> HBM object store -> streaming_split -> TorchTrainer "
                               "workers iter_torch_batches(cuda)" if path == "hbm" else
                               "read -> streaming_split -> TorchTrainer workers "
                               "iter_torch_batches(cuda, pinned H2D) -> HIP image_normalize",
                   "batch_size_per_worker": bs, "data_path": path,
                   "parallelism": f"dp{n_gpus}"},
        "rccl_world_size": m.get("rccl_world_size")}), flush=True)


def bench_data(args):
    import torch

    n_gpus = max(1, int(getattr(args, "gpus", 1) or 1))
    if n_gpus > 1 or os.environ.get("RAY_AMD_DATA_TRAINER", "0") == "1":
        return bench_data_trainer(args, n_gpus)

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
        ds = GPUImageNormalize(out_dtype="bf16", batch_size=bs, num_gpus=0.5 / _gpu_actors(),
                               concurrency=_gpu_actors(), keep_on_device=True).transform(ds)
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
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic uint8 images (pre-generated pool, per-block rotation)",
        "config": {"pipeline": pipe, "batch_size": bs, "data_path": path}}), flush=True)
    ray.shutdown()
