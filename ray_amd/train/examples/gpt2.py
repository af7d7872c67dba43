"""GPT-2 DDP training as a Ray Train workload — the headline benchmark body.

``train_func`` is the ``train_loop_per_worker`` that ``bench.py`` hands to
``TorchTrainer(scaling_config=ScalingConfig(num_workers=N, use_gpu=True))``. Each
worker actor owns one MI355X (the raylet binds the device before the process
starts), the TorchConfig backend has already initialised an RCCL process group
over all N workers, and the loop runs ``GPT2Trainer.step`` (forward, backward with
bucketed RCCL all-reduce overlapped, clip, fused AdamW) on synthetic tokens.

Timing protocol (same as the bare-loop baseline ``bench.py --no-ray``): ``warmup``
untimed steps, then exactly ``steps`` timed steps bracketed by barrier +
device synchronize on both sides; the MAX elapsed time over ranks is the step
time. Rank 0 reports through ``train.report``.

Reference parity: release/air_tests/air_benchmarks/workloads/torch_benchmark.py:81
(train_func run under TorchTrainer, :233, compared against a vanilla torch run).
"""

from __future__ import annotations

import os
import sys
import threading
import time

DEFAULTS = dict(model="small", micro_batch=64, seq_len=1024, steps=20, warmup=5,
                grad_accum=1, bucket_mb=32.0, grad_dtype="fp32", tunableop="auto",
                lm_head_chunk=65536, device=None, ddp_hooks="auto")


def tunableop_file(model: str, micro_batch: int, seq_len: int) -> str:
    # ray_amd/tuned/: shipped with the package (profiles/ is not uploaded to GPU boxes)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    return os.path.join(root, "tuned", f"gpt2_{model}_mb{micro_batch}_t{seq_len}.csv")


def setup_tunableop(mode: str, src: str, rank: int):
    """Per-shape GEMM kernel selection (PyTorch TunableOp) from a committed results file.

    'tune' benchmarks every hipBLASLt/rocBLAS solution per GEMM shape during warmup (the
    caller writes the file afterwards with ``save_tunableop``); 'auto' uses the file if
    present; 'off' keeps hipBLASLt's heuristic. Returns the selection label."""
    import shutil

    import torch

    if mode == "off" or (mode == "auto" and not os.path.exists(src)):
        return "heuristic"
    os.makedirs("/tmp/ray_amd_tunableop", exist_ok=True)
    dst = f"/tmp/ray_amd_tunableop/{os.getpid()}_{rank}_{os.path.basename(src)}"
    if os.path.exists(src):
        shutil.copyfile(src, dst)
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(mode == "tune")
    torch.cuda.tunable.set_filename(dst, insert_device_ordinal=False)
    if os.path.exists(dst):
        torch.cuda.tunable.read_file(dst)
    if mode == "tune":
        # per candidate solution: at most 20 ms / 10 timed runs (hundreds of hipBLASLt
        # solutions per GEMM shape)
        torch.cuda.tunable.set_max_tuning_duration(20)
        torch.cuda.tunable.set_max_tuning_iterations(10)

        def _beat(t0=time.time()):  # tuning can run minutes without output
            while torch.cuda.tunable.tuning_is_enabled():
                time.sleep(30)
                print(f"[gpt2] tunableop tuning... {time.time() - t0:.0f}s", file=sys.stderr,
                      flush=True)

        threading.Thread(target=_beat, daemon=True).start()
        return "tunableop-tuning"
    return "tunableop"


def save_tunableop(dst: str):
    import torch

    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:  # TunableOp results-file format
        for k, v in torch.cuda.tunable.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for op, params, kernel, t in torch.cuda.tunable.get_results():
            f.write(f"{op},{params},{kernel},{t}\n")
    torch.cuda.tunable.tuning_enable(False)


def _master_checksum(p32):
    """Device-side checksum of the WHOLE fp32 master buffer: its sum and a position-weighted
    sum (weights 1..9973 by index), in fp64, in 16M-element chunks, so ranks whose masters
    differ anywhere (or are permuted) disagree."""
    import torch

    flat = p32.reshape(-1)
    acc = torch.zeros(2, dtype=torch.float64, device=flat.device)
    step = 1 << 24
    for s in range(0, flat.numel(), step):
        x = flat[s:s + step].double()
        w = torch.arange(s, s + x.numel(), device=x.device, dtype=torch.float64) \
            .remainder_(9973).add_(1.0)
        acc[0] += x.sum()
        acc[1] += (x * w).sum()
    return acc


def run_steps(cfg: dict, device, rank: int, world: int) -> dict:
    """Build the model on ``device`` and run warmup + timed steps (shared by the Ray Train
    worker and the bare torchrun baseline). torch.distributed must already be set up
    when world > 1."""
    import torch
    import torch.distributed as dist

    from ray_amd.models.gpt2 import GPT2Config
    from ray_amd.train.gpt2_step import GPT2Trainer

    c = dict(DEFAULTS, **(cfg or {}))
    on_gpu = device.type == "cuda"
    gemm = "heuristic"
    tfile = tunableop_file(c["model"], c["micro_batch"], c["seq_len"])
    if on_gpu:
        gemm = setup_tunableop(c["tunableop"], tfile, rank)
        if c["tunableop"] == "tune":
            from ray_amd.ops import lt

            lt.set_tuning(True)  # fp32-output wgrad GEMMs: ops/lt.py selector
    mcfg = getattr(GPT2Config, c["model"])()
    gdt = torch.float32 if c["grad_dtype"] == "fp32" else torch.bfloat16
    tr = GPT2Trainer(mcfg, c["micro_batch"], c["seq_len"], device, bucket_mb=c["bucket_mb"],
                     total_steps=c["warmup"] + c["steps"], grad_accum=c["grad_accum"],
                     seed=1234, grad_dtype=gdt, lm_head_chunk=c["lm_head_chunk"],
                     ddp_always_hook=c["ddp_hooks"] == "always")
    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + rank)
    # synthetic token pool generated up front: data generation is not timed work
    pool = [tr.synthetic_batch(gen) for _ in range(4 * c["grad_accum"])]

    def batches(i):
        ga = c["grad_accum"]
        return [pool[(i * ga + j) % len(pool)] for j in range(ga)]

    def sync():
        if on_gpu:
            torch.cuda.synchronize(device)

    # Side-stream autotune inside the warmup (RAY_AMD_STREAM_AUTOTUNE=1, default): the last
    # 4 of >= 5 warmup steps alternate single-stream / side-stream weight gradients (each
    # step timed on its own), and the timed steps use the side stream unless the single
    # stream was clearly (>3 %) faster. On a settled box the side stream wins by ~1 ms
    # (profiles/r5/r5s: 62.7 vs 63.8 ms); on MI355X boxes right after another multi-stream
    # process exited, two-stream steps ran ~180 ms against ~64 ms single-stream for ~30 s
    # (profiles/r5/r5p). The decision is all-reduced so every rank runs one mode. Still
    # exactly `warmup` untimed steps.
    from ray_amd.ops import functional as rf

    auto = on_gpu and os.environ.get("RAY_AMD_STREAM_AUTOTUNE", "1") == "1" and \
        c["warmup"] >= 5 and rf._WGRAD_STREAM
    first_ab = c["warmup"] - 4
    times = {True: [], False: []}
    ab = None
    for i in range(c["warmup"]):
        mode = None
        if auto and i >= first_ab:
            mode = (i - first_ab) % 2 == 1  # serial, side, serial, side
            sync()
            rf._WGRAD_STREAM = mode
            t_mark = time.perf_counter()
        tr.step(batches(i))
        if mode is not None:
            sync()
            times[mode].append(time.perf_counter() - t_mark)
    sync()
    if auto:
        side_ms = sum(times[True]) / len(times[True]) * 1e3
        serial_ms = sum(times[False]) / len(times[False]) * 1e3
        v = torch.tensor([side_ms, serial_ms], device=device, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
        side_ms, serial_ms = float(v[0]), float(v[1])
        rf._WGRAD_STREAM = not (serial_ms < 0.97 * side_ms)
        ab = {"side_stream_ms": round(side_ms, 3), "serial_ms": round(serial_ms, 3),
              "chosen": "side" if rf._WGRAD_STREAM else "serial"}
    if gemm == "tunableop-tuning":
        if rank == 0:
            save_tunableop(tfile)
        else:
            torch.cuda.tunable.tuning_enable(False)
        gemm = "tunableop"
    if on_gpu:
        from ray_amd.ops import lt

        if lt._tuning:  # tunableop=tune or RAY_AMD_LT_TUNE=1: keep the fp32-out choices
            if rank == 0:
                print(f"[gpt2] hipBLASLt fp32-out choices -> {lt.save()}", file=sys.stderr)
            lt.set_tuning(False)
    graphed = False
    # whole-step HIP graph: opt-in (step_graph=True or RAY_AMD_STEP_GRAPH=1); eager is
    # faster on MI355X at this config (profiles/r4/README.md)
    if on_gpu and (c.get("step_graph") or os.environ.get("RAY_AMD_STEP_GRAPH") == "1"):
        graphed = tr.enable_graph(batches(c["warmup"]))
        sync()
    diag = on_gpu and tr.ddp.enabled and os.environ.get("RAY_AMD_DDP_STATS", "1") == "1"
    tr.ddp.stats = diag
    tr.ddp.reset_stats()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(c["steps"]):
        tr.step(batches(c["warmup"] + i))
    sync()
    if world > 1:
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    ddp_stats = tr.ddp.read_stats(c["steps"])
    if world > 1:  # per-rank diagnostics gathered to every rank (rank 0 reports them)
        vals = torch.tensor([ddp_stats["ddp_exposed_comm_ms_per_step"],
                             ddp_stats["ddp_allreduce_ms_per_step"]], device=device,
                            dtype=torch.float64)
        allv = [torch.zeros_like(vals) for _ in range(world)]
        dist.all_gather(allv, vals)
        ddp_stats["per_rank_exposed_comm_ms"] = [round(float(v[0]), 4) for v in allv]
        ddp_stats["per_rank_allreduce_ms"] = [round(float(v[1]), 4) for v in allv]
    loss = float(tr.last_loss)
    per_rank = [dt]
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per_rank = [float(x) for x in allt]
        dt = max(per_rank)
        # ranks must hold identical weights after the run (same all-reduced grads)
        chk = _master_checksum(tr.flat.p32)
        allc = [torch.zeros_like(chk) for _ in range(world)]
        dist.all_gather(allc, chk)
        in_sync = all(torch.equal(x, allc[0]) for x in allc)
    else:
        in_sync = True
    tokens = tr.tokens_per_step() * c["steps"]
    flops = tr.model.flops_per_token(c["seq_len"]) * tokens
    mem = None
    if on_gpu:
        st = torch.cuda.memory_stats(device)
        mem = {"max_allocated_gb": round(torch.cuda.max_memory_allocated(device) / 2**30, 2),
               "reserved_gb": round(torch.cuda.memory_reserved(device) / 2**30, 2),
               "alloc_retries": int(st.get("num_alloc_retries", 0)),
               "device_mallocs": int(st.get("num_device_alloc", 0)),
               "device_frees": int(st.get("num_device_free", 0)),
               "segments": int(st.get("segment.all.current", 0))}
    return {
        "tokens_per_sec": tokens / dt,
        "ms_per_step": dt / c["steps"] * 1000,
        "per_rank_ms_per_step": [round(x / c["steps"] * 1000, 3) for x in per_rank],
        "world_size": world,
        "rccl_world_size": dist.get_world_size() if dist.is_initialized() else 1,
        "dist_backend": dist.get_backend() if dist.is_initialized() else None,
        "model_tflops_per_gpu": flops / dt / world / 1e12,
        "params": tr.model.num_params(),
        "loss": loss,
        "ranks_in_sync": in_sync,
        "gemm_selection": gemm,
        "wgrad_gemm": _wgrad_mode(on_gpu),
        "grad_dtype": c["grad_dtype"],
        "global_batch": c["micro_batch"] * c["grad_accum"] * world,
        "ddp_hooks": "on" if tr.ddp.enabled else "off",
        "ddp_allreduce_launches": tr.ddp.launched,
        "step_graph": graphed,
        "ddp_stats": ddp_stats,
        "wgrad_stream_autotune": ab,
        "hbm": mem,
    }


def _wgrad_mode(on_gpu: bool) -> str:
    return "hip-wgrad-kernel" if on_gpu else "torch"


def train_func(config: dict):
    """train_loop_per_worker for TorchTrainer."""
    import torch.distributed as dist

    from ray_amd import train
    from ray_amd.train.torch import get_device

    ctx = train.get_context()
    dev = get_device()
    if (config or {}).get("device") == "cpu":
        import torch

        dev = torch.device("cpu")
    world = dist.get_world_size() if dist.is_initialized() else ctx.get_world_size()
    out = run_steps(config, dev, ctx.get_world_rank(), world)
    out["device"] = str(dev)
    release_device_memory(dev)
    train.report(out)


def release_device_memory(dev):
    """Hand the step's cached HBM back to the driver before the process ends (the model and
    activations are garbage once run_steps returned). A process that exits holding tens of
    GB stays in the KFD table for ~30 s while the kernel tears it down, and two-stream work
    of the NEXT process on that GPU is 2-5x slower meanwhile (profiles/r5/r5p, r5aa)."""
    import gc

    import torch

    if getattr(dev, "type", None) != "cuda":
        return
    gc.collect()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
