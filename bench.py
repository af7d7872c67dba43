#!/usr/bin/env python
"""ray_amd headline benchmark.

Default workload (BASELINE.json config 2): Ray Train TorchTrainer GPT-2-small DDP,
bf16, synthetic tokens, random init. ``ray_amd.init`` + ``TorchTrainer`` with
``--gpus`` worker actors, one per MI355X, joined in an RCCL process group; each
worker runs ``ray_amd.train.examples.gpt2.train_func`` (forward, backward with
bucketed RCCL all-reduce overlapped, clip, fused AdamW) and reports through
``train.report``. ``--no-ray`` runs the identical step as a bare
torch.distributed loop for comparison.

    python bench.py                       # N=1, TorchTrainer
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8
    # (under the launcher, rank 0 drives Ray; ranks 1..7 wait on a gloo barrier)

``--workload ppo`` runs the RLlib PPO synthetic-Atari throughput bench (BASELINE.json
config 3), ``impala`` the IMPALA V-trace one (config 5; ``--gpus N`` = N RCCL-joined GPU
learners), ``data`` the Ray Data → GPU ingest pipeline (config 4; ``--gpus N`` = N
TorchTrainer workers consuming dataset shards) and ``microbench`` the task/actor
call-rate microbenchmark (config 1). Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

# 8 hardware queues per process before HIP initialises (ray_amd/_private/worker_main.py has
# the measurement); Ray workers inherit it through the raylet's environment
if os.environ.get("RAY_AMD_HW_QUEUES", "8") != "0":  # 0: leave HIP's setting alone
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RAY_AMD_HW_QUEUES", "8")
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 20; the data workload defaults to 300: its "
                         "pipeline prefetches, so a 20-step window times blocks produced "
                         "during warmup)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="gpt2",
                    choices=["gpt2", "ppo", "impala", "data", "microbench", "allreduce"])
    ap.add_argument("--max-mb", type=int, default=256,
                    help="allreduce workload: largest all-reduce size (MiB), swept from 1 MiB "
                         "in powers of two")
    ap.add_argument("--no-ray", action="store_true",
                    help="gpt2: run the identical step in a bare torch.distributed loop "
                         "(one process per GPU under torch.distributed.run) instead of "
                         "TorchTrainer worker actors — the reference's vanilla-torch "
                         "comparison")
    ap.add_argument("--micro-batch", type=int, default=64,
                    help="per-GPU sequences; 64 x 1024 tokens x 8 GPUs = 524k tokens, the GPT-3 "
                         "Small global batch")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="flat gradient buffer / all-reduce dtype; bf16 = explicit gradient "
                         "compression")
    ap.add_argument("--lm-head-chunk", type=int, default=65536,
                    help="tokens per fused LM-head + cross-entropy chunk (65536 = the whole "
                         "64x1024 micro-batch in one chunk: 6.6 GB of bf16 logits, the "
                         "fastest on MI355X, profiles/r3/chunk/README.md)")
    ap.add_argument("--ddp-hooks", default="auto", choices=["auto", "always"],
                    help="gpt2: 'always' runs FlatDDP's bucket hooks, per-bucket events, comm "
                         "stream and RCCL all-reduce launches even at world size 1 (measures "
                         "the overlap machinery's cost on one GPU)")
    ap.add_argument("--step-graph", default="off", choices=["on", "off"],
                    help="gpt2: capture the whole training step as a HIP graph after warmup "
                         "(world-1 groups only). Off by default: measured 68.4 vs 67.1 ms "
                         "eager (profiles/r4/README.md) - the replayed graph overlaps the "
                         "wgrad side stream less than eager launches do")
    ap.add_argument("--model", default="small")
    ap.add_argument("--data-path", default="hbm", choices=["hbm", "h2d"],
                    help="data workload: GPU-preprocessed device blocks through the HBM "
                         "store (hbm) or host blocks + pinned H2D + consumer-side kernel")
    ap.add_argument("--tunableop", default="auto", choices=["off", "tune", "auto"],
                    help="PyTorch TunableOp GEMM selection: 'tune' benchmarks every hipBLASLt/"
                         "rocBLAS solution per GEMM shape during warmup and writes "
                         "ray_amd/tuned/<config>.csv; 'auto' uses that file if present")
    ap.add_argument("--device", default=None, help="gpt2: 'cpu' runs the launcher on gloo "
                    "(tests)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 300 if args.workload == "data" else 20
    return args


def _gpt2_config(args) -> dict:
    return dict(model=args.model, micro_batch=args.micro_batch, seq_len=args.seq_len,
                steps=args.steps, warmup=args.warmup, grad_accum=args.grad_accum,
                bucket_mb=args.bucket_mb, grad_dtype=args.grad_dtype, tunableop=args.tunableop,
                lm_head_chunk=args.lm_head_chunk, device=args.device, ddp_hooks=args.ddp_hooks,
                step_graph=args.step_graph == "on")


def _emit(args, r: dict, mode: str, n_gpus: int):
    out = {
        "metric": "ray_train_gpt2_small_ddp_tokens_per_sec" if args.model == "small"
        else f"ray_train_gpt2_{args.model}_ddp_tokens_per_sec",
        "value": round(r["tokens_per_sec"], 1),
        "unit": "tokens/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(r["ms_per_step"], 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic tokens, random-init weights",
        "config": {
            "model": f"gpt2-{args.model}",
            "params": r["params"],
            "global_batch": r["global_batch"],
            "micro_batch_per_gpu": args.micro_batch,
            "seq_len": args.seq_len,
            "parallelism": f"dp{n_gpus}",
            "bucket_mb": args.bucket_mb,
            "grad_dtype": r["grad_dtype"],
            "gemm_selection": r["gemm_selection"],
            "wgrad_gemm": r.get("wgrad_gemm"),
            "lm_head_chunk": args.lm_head_chunk,
            "launcher": mode,
            "ddp_hooks": r.get("ddp_hooks"),
            "step_graph": r.get("step_graph"),
        },
        "rccl_world_size": r["rccl_world_size"],
        "dist_backend": r["dist_backend"],
        "per_rank_ms_per_step": r["per_rank_ms_per_step"],
        "ranks_in_sync": r["ranks_in_sync"],
        "model_tflops_per_gpu": round(r["model_tflops_per_gpu"], 1),
        "final_loss": round(r["loss"], 4),
        "ddp_allreduce_launches": r.get("ddp_allreduce_launches"),
        "wgrad_stream_autotune": r.get("wgrad_stream_autotune"),
        "hbm": r.get("hbm"),
        "gpu_settle_wait_s": _SETTLE_WAIT,
    }
    # self-diagnosing multi-GPU runs: exposed comm, all-reduce launches / bytes and
    # per-bucket bus bandwidth per rank (FlatDDP.read_stats; zeros at world 1)
    out.update(r.get("ddp_stats") or {"ddp_exposed_comm_ms_per_step": 0.0,
                                       "ddp_allreduce_launches_per_step": 0.0,
                                       "ddp_allreduce_mb_per_step": 0.0})
    print(json.dumps(out), flush=True)


_LAUNCHER_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                  "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME",
                  "MASTER_ADDR", "MASTER_PORT")


def bench_gpt2_bare(args):
    """One process per GPU under torch.distributed.run, no Ray: the comparison baseline."""
    import torch
    import torch.distributed as dist

    from ray_amd.train.examples.gpt2 import run_steps

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device == "cpu":
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world == 1 and args.ddp_hooks == "always":  # a world-1 RCCL group to hook into
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29561")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if world > 1 or args.ddp_hooks == "always":
            dist.init_process_group("nccl", device_id=dev)
    r = run_steps(_gpt2_config(args), dev, rank, world)
    if rank == 0:
        _emit(args, r, "torch.distributed.run (no Ray)", world)
    from ray_amd.train.examples.gpt2 import release_device_memory

    release_device_memory(dev)
    if dist.is_initialized():
        dist.destroy_process_group()


def bench_gpt2_ray(args):
    """Ray Train: TorchTrainer with ``--gpus`` GPU worker actors on an RCCL group.

    Under torch.distributed.run (the driver's N>1 launch) only rank 0 drives Ray; the
    other launcher ranks hold no GPU and wait on a CPU (gloo) barrier until the Ray job
    is done, so each GPU is used by exactly one Train worker."""
    from datetime import timedelta

    import torch.distributed as dist

    launched = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if launched > 1:
        if launched != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} != launcher world size {launched}")
        dist.init_process_group("gloo", timeout=timedelta(hours=2))
        if rank != 0:
            dist.barrier()
            dist.destroy_process_group()
            return
    # the Ray cluster must not inherit the launcher's rendezvous identity
    for k in list(os.environ):
        if k in _LAUNCHER_VARS or k.startswith("TORCHELASTIC_"):
            os.environ.pop(k)
    import ray_amd as ray
    from ray_amd.train import RunConfig, ScalingConfig
    from ray_amd.train.examples.gpt2 import train_func
    from ray_amd.train.torch import TorchTrainer

    use_gpu = args.device != "cpu"
    try:
        ray.init(num_cpus=max(4, args.gpus + 2), num_gpus=args.gpus if use_gpu else 0,
                 include_dashboard=False, log_to_driver=True)
        trainer = TorchTrainer(
            train_func, train_loop_config=_gpt2_config(args),
            scaling_config=ScalingConfig(num_workers=args.gpus, use_gpu=use_gpu),
            run_config=RunConfig(name="bench_gpt2", storage_path="/tmp/ray_amd_bench"))
        result = trainer.fit()
        _emit(args, result.metrics, "ray_amd TorchTrainer", args.gpus)
    finally:
        ray.shutdown()
        if launched > 1:
            dist.barrier()
            dist.destroy_process_group()


def _rank0_only(args, fn):
    """Ray-driven workloads under torch.distributed.run: rank 0 runs ``fn`` (which starts
    Ray with --gpus GPU workers / learners), the other launcher ranks hold no GPU and wait
    on a CPU (gloo) barrier."""
    from datetime import timedelta

    import torch.distributed as dist

    launched = int(os.environ.get("WORLD_SIZE", "1"))
    if launched <= 1:
        return fn(args)
    if launched != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} != launcher world size {launched}")
    dist.init_process_group("gloo", timeout=timedelta(hours=2))
    rank = int(os.environ.get("RANK", "0"))
    try:
        if rank == 0:
            for k in list(os.environ):
                if k in _LAUNCHER_VARS or k.startswith("TORCHELASTIC_"):
                    os.environ.pop(k)
            fn(args)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def bench_allreduce(args):
    """RCCL (gloo with --device cpu) all-reduce size sweep, 1 MiB .. --max-mb MiB fp32, one
    process per GPU under torch.distributed.run: per size the median time of --steps
    launches after --warmup, algorithm and bus bandwidth (busbw = bytes / t x 2 (n-1) / n,
    what each xGMI link of the ring carries). Explains a GPT-2 scaling curve: FlatDDP's
    32 MiB buckets sit on this curve."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    if args.device == "cpu":
        dev = torch.device("cpu")
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=dev)
    rows = []
    mib = 1
    while mib <= args.max_mb:
        x = torch.ones(mib * (1 << 20) // 4, dtype=torch.float32, device=dev)
        for _ in range(args.warmup):
            dist.all_reduce(x)
        times = []
        for _ in range(args.steps):
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            dist.all_reduce(x)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t0)
        t = sorted(times)[len(times) // 2]
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt)
        nbytes = mib * (1 << 20)
        algbw = nbytes / t / 1e9
        # busbw = algbw x 2 (n-1) / n is a LINK figure: one rank has no link, so at N = 1 it
        # is null (the all-reduce is a local no-op copy, not a bus transfer)
        busbw = round(algbw * 2.0 * (world - 1) / world, 2) if world > 1 else None
        rows.append({"mib": mib, "ms": round(t * 1e3, 4), "algbw_gbps": round(algbw, 2),
                     "busbw_gbps": busbw})
        mib *= 2
    if rank == 0:
        print(json.dumps({"metric": "allreduce_busbw_gbps", "value": rows[-1]["busbw_gbps"],
                          "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "higher_is_better": True,
                          "backend": dist.get_backend(), "dtype": "fp32",
                          "data": "synthetic", "sweep": rows}), flush=True)
    dist.destroy_process_group()


def _other_gpu_processes_vram() -> int:
    """Bytes of HBM that OTHER processes hold on the visible GPU(s), from `rocm-smi
    --showpids` (KFD process table; processes of this job — our torchrun siblings — are
    excluded). -1 when rocm-smi is unavailable."""
    import shutil
    import subprocess

    exe = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
    if not os.path.exists(exe):
        return -1
    try:
        out = subprocess.run([exe, "--showpids"], capture_output=True, text=True,
                             timeout=20).stdout
    except (OSError, subprocess.SubprocessError):
        return -1
    me, parent = os.getpid(), os.getppid()
    total = 0
    for line in out.splitlines():
        f = line.split()
        if len(f) < 4 or not f[0].isdigit() or not f[3].isdigit():
            continue
        pid = int(f[0])
        if pid == me:
            continue
        try:
            with open(f"/proc/{pid}/stat") as fh:
                if int(fh.read().rsplit(")", 1)[1].split()[1]) == parent:
                    continue  # a sibling rank of this job
        except (OSError, ValueError, IndexError):
            pass  # gone from /proc but still in the KFD table: its teardown is running
        total += int(f[3])
    return total


def _settle_gpu(max_wait_s: float) -> float:
    """Wait (before any GPU work) until no other process holds HBM on this GPU. A process
    that exits with tens of GB allocated stays in the KFD table with that memory for
    ~30 s while the driver tears it down; a two-stream step started in that window ran
    140-316 ms instead of 62-64 (profiles/r5/r5p, r5y, r5aa). Returns seconds waited."""
    t0 = time.time()
    while time.time() - t0 < max_wait_s:
        held = _other_gpu_processes_vram()
        if held < (1 << 30):  # -1 (no rocm-smi) or under 1 GiB
            break
        time.sleep(2.0)
    return round(time.time() - t0, 1)


_SETTLE_WAIT = None


def main():
    global _SETTLE_WAIT
    args = parse()
    # not under a profiler: its preloaded library has initialised the GPU before main(),
    # and the settle check starts rocm-smi (a Python script) as a child process
    profiled = any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)
    if args.workload in ("gpt2", "allreduce") and args.device != "cpu" and not profiled and \
            os.environ.get("RAY_AMD_BENCH_SETTLE", "1") == "1":
        _SETTLE_WAIT = _settle_gpu(float(os.environ.get("RAY_AMD_BENCH_SETTLE_MAX_S", "120")))
    if args.workload == "gpt2":
        if args.no_ray:
            bench_gpt2_bare(args)
        else:
            bench_gpt2_ray(args)
    elif args.workload == "ppo":
        from ray_amd.rllib.bench import bench_ppo

        _rank0_only(args, bench_ppo)
    elif args.workload == "impala":
        from ray_amd.rllib.bench import bench_impala

        _rank0_only(args, bench_impala)
    elif args.workload == "allreduce":
        bench_allreduce(args)
    elif args.workload == "data":
        from ray_amd.data.bench import bench_data

        _rank0_only(args, bench_data)
    else:  # BASELINE.json config 1: task/actor call rates (CPU plumbing)
        from ray_amd._private import ray_perf

        from ray_amd._private.raylet import detect_cpus

        res = ray_perf.main(quick=False, num_cpus=min(16, detect_cpus()))
        print(json.dumps({"metric": "ray_microbenchmark_calls_per_sec", "results": {
            r[0]: round(r[1], 1) for r in res}, "unit": "calls/s", "n_gpus": 0,
            "higher_is_better": True, "data": "synthetic"}), flush=True)


if __name__ == "__main__":
    main()
