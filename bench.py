#!/usr/bin/env python
"""ray_amd headline benchmark.

Default workload (BASELINE.json config 2): Ray Train TorchTrainer GPT-2-small DDP,
bf16, synthetic tokens, random init — one rank per MI355X over RCCL. Each rank
runs exactly the per-worker step of ``ray_amd.train.examples.gpt2.train_func``
(forward, backward with bucketed RCCL all-reduce overlapped, clip, fused AdamW).

    python bench.py                       # N=1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

``--workload ppo`` runs the RLlib PPO synthetic-Atari throughput bench (BASELINE.json
config 3), ``impala`` the IMPALA V-trace one (config 5, 1 learner), ``data`` the Ray Data
→ GPU ingest pipeline (config 4, 1 GPU) and ``microbench`` the task/actor call-rate
microbenchmark (config 1). Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="gpt2",
                    choices=["gpt2", "ppo", "impala", "data", "microbench"])
    ap.add_argument("--micro-batch", type=int, default=64,
                    help="per-GPU sequences; 64 x 1024 tokens x 8 GPUs = 524k tokens, the GPT-3 "
                         "Small global batch")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--model", default="small")
    ap.add_argument("--tunableop", default="auto", choices=["off", "tune", "auto"],
                    help="PyTorch TunableOp GEMM selection: 'tune' benchmarks every hipBLASLt/"
                         "rocBLAS solution per GEMM shape during warmup and writes "
                         "profiles/tunableop/<config>.csv; 'auto' uses that file if present")
    return ap.parse_args()


def _setup_tunableop(args, rank):
    """Per-shape GEMM kernel selection (TunableOp) from a committed results file.

    TunableOp's validators pin the ROCm/hipBLASLt versions and the gfx arch, so a file
    tuned on this image's MI355X applies to every rank (each gets its own copy: the
    library keys result files by device)."""
    import shutil

    import torch

    if args.tunableop == "off":
        return None
    tdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "tunableop")
    name = f"gpt2_{args.model}_mb{args.micro_batch}_t{args.seq_len}.csv"
    src = os.path.join(tdir, name)
    if args.tunableop == "auto" and not os.path.exists(src):
        return None
    os.makedirs("/tmp/ray_amd_tunableop", exist_ok=True)
    dst = f"/tmp/ray_amd_tunableop/{os.getpid()}_{rank}_{name}"
    if os.path.exists(src):
        shutil.copyfile(src, dst)
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(args.tunableop == "tune")
    torch.cuda.tunable.set_filename(dst, insert_device_ordinal=False)
    if os.path.exists(dst):
        torch.cuda.tunable.read_file(dst)
    if args.tunableop == "tune":
        torch.cuda.tunable.set_max_tuning_duration(30)
        torch.cuda.tunable.set_max_tuning_iterations(20)
    return (dst, src) if args.tunableop == "tune" else None


def bench_gpt2(args):
    import torch
    import torch.distributed as dist

    from ray_amd.models.gpt2 import GPT2Config
    from ray_amd.train.gpt2_step import GPT2Trainer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    tuned = _setup_tunableop(args, rank)
    if tuned is not None:
        # GEMM tuning can run minutes without output: keep a heartbeat on stderr
        import threading

        def _beat(t0=time.time()):
            while True:
                time.sleep(30)
                print(f"[bench] tunableop tuning... {time.time() - t0:.0f}s", file=sys.stderr,
                      flush=True)

        threading.Thread(target=_beat, daemon=True).start()
    cfg = getattr(GPT2Config, args.model)()
    tr = GPT2Trainer(cfg, args.micro_batch, args.seq_len, dev, bucket_mb=args.bucket_mb,
                     total_steps=args.warmup + args.steps, grad_accum=args.grad_accum,
                     seed=1234)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    # synthetic token stream: pre-generate a pool so data generation is not timed work
    pool = [tr.synthetic_batch(gen) for _ in range(4 * args.grad_accum)]

    def batches(i):
        return [pool[(i * args.grad_accum + j) % len(pool)] for j in range(args.grad_accum)]

    for i in range(args.warmup):
        tr.step(batches(i))
    torch.cuda.synchronize()
    if tuned is not None and rank == 0:
        import shutil

        os.makedirs(os.path.dirname(tuned[1]), exist_ok=True)
        with open(tuned[1], "w") as f:  # TunableOp results-file format
            for k, v in torch.cuda.tunable.get_validators():
                f.write(f"Validator,{k},{v}\n")
            for op, params, kernel, t in torch.cuda.tunable.get_results():
                f.write(f"{op},{params},{kernel},{t}\n")
        torch.cuda.tunable.tuning_enable(False)
        shutil  # noqa: B018
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        tr.step(batches(args.warmup + i))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    loss = float(tr.last_loss)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    tokens = tr.tokens_per_step() * args.steps
    value = tokens / dt
    n_params = tr.model.num_params()
    flops = tr.model.flops_per_token(args.seq_len) * tokens
    if rank == 0:
        out = {
            "metric": "ray_train_gpt2_small_ddp_tokens_per_sec" if args.model == "small"
            else f"ray_train_gpt2_{args.model}_ddp_tokens_per_sec",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {
                "model": f"gpt2-{args.model}",
                "params": n_params,
                "global_batch": args.micro_batch * args.grad_accum * world,
                "micro_batch_per_gpu": args.micro_batch,
                "seq_len": args.seq_len,
                "parallelism": f"dp{world}",
                "bucket_mb": args.bucket_mb,
                "gemm_selection": "tunableop" if torch.cuda.tunable.is_enabled() else "heuristic",
            },
            "model_tflops_per_gpu": round(flops / dt / world / 1e12, 1),
            "final_loss": round(loss, 4),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.workload == "gpt2":
        bench_gpt2(args)
    elif args.workload == "ppo":
        from ray_amd.rllib.bench import bench_ppo

        bench_ppo(args)
    elif args.workload == "impala":
        from ray_amd.rllib.bench import bench_impala

        bench_impala(args)
    elif args.workload == "data":
        from ray_amd.data.bench import bench_data

        bench_data(args)
    else:  # BASELINE.json config 1: task/actor call rates (CPU plumbing)
        from ray_amd._private import ray_perf

        from ray_amd._private.raylet import detect_cpus

        res = ray_perf.main(quick=False, num_cpus=min(16, detect_cpus()))
        print(json.dumps({"metric": "ray_microbenchmark_calls_per_sec", "results": {
            r[0]: round(r[1], 1) for r in res}, "unit": "calls/s", "n_gpus": 0,
            "higher_is_better": True, "data": "synthetic"}), flush=True)


if __name__ == "__main__":
    main()
