"""Worker process entry point (reference: python/ray/_private/workers/default_worker.py)."""

from __future__ import annotations

import argparse
import json
import os
import sys

# Hardware queues per process (HIP's default is 4). A training process drives more streams
# than that — the compute stream, the weight-gradient side streams, the DDP comm stream and
# RCCL's internal streams — and streams beyond the queue count share a hardware queue,
# where one stream's event wait stalls the other's kernels. With 8 queues the GPT-2
# TorchTrainer step went from 68.6-68.7 to 65.8-66.1 ms and the DDP-hooks-on step from
# 69.6 to 66.4-66.5 ms on MI355X (profiles/r4/README.md §8). Set before HIP initialises,
# overriding an inherited GPU_MAX_HW_QUEUES (RAY_AMD_HW_QUEUES=<n> picks the count, 0 keeps
# the inherited setting).
if os.environ.get("RAY_AMD_HW_QUEUES", "8") != "0":  # 0: leave HIP's setting alone
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RAY_AMD_HW_QUEUES", "8")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--session-dir", required=True)
    ap.add_argument("--raylet", required=True)
    ap.add_argument("--token", type=int, required=True)
    ap.add_argument("--job", default=None)
    ap.add_argument("--node-id", default=None)
    args = ap.parse_args()
    lvl = os.environ.get("RAY_AMD_LOGGING_LEVEL")
    if lvl:  # init(logging_level=...): the workers' ray_amd logger follows the driver's
        import logging

        logging.getLogger("ray_amd").setLevel(int(lvl) if lvl.isdigit() else lvl.upper())
    try:  # die with the raylet / node agent that forked us (PR_SET_PDEATHSIG)
        import ctypes
        import signal

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGKILL))
    except Exception:
        pass
    extra = os.environ.get("RAY_AMD_JOB_SYS_PATH")
    if extra:
        for p in reversed(json.loads(extra)):
            if p and p not in sys.path:
                sys.path.insert(1, p)
    from ray_amd._private import worker as W
    from ray_amd._private.core_worker import CoreWorker
    from ray_amd._private.ids import random_bytes

    job = int(args.job) if args.job not in (None, "None") else None
    gpu_ids = [int(x) for x in os.environ.get("RAY_AMD_GPU_IDS", "").split(",") if x != ""]
    cw = CoreWorker(mode="worker", session_dir=args.session_dir, raylet_addr=args.raylet,
                    worker_id=random_bytes(16), job_id=job, gpu_ids=gpu_ids,
                    startup_token=args.token)
    W.global_worker.connect_worker(cw)
    cw.install_cancel_handler()  # ray.cancel interrupts the main thread with a real SIGINT
    hook = os.environ.get("RAY_AMD_SETUP_HOOK")
    if hook:
        cw.run_setup_hook(hook)
    try:
        # RAY_AMD_WORKER_CPROFILE=<dir>: the task loop and the dispatcher thread dump
        # cProfile stats there every 2 s (core-worker throughput diagnostics)
        cw.run_task_loop()
    finally:
        os._exit(0)


if __name__ == "__main__":
    main()
