"""Cross-stream latency probe: N round trips of (tiny kernel on stream A -> event ->
stream B waits, tiny kernel -> event -> stream A waits). On a healthy MI355X a round trip
is tens of microseconds; when the process's hardware queues are being time-sliced (the
state seen right after another large process exited, profiles/r5/r5p) it is milliseconds.

    python scripts/stream_probe.py [--iters 200] [--every 2] [--duration 40]
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def probe(iters=200):
    import torch

    a = torch.cuda.Stream()
    b = torch.cuda.Stream()
    x = torch.zeros(1024, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        with torch.cuda.stream(a):
            x.add_(1)
        b.wait_stream(a)
        with torch.cuda.stream(b):
            x.add_(1)
        a.wait_stream(b)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--every", type=float, default=2.0)
    ap.add_argument("--duration", type=float, default=40.0)
    args = ap.parse_args()
    import torch

    torch.zeros(1, device="cuda")
    t0 = time.time()
    while True:
        us = probe(args.iters)
        print(json.dumps({"t": round(time.time() - t0, 1), "roundtrip_us": round(us, 1)}),
              flush=True)
        if time.time() - t0 > args.duration:
            break
        time.sleep(args.every)


if __name__ == "__main__":
    main()
