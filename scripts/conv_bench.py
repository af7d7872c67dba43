#!/usr/bin/env python
"""Nature-CNN conv layers at the PPO learner minibatch (B=500): MFMA kernels (ops/csrc/conv.hip)
vs MIOpen NHWC, forward and weight gradient.

    python scripts/conv_bench.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops import _lib  # noqa: E402
from ray_amd.ops import functional as rf  # noqa: E402
from ray_amd.ops._lib import check, ptr, stream_ptr  # noqa: E402

LAYERS = [("conv1_u8", 84, 4, 32, 8, 4, True), ("conv2", 20, 32, 64, 4, 2, False),
          ("conv3", 9, 64, 64, 3, 1, False)]


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=500)
    a = ap.parse_args()
    L = _lib.lib()
    dev = torch.device("cuda")
    out = []
    for name, HW, C, O, K, S, u8 in LAYERS:
        B = a.B
        w = (torch.randn(O, C, K, K, device=dev) * 0.05).bfloat16().contiguous(
            memory_format=torch.channels_last)
        b = torch.zeros(O, device=dev).bfloat16()
        if u8:
            frames = torch.randint(0, 256, (5000, HW, HW, C), dtype=torch.uint8, device=dev)
            idx = torch.randperm(5000, device=dev)[:B]
            xin = frames
            xb = (frames[idx].float() / 255).bfloat16().permute(0, 3, 1, 2)
        else:
            idx = None
            xb = torch.randn(B, HW, HW, C, device=dev).bfloat16().permute(0, 3, 1, 2)
            xin = xb
        OH = (HW - K) // S + 1
        y = torch.empty(B, OH, OH, O, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(B, OH, OH, O, device=dev).bfloat16()
        dw = torch.empty(O, K, K, C, device=dev, dtype=torch.bfloat16)
        xh = xin if u8 else xin.permute(0, 2, 3, 1)
        rec = {"layer": name, "B": B}
        rec["fwd_us"] = round(timeit(lambda: check(L.ra_conv_fwd(
            ptr(xh), ptr(idx), int(u8), ptr(w), ptr(b), ptr(y), B, HW, HW, C, K, K, S, O,
            1 / 255.0, 1, stream_ptr()), "fwd")), 2)
        work = torch.empty(L.ra_conv_wgrad_work(B, HW, HW, C, K, K, S, O), device=dev)
        rec["wgrad_us"] = round(timeit(lambda: check(L.ra_conv_wgrad(
            ptr(xh), ptr(idx), int(u8), ptr(dy), ptr(work), work.numel(), ptr(dw), 0, B, HW, HW,
            C, K, K, S, O, 1 / 255.0, stream_ptr()), "wgrad")), 2)
        dyc = dy.permute(0, 3, 1, 2)
        rec["miopen_fwd_us"] = round(timeit(lambda: torch.nn.functional.conv2d(xb, w, b, S)), 2)
        rec["miopen_wgrad_us"] = round(timeit(lambda: torch.ops.aten.convolution_backward(
            dyc, xb, w, None, [S, S], [0, 0], [1, 1], False, [0, 0], 1,
            [False, True, False])), 2)
        if not u8 and L.ra_conv_dgrad_supported(K, K, C, S, O):
            dx = torch.empty(B, HW, HW, C, device=dev, dtype=torch.bfloat16)
            rec["dgrad_us"] = round(timeit(lambda: check(L.ra_conv_dgrad(
                ptr(dy), ptr(w), ptr(dx), B, HW, HW, C, K, K, S, O, stream_ptr()), "dgrad")), 2)
        if not u8:
            rec["miopen_dgrad_us"] = round(timeit(lambda: torch.ops.aten.convolution_backward(
                dyc, xb, w, None, [S, S], [0, 0], [1, 1], False, [0, 0], 1,
                [True, False, False])), 2)
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()
