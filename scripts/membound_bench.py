#!/usr/bin/env python
"""Memory-bound passes of the GPT-2-small step, solo, at the bench shapes (65536 tokens):
bias+GELU forward / backward (+ bias gradient), residual LayerNorm forward / backward
(+ 3 column sums into fp32 sinks), the fused LM-head cross-entropy and the flat AdamW.
Prints one JSON line per pass: us per call and algorithmic TB/s (bytes each pass must move).

    python scripts/membound_bench.py [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops import functional as rf  # noqa: E402
from ray_amd.ops._lib import check, lib, ptr, stream_ptr  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3  # us


def report(name, us, nbytes, **kw):
    print(json.dumps({"pass": name, "us": round(us, 1), "GB": round(nbytes / 1e9, 3),
                      "TBps": round(nbytes / us / 1e6, 2), **kw}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = "cuda"
    N, C, F, V = 65536, 768, 3072, 50304
    L = lib()
    want = set(a.only.split(",")) if a.only else None

    def on(n):
        return want is None or n in want

    bf = torch.bfloat16
    if on("gelu"):
        h = torch.randn(N, F, device=dev).to(bf)
        b = (0.1 * torch.randn(F, device=dev)).to(bf)
        y = torch.empty_like(h)
        report("bias_gelu_fwd", timeit(lambda: check(L.ra_bias_gelu_fwd(
            ptr(h), ptr(b), ptr(y), N, F, stream_ptr())), a.iters), 2 * h.numel() * 2)
        dy = torch.randn(N, F, device=dev).to(bf)
        dh = torch.empty_like(h)
        db = torch.zeros(F, device=dev)
        work = torch.empty(L.ra_colsum_work(N, F), device=dev)
        report("bias_gelu_bwd", timeit(lambda: check(L.ra_bias_gelu_bwd(
            ptr(dy), ptr(h), ptr(b), ptr(dh), ptr(db), ptr(work), N, F, 1 | 2, stream_ptr())),
            a.iters), 3 * h.numel() * 2)
        del h, y, dy, dh
    if on("ln"):
        hh = torch.randn(N, C, device=dev).to(bf)
        sk = torch.randn(N, C, device=dev).to(bf)
        rb = (0.1 * torch.randn(C, device=dev)).to(bf)
        w = (1 + 0.1 * torch.randn(C, device=dev)).to(bf)
        bb = (0.1 * torch.randn(C, device=dev)).to(bf)
        xo = torch.empty_like(hh)
        yy = torch.empty_like(hh)
        mean = torch.empty(N, device=dev)
        rstd = torch.empty(N, device=dev)
        report("residual_ln_fwd", timeit(lambda: check(L.ra_residual_layernorm_fwd(
            ptr(hh), ptr(rb), ptr(sk), ptr(xo), ptr(w), ptr(bb), ptr(yy), ptr(mean), ptr(rstd),
            N, C, 1e-5, stream_ptr())), a.iters), 4 * hh.numel() * 2)
        dy = torch.randn(N, C, device=dev).to(bf)
        dres = torch.randn(N, C, device=dev).to(bf)
        dx = torch.empty_like(hh)
        sinks = [torch.zeros(C, device=dev) for _ in range(3)]
        work = torch.empty(L.ra_layernorm_bwd_work(N, C), device=dev)
        report("residual_ln_bwd", timeit(lambda: check(L.ra_layernorm_bwd(
            ptr(dy), ptr(xo), ptr(w), ptr(mean), ptr(rstd), ptr(dres), ptr(dx), ptr(sinks[0]),
            ptr(sinks[1]), ptr(sinks[2]), ptr(work), N, C, 2, stream_ptr())), a.iters),
            4 * hh.numel() * 2)
        del hh, sk, xo, yy, dy, dres, dx
    if on("xent"):
        logits = (2 * torch.randn(N, V, device=dev)).to(bf)
        tg = torch.randint(0, 50257, (N,), device=dev)
        inv = torch.full((1,), 1.0 / N, device=dev)
        loss = torch.empty(N, device=dev)
        # in place: later iterations read gradients, same traffic and the same VALU work
        report("xent_fused", timeit(lambda: check(L.ra_xent_fused(
            ptr(logits), ptr(tg), ptr(inv), ptr(loss), N, 50257, V, -100, stream_ptr())),
            max(3, a.iters // 4)), 2 * logits.numel() * 2)
        del logits
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
