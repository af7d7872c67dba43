"""HIP causal attention at the GPT-2 small training shape (B 64, T 1024, H 12, D 64):
forward, backward (split dK/dV + dQ) timings and TFLOP/s (causal FLOPs: fwd 2 GEMMs,
bwd 5 GEMM-equivalents). Prints one JSON line.
    python scripts/attn_bench3.py [--B 64] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops import _lib  # noqa: E402
from ray_amd.ops._lib import ptr, stream_ptr  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B, T, H, D = a.B, a.T, a.H, 64
    L = _lib.lib()
    dev = "cuda"
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3, H, D, device=dev).bfloat16()
    out = torch.empty(B, T, H, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, T, device=dev)
    dout = torch.randn(B, T, H, D, device=dev).bfloat16()
    delta = torch.empty(B, H, T, device=dev)
    dqkv = torch.empty_like(qkv)
    sc = D ** -0.5
    f_fwd = lambda: L.ra_attn_fwd(ptr(qkv), ptr(out), ptr(lse), B, T, H, D, sc, stream_ptr())
    f_pre = lambda: L.ra_attn_bwd_pre(ptr(out), ptr(dout), ptr(delta), B, T, H, stream_ptr())
    f_kv = lambda: L.ra_attn_bwd_kv(ptr(qkv), ptr(dout), ptr(lse), ptr(delta), ptr(dqkv), B, T,
                                    H, D, sc, stream_ptr())
    f_q = lambda: L.ra_attn_bwd_q(ptr(qkv), ptr(dout), ptr(lse), ptr(delta), ptr(dqkv), B, T, H,
                                  D, sc, stream_ptr())
    f_fwd()
    f_pre()
    fl = 2 * 2 * B * H * T * T * D / 2  # one causal GEMM-pair (QK^T + PV)
    r = {}
    for name, fn, mult in (("fwd", f_fwd, 1.0), ("bwd_pre", f_pre, 0), ("bwd_kv", f_kv, 2.0),
                           ("bwd_q", f_q, 1.5)):
        ms = min(timeit(fn, a.iters) for _ in range(3))
        r[name] = {"ms": round(ms, 4)}
        if mult:
            r[name]["tflops_mfma"] = round(mult * fl / ms / 1e9, 1)
    tb = r["bwd_pre"]["ms"] + r["bwd_kv"]["ms"] + r["bwd_q"]["ms"]
    r["bwd_total"] = {"ms": round(tb, 4), "tflops_useful": round(2.5 * fl / tb / 1e9, 1)}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
