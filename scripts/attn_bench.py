"""Time the HIP flash attention against torch SDPA (aotriton on ROCm) at GPT-2 shape.

python scripts/attn_bench.py [--B 16 --T 1024 --H 12]
"""

import argparse
import json

import torch
import torch.nn.functional as F

from ray_amd.ops import functional as rf


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
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
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    a = ap.parse_args()
    B, T, H, D = a.B, a.T, a.H, 64
    dev = "cuda"
    qkv = torch.randn(B, T, 3, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16)
    flops_fwd = 4 * B * H * T * T * D / 2  # causal
    res = {}

    def ours_fwd():
        with torch.no_grad():
            rf.causal_attention_qkv(qkv)

    def ours_fb():
        y = rf.causal_attention_qkv(qkv)
        y.backward(g)

    def sdpa(x):
        q, k, v = x.permute(2, 0, 3, 1, 4).unbind(0)
        return F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2)

    def sdpa_fwd():
        with torch.no_grad():
            sdpa(qkv)

    def sdpa_fb():
        sdpa(qkv).backward(g)

    for name, fn in (("ours_fwd", ours_fwd), ("ours_fwd_bwd", ours_fb), ("sdpa_fwd", sdpa_fwd),
                     ("sdpa_fwd_bwd", sdpa_fb)):
        ms = timeit(fn)
        mult = 1 if name.endswith("fwd") else 3.5  # bwd = 2.5x fwd flops
        res[name] = {"ms": round(ms, 4), "tflops": round(mult * flops_fwd / ms / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
