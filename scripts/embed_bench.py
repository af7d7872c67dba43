"""Embedding backward at the GPT-2 bench shape (B 64, T 1024, C 768, V 50304): the HIP
kernel (ops/csrc/embed.hip) vs torch's index_add_ + batch-sum into fp32 sinks."""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops._lib import check, lib, ptr, stream_ptr  # noqa: E402


def timed(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    B, T, C, V = 64, 1024, 768, 50304
    idx = torch.randint(0, 50257, (B * T,), device="cuda")
    dx = torch.randn(B * T, C, device="cuda").bfloat16()
    wte = torch.zeros(V, C, device="cuda")
    wpe = torch.zeros(1024, C, device="cuda")
    L = lib()

    def hip():
        check(L.ra_embed_bwd(ptr(dx), ptr(idx), ptr(wte), ptr(wpe), B, T, C, V, stream_ptr()),
              "embed_bwd")

    def ref():
        wte.index_add_(0, idx, dx.to(torch.float32))
        wpe[:T].add_(dx.view(B, T, C).float().sum(0))

    print(json.dumps({"hip_ms": round(timed(hip), 4), "torch_ms": round(timed(ref), 4)}),
          flush=True)


if __name__ == "__main__":
    main()
