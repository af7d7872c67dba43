"""GELU backward + bias colsum at the GPT-2 MLP shape (65536 x 3072): v1 (knob 3 = 1) vs
v2 (branch-free, two-row register ring). Kernel-only times via rocprofv3."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_amd.ops import _lib  # noqa: E402
from ray_amd.ops._lib import ptr, stream_ptr  # noqa: E402


def main(N=65536, F=3072):
    L = _lib.lib()
    dev = "cuda"
    dy = torch.randn(N, F, device=dev).bfloat16()
    h = torch.randn(N, F, device=dev).bfloat16()
    fb = torch.zeros(F, device=dev).bfloat16()
    db = torch.zeros(F, device=dev)
    dh = torch.empty_like(h)
    work = torch.empty(L.ra_colsum_work(N, F), device=dev)
    gb = 3 * N * F * 2 / 1e9
    ref = None
    for name, knob in (("v1", 1), ("v2", 0), ("v1_again", 1), ("v2_again", 0)):
        L.ra_set_knob(3, knob)

        def f():
            L.ra_bias_gelu_bwd(ptr(dy), ptr(h), ptr(fb), ptr(dh), ptr(db), ptr(work), N, F, 2,
                               stream_ptr())
        f()
        torch.cuda.synchronize()
        got = torch.cat([dh.float().flatten()[:200000], db.clone()])
        ref = got if ref is None else ref
        err = ((got - ref).norm() / ref.norm()).item()
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30):
            f()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 30 * 1e3
        print(f"{name}: {ms:.4f} ms {gb / ms:.2f} TB/s rel-diff {err:.2e}", flush=True)
    L.ra_set_knob(3, 0)


if __name__ == "__main__":
    main()
