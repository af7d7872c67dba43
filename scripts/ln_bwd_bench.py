"""LayerNorm backward at the GPT-2 shape (65536 x 768, residual seam, 3 column sums):
v1 (guarded, knob 3 = 1) vs v2 (branch-free buffer ops) over grid sizes. Kernel-only
times come from rocprofv3; this prints wall times per call."""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from ray_amd.ops import _lib  # noqa: E402
from ray_amd.ops import functional as rf  # noqa: E402


def main(N=65536, D=768):
    dev = "cuda"
    L = _lib.lib()
    x = torch.randn(N, D, device=dev).bfloat16()
    dy = torch.randn(N, D, device=dev).bfloat16()
    dres = torch.randn(N, D, device=dev).bfloat16()
    w = torch.ones(D, device=dev).bfloat16()
    b = torch.zeros(D, device=dev).bfloat16()
    rb = torch.zeros(D, device=dev).bfloat16()
    mean = x.float().mean(-1)
    rstd = torch.rsqrt(x.float().var(-1, unbiased=False) + 1e-5)
    sinks = [torch.zeros(D, device=dev) for _ in range(3)]
    for p_, s_ in zip((w, b, rb), sinks):
        p_._ra_direct_grad = True
        p_._ra_grad = s_
    gb = 4 * N * D * 2 / 1e9
    ref = None
    for name in ("v2_p512",):
        for s_ in sinks:
            s_.zero_()
        dx = rf._ln_backward(dy, x, w, b, mean, rstd, dres=dres, rbias=rb)[0]
        torch.cuda.synchronize()
        got = torch.cat([dx.float().flatten()[:100000]] + [s_.clone() for s_ in sinks])
        if ref is None:
            ref = got
        err = ((got - ref).norm() / ref.norm()).item()
        for _ in range(3):
            rf._ln_backward(dy, x, w, b, mean, rstd, dres=dres, rbias=rb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 50
        for _ in range(n):
            rf._ln_backward(dy, x, w, b, mean, rstd, dres=dres, rbias=rb)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        print(f"{name}: {ms:.4f} ms/call (incl. colsums) {gb / ms:.2f} TB/s  rel-diff "
              f"{err:.2e}", flush=True)


if __name__ == "__main__":
    main()
