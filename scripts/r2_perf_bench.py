"""Round-2 GPT-2 component microbenchmarks on one MI355X (GPT-2 small, 64 x 1024 tokens).

    python scripts/r2_perf_bench.py [--part wgrad,lmhead,xent]

wgrad : weight-gradient GEMM variants into an fp32 flat-gradient sink
lmhead: fused chunked LM-head cross-entropy (fwd+bwd) per chunk size
xent  : the in-place fused softmax-xent kernel alone (HBM GB/s)
"""

import argparse
import json

import torch

from ray_amd.ops import _lib
from ray_amd.ops import functional as rf
from ray_amd.ops._lib import ptr, stream_ptr


def timeit(fn, iters=20, warmup=3):
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


def bench_wgrad(M=65536, C=768):
    dev, bf = "cuda", torch.bfloat16
    L = _lib.lib()
    out = {}
    for name, (N, K) in {"qkv": (3 * C, C), "proj": (C, C), "fc": (4 * C, C),
                         "mlp_proj": (C, 4 * C)}.items():
        x = torch.randn(M, K, device=dev, dtype=bf)
        dy = torch.randn(M, N, device=dev, dtype=bf)
        sink = torch.zeros(N, K, device=dev, dtype=torch.float32)
        fl = 2 * M * N * K
        r = {}
        for S in (1, 2, 4, 8, 16):
            dys = dy.view(S, M // S, N).transpose(1, 2)
            xs = x.view(S, M // S, K)

            def f(S=S, dys=dys, xs=xs):
                part = torch.bmm(dys, xs, out_dtype=torch.float32)
                L.ra_splitk_accum(ptr(part), S, N * K, ptr(sink), 3, stream_ptr())

            r[f"splitk{S}"] = timeit(f)
        r["addmm_f32"] = timeit(lambda: torch.addmm(sink, dy.t(), x, out_dtype=torch.float32,
                                                    out=sink))
        r["addmm_f32_T"] = timeit(lambda: torch.addmm(sink.t(), x.t(), dy,
                                                      out_dtype=torch.float32, out=sink.t()))
        out[name] = {k: f"{v:.4f} ms {fl / v / 1e9:.0f} TF" for k, v in r.items()}
    return out


def bench_lmhead(N=65536, C=768, V=50257, Vp=50304):
    dev = "cuda"
    h = (torch.randn(N, C, device=dev) * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(Vp, C, device=dev) * 0.05).bfloat16().requires_grad_()
    t = torch.randint(0, V, (N,), device=dev)
    fl = 3 * 2 * N * Vp * C
    out = {}
    for ch in (2048, 4096, 8192, 16384):
        def f(ch=ch):
            h.grad = None
            w.grad = None
            rf.lm_head_cross_entropy(h, w, t, V, chunk=ch).backward()

        ms = timeit(f, iters=5, warmup=2)
        out[f"chunk{ch}"] = f"{ms:.3f} ms {fl / ms / 1e9:.0f} TF(gemm-equiv)"
    return out


def bench_xent(N=8192, V=50257, Vp=50304):
    dev = "cuda"
    L = _lib.lib()
    lg = torch.randn(N, Vp, device=dev).bfloat16()
    t = torch.randint(0, V, (N,), device=dev)
    inv = torch.ones(1, device=dev)
    loss = torch.empty(N, device=dev)
    ms = timeit(lambda: L.ra_xent_fused(ptr(lg), ptr(t), ptr(inv), ptr(loss), N, V, Vp, -100,
                                        stream_ptr()))
    gb = 2 * N * Vp * 2 / 1e9
    return {"xent_fused_8192": f"{ms:.4f} ms {gb / ms:.2f} TB/s"}


def bench_norm(N=65536, D=768, F=3072):
    """LayerNorm backward (residual seam, 3 column sums into fp32 sinks) and bias-GELU
    backward at the GPT-2 shape, under the occupancy / colsum knobs."""
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
    h = torch.randn(N, F, device=dev).bfloat16()
    dyf = torch.randn(N, F, device=dev).bfloat16()
    fb = torch.zeros(F, device=dev).bfloat16()
    fb._ra_direct_grad = True
    fb._ra_grad = torch.zeros(F, device=dev)
    out = {}
    for cap, waves, atom in ((512, 2048, 0), (2048, 2048, 0), (2048, 8192, 0), (2048, 8192, 1),
                             (1024, 8192, 1), (4096, 16384, 1)):
        L.ra_set_knob(0, cap)
        L.ra_set_knob(1, waves)
        L.ra_set_knob(2, atom)
        t_ln = timeit(lambda: rf._ln_backward(dy, x, w, b, mean, rstd, dres=dres, rbias=rb))
        ctx = type("C", (), {})()

        def gelu_bwd():
            dh = torch.empty_like(h)
            work = torch.empty(L.ra_colsum_work(N, F), device=dev)
            L.ra_bias_gelu_bwd(ptr(dyf), ptr(h), ptr(fb), ptr(dh), ptr(fb._ra_grad), ptr(work),
                               N, F, 3, stream_ptr())

        t_g = timeit(gelu_bwd)
        t_c = timeit(lambda: rf._colsum_bf16(dyf, out=fb._ra_grad))
        ln_gb = 4 * N * D * 2 / 1e9
        g_gb = 3 * N * F * 2 / 1e9
        out[f"cap{cap}_waves{waves}_atomic{atom}"] = (
            f"ln_bwd {t_ln:.4f} ms {ln_gb / t_ln:.2f} TB/s | gelu_bwd {t_g:.4f} ms "
            f"{g_gb / t_g:.2f} TB/s | colsum {t_c:.4f} ms {N * F * 2 / 1e9 / t_c:.2f} TB/s")
    L.ra_set_knob(0, 2048)
    L.ra_set_knob(1, 8192)
    L.ra_set_knob(2, 1)
    return out


def bench_imgnorm(N=256, H=224, W=224, C=3):
    """uint8 NHWC -> bf16/fp32 NCHW normalisation: HBM bytes moved per second."""
    x = torch.randint(0, 256, (N, H, W, C), dtype=torch.uint8, device="cuda")
    out = {}
    L = _lib.lib()
    for mode, knob in (("cached", 0), ("nontemporal", 2)):
        L.ra_set_knob(5, knob)
        for name, dt, ob in (("bf16", torch.bfloat16, 2), ("fp32", torch.float32, 4)):
            ms = timeit(lambda dt=dt: rf.image_normalize(x, (0.485, 0.456, 0.406),
                                                         (0.229, 0.224, 0.225), dt), iters=50)
            nbytes = N * H * W * C * (1 + ob)
            out[f"{name}_{mode}"] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                                     "images_per_s": round(N / ms * 1e3, 1)}
    L.ra_set_knob(5, 0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", default="norm,wgrad,lmhead,xent")
    a = ap.parse_args()
    res = {}
    for p in a.part.split(","):
        res[p] = {"wgrad": bench_wgrad, "lmhead": bench_lmhead, "xent": bench_xent,
                  "norm": bench_norm, "imgnorm": bench_imgnorm}[p]()
        print(json.dumps({p: res[p]}), flush=True)


if __name__ == "__main__":
    main()
