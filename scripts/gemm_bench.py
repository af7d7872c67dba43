"""Per-shape hipBLASLt timing of the GPT-2 GEMMs (fwd / dgrad / wgrad) at B*T tokens.

python scripts/gemm_bench.py [--tokens 16384] [--model small]
"""

import argparse
import json

import torch


def timeit(fn, iters=30, warmup=5):
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
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--V", type=int, default=50304)
    a = ap.parse_args()
    M, C = a.tokens, a.C
    dev = "cuda"
    bf = torch.bfloat16
    shapes = {"qkv": (3 * C, C), "proj": (C, C), "fc": (4 * C, C), "mlp_proj": (C, 4 * C),
              "lm_head": (a.V, C)}
    out = {}
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf)
        dy = torch.randn(M, N, device=dev, dtype=bf)
        fl = 2 * M * N * K
        r = {}
        r["fwd"] = timeit(lambda: torch.nn.functional.linear(x, w))
        r["dgrad"] = timeit(lambda: dy @ w)
        r["wgrad"] = timeit(lambda: dy.t() @ x)
        r["wgrad_alt"] = timeit(lambda: (x.t() @ dy).t())
        g = torch.zeros(N, K, device=dev, dtype=bf)
        r["wgrad_accum"] = timeit(lambda: g.addmm_(dy.t(), x))
        if name != "lm_head":
            for S in (2, 4, 8):
                dys = dy.view(S, M // S, N).transpose(1, 2)
                xs = x.view(S, M // S, K)
                r[f"splitk{S}_bf16"] = timeit(lambda: torch.bmm(dys, xs))
                r[f"splitk{S}_f32"] = timeit(lambda: torch.bmm(dys, xs, out_dtype=torch.float32))
                part = torch.bmm(dys, xs, out_dtype=torch.float32)
                r[f"splitk{S}_f32+sum"] = timeit(
                    lambda: torch.bmm(dys, xs, out_dtype=torch.float32).sum(0))
                ref = (dy.float().t() @ x.float())
                err = ((part.sum(0) - ref).norm() / ref.norm()).item()
                r[f"splitk{S}_relerr"] = err
                e2 = ((torch.bmm(dys, xs).float().sum(0) - ref).norm() / ref.norm()).item()
                r[f"splitk{S}_bf16_relerr"] = e2
            r["plain_relerr"] = (((dy.t() @ x).float() - ref).norm() / ref.norm()).item()
        out[name] = {k: (f"{v:.2e}" if "err" in k else
                         f"{v:.4f} ms {fl / v / 1e9:.0f} TF") for k, v in r.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
