"""Quadrant-phased MFMA GEMM (ops/csrc/gemm.hip variant 3) vs hipBLASLt (torch.mm).

Correctness vs an fp32 reference (incl. ragged shapes), then interleaved timing rounds in
one process on uniform random [-1, 1) operands. One JSON line per shape.
    python scripts/gemm8_bench.py [--variants 3,0] [--only qkv_fwd,...]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops import gemm  # noqa: E402
from ray_amd.ops._lib import lib  # noqa: E402

_L = None


def set_variant(v):
    """v < 4: gemm.hip schedule ra_knobs[5] = v; v == 4: the 4-wave gemm4w.hip kernel."""
    gemm.set_four_wave(v == 4)
    if v < 4:
        _L.ra_set_knob(5, v)

SHAPES = [  # name, M, N, K
    ("sq4096", 4096, 4096, 4096),
    ("sq8192", 8192, 8192, 8192),
    ("qkv_fwd", 65536, 2304, 768),
    ("proj_fwd", 65536, 768, 768),
    ("fc_fwd", 65536, 3072, 768),
    ("fc2_fwd", 65536, 768, 3072),
    ("qkv_dgrad", 65536, 768, 2304),
    ("fc2_dgrad", 65536, 3072, 768),
    ("lm_fwd", 8192, 50304, 768),
    ("lm_dgrad", 8192, 768, 50304),
]
RAGGED = [(300, 260, 128), (1000, 516, 192), (257, 1028, 64), (4096, 772, 640)]


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def rel_err(out, a, b):
    ref = a.float() @ b.float().t()
    return ((out.float() - ref).abs().max() / ref.abs().max()).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="3")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    global _L
    L = _L = lib()
    for M, N, K in RAGGED:
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        for v in variants:
            set_variant(v)
            e = rel_err(gemm.gemm_nt(a, b), a, b)
            print(json.dumps({"ragged": [M, N, K], "variant": v, "max_rel_err": round(e, 5)}),
                  flush=True)
            assert e < 0.02, (M, N, K, v, e)
    for name, M, N, K in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        errs = {}
        for v in variants:
            set_variant(v)
            errs[v] = round(rel_err(gemm.gemm_nt(a, b), a, b), 5) if M * N <= 65536 * 3072 else None
        times = {v: [] for v in variants}
        t_lt = []
        for _ in range(args.rounds):
            for v in variants:
                set_variant(v)
                times[v].append(timeit(lambda: gemm.gemm_nt(a, b, out=c), args.iters))
            t_lt.append(timeit(lambda: torch.mm(a, b.t(), out=c), args.iters))
        fl = 2.0 * M * N * K
        tl = min(t_lt)
        rec = {"shape": name, "M": M, "N": N, "K": K, "torch_ms": round(tl, 4),
               "torch_tflops": round(fl / tl / 1e9, 1)}
        for v in variants:
            th = min(times[v])
            rec[f"v{v}_ms"] = round(th, 4)
            rec[f"v{v}_tflops"] = round(fl / th / 1e9, 1)
            rec[f"v{v}_vs_torch"] = round(tl / th, 3)
            rec[f"v{v}_err"] = errs[v]
        print(json.dumps(rec), flush=True)
        del a, b, c
    L.ra_set_knob(5, 0)


if __name__ == "__main__":
    main()
