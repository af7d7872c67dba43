"""GPT-2 MLP passes: hipBLASLt GEMM + separate elementwise kernel vs ops/csrc/gemm.hip with
the elementwise work fused into the GEMM epilogue (M = 65536 tokens, C = 768, F = 3072).

  fc fwd   : h = x @ Wfc^T ; a = gelu(h + b)            vs gemm_nt(epi="bias_gelu")
  proj dgrad: g = dy @ Wp  ; dh = g * gelu'(h + b), db   vs gemm_nt(epi="dgelu")

Correctness against the unfused pair, then interleaved timing rounds (CUDA events) in one
process. One JSON line per pass.
    python scripts/mlp_fused_bench.py [--rounds 3] [--iters 20]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops import functional as rf  # noqa: E402
from ray_amd.ops import gemm  # noqa: E402
from ray_amd.ops._lib import check, lib, ptr, stream_ptr  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="0")
    args = ap.parse_args()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    M, C, F = 65536, 768, 3072
    x = (torch.randn(M, C, device=dev) * 0.5).bfloat16()
    wfc = (torch.randn(F, C, device=dev) * 0.03).bfloat16()
    bfc = (torch.randn(F, device=dev) * 0.1).bfloat16()
    wp = (torch.randn(C, F, device=dev) * 0.03).bfloat16()
    wpt = wp.t().contiguous()  # [F, C]: dgrad B operand (the W^T AdamW keeps)
    dy = (torch.randn(M, C, device=dev) * 0.5).bfloat16()
    L = lib()

    # ---- fc forward
    def fwd_unfused():
        h = torch.mm(x, wfc.t())
        return rf.bias_gelu(h, bfc), h

    def fwd_fused():
        return gemm.gemm_nt(x, wfc, epi="bias_gelu", bias=bfc)

    a0, h0 = fwd_unfused()
    a1, h1 = fwd_fused()
    out = {"fc_fwd": {"rel_act": rel(a1, a0), "rel_pre": rel(h1, h0)}}

    # ---- proj dgrad + GELU backward + bias grad
    hpre = h0  # pre-activation without bias (as the fused forward saves it)
    work = torch.empty(L.ra_colsum_work(M, F), device=dev, dtype=torch.float32)
    db0 = torch.zeros(F, device=dev, dtype=torch.float32)
    db1 = torch.zeros(F, device=dev, dtype=torch.float32)

    def bwd_unfused():
        g = torch.mm(dy, wpt.t())  # dy @ wp
        dh = torch.empty_like(g)
        check(L.ra_bias_gelu_bwd(ptr(g), ptr(hpre), ptr(bfc), ptr(dh), ptr(db0), ptr(work),
                                 M, F, 1 | 2, stream_ptr()), "bias_gelu_bwd")
        return dh

    def bwd_fused():
        return gemm.gemm_nt(dy, wpt, epi="dgelu", bias=bfc, aux=hpre, db=db1, db_acc=False)

    db0.zero_()
    d0 = bwd_unfused()
    d1 = bwd_fused()
    torch.cuda.synchronize()
    out["proj_dgrad"] = {"rel_dh": rel(d1, d0), "rel_db": rel(db1, db0)}

    variants = [int(v) for v in args.variants.split(",")]
    t = {k: [] for k in ("fwd_unfused", "bwd_unfused")}
    for v in variants:
        t[f"fwd_fused_v{v}"] = []
        t[f"bwd_fused_v{v}"] = []
    for _ in range(args.rounds):
        t["fwd_unfused"].append(round(timed(fwd_unfused, args.iters), 4))
        t["bwd_unfused"].append(round(timed(bwd_unfused, args.iters), 4))
        for v in variants:
            L.ra_set_knob(5, v)
            t[f"fwd_fused_v{v}"].append(round(timed(fwd_fused, args.iters), 4))
            t[f"bwd_fused_v{v}"].append(round(timed(bwd_fused, args.iters), 4))
        L.ra_set_knob(5, 0)
    # parts of the unfused pair
    t["fc_gemm_only"] = [round(timed(lambda: torch.mm(x, wfc.t()), args.iters), 4)]
    t["dgrad_gemm_only"] = [round(timed(lambda: torch.mm(dy, wpt.t()), args.iters), 4)]
    out["ms"] = t
    out["shape"] = {"M": M, "C": C, "F": F}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
