"""Hand-written MFMA GEMM (ops/csrc/gemm.hip) vs torch/hipBLASLt at the GPT-2 small shapes.

Checks each shape against an fp32 reference, then times both (CUDA events, interleaved
rounds in one process, uniform random operands). Prints one JSON line per shape.
    python scripts/hip_gemm_bench.py [--iters 20] [--grid 0]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops import gemm  # noqa: E402
from ray_amd.ops._lib import lib  # noqa: E402

SHAPES = [  # name, M, N, K
    ("qkv_fwd", 65536, 2304, 768),
    ("proj_fwd", 65536, 768, 768),
    ("fc_fwd", 65536, 3072, 768),
    ("fc2_fwd", 65536, 768, 3072),
    ("qkv_dgrad", 65536, 768, 2304),
    ("fc_dgrad", 65536, 768, 3072),
    ("fc2_dgrad", 65536, 3072, 768),
    ("lm_fwd", 8192, 50304, 768),
    ("lm_dgrad", 8192, 768, 50304),
]


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--no-epi", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for name, M, N, K in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        b = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        ref = a.float() @ b.float().t()
        out = gemm.gemm_nt(a, b)
        torch.cuda.synchronize()
        err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        del ref
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_hip, t_lt = [], []
        for _ in range(args.rounds):
            t_hip.append(timeit(lambda: gemm.gemm_nt(a, b, out=c), args.iters))
            t_lt.append(timeit(lambda: torch.mm(a, b.t(), out=c), args.iters))
        fl = 2.0 * M * N * K
        th, tl = min(t_hip), min(t_lt)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "max_rel_err": round(err, 5),
                          "hip_ms": round(th, 4), "torch_ms": round(tl, 4),
                          "hip_tflops": round(fl / th / 1e9, 1),
                          "torch_tflops": round(fl / tl / 1e9, 1),
                          "speedup": round(tl / th, 3)}), flush=True)
        del a, b, c, out
    if args.no_epi:
        return
    # fused epilogues at the MLP shapes
    M, F, C = 65536, 3072, 768
    x = (torch.rand(M, C, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(F, C, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    bias = ((torch.rand(F, device=dev) * 2 - 1) * 0.1).to(torch.bfloat16)
    y, pre = gemm.gemm_nt(x, w, epi="bias_gelu", bias=bias)
    pre_ref = x.float() @ w.float().t()
    y_ref = torch.nn.functional.gelu(pre.float() + bias.float(), approximate="tanh")
    e1 = ((pre.float() - pre_ref).abs().max() / pre_ref.abs().max()).item()
    e2 = ((y.float() - y_ref).abs().max() / y_ref.abs().max()).item()
    w2t = ((torch.rand(F, C, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # W_proj^T
    dy = ((torch.rand(M, C, device=dev) * 2 - 1)).to(torch.bfloat16)
    db = torch.zeros(F, device=dev, dtype=torch.float32)
    dh = gemm.gemm_nt(dy, w2t, epi="dgelu", bias=bias, aux=pre, db=db)
    u = (pre.float() + bias.float()).requires_grad_(True)
    g = torch.autograd.grad(torch.nn.functional.gelu(u, approximate="tanh"), u,
                            dy.float() @ w2t.float().t())[0]
    e3 = ((dh.float() - g).abs().max() / g.abs().max()).item()
    e4 = ((db - g.sum(0)).abs().max() / g.sum(0).abs().max()).item()
    t_fused = min(timeit(lambda: gemm.gemm_nt(x, w, epi="bias_gelu", bias=bias, out=y, aux=pre),
                         args.iters) for _ in range(args.rounds))
    t_dg = min(timeit(lambda: gemm.gemm_nt(dy, w2t, epi="dgelu", bias=bias, aux=pre, out=dh,
                                           db=db, db_acc=True), args.iters)
               for _ in range(args.rounds))
    print(json.dumps({"epilogues": "mlp", "bias_gelu_pre_err": round(e1, 5),
                      "bias_gelu_y_err": round(e2, 5), "dgelu_err": round(e3, 5),
                      "dbias_err": round(e4, 5), "bias_gelu_ms": round(t_fused, 4),
                      "dgelu_db_ms": round(t_dg, 4)}), flush=True)


if __name__ == "__main__":
    main()
