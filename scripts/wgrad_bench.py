"""Weight-gradient GEMM at the GPT-2 small shapes (M = 65536 tokens): the hand-written
CDNA4 kernel (ops/csrc/wgrad.hip, incl. its slab reduction into an fp32 sink) against the
hipBLASLt split-K partials + ra_splitk_accum path it replaces, and against the fp32
reference for accuracy. Interleaved rounds in one process (rule 24), random operands.

    python scripts/wgrad_bench.py [--rounds 5]
"""

import argparse
import json

import torch

from ray_amd.ops import _lib, lt
from ray_amd.ops import functional as rf
from ray_amd.ops._lib import ptr, stream_ptr

SHAPES = {"qkv": (65536, 2304, 768), "proj": (65536, 768, 768), "fc": (65536, 3072, 768),
          "mlp_proj": (65536, 768, 3072)}


def timeit(fn, iters=20):
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bias", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    out = {}
    for name, (M, N, K) in SHAPES.items():
        torch.manual_seed(0)
        dy = (torch.rand(M, N, device=dev) * 2 - 1).bfloat16()
        x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        sink = torch.zeros(N, K, device=dev)
        bsink = torch.zeros(N, device=dev) if args.bias else None
        S_lt = rf._splitk(M, N, K)

        def hip():
            rf.wgrad_accumulate(dy, x, sink, bsink)

        def blas():
            part = lt.wgrad_partials(dy, x, S_lt)
            L.ra_splitk_accum(ptr(part), S_lt, N * K, ptr(sink), 3, stream_ptr())

        def hip_kernel_only():
            S = L.ra_wgrad_splits(M, N, K)
            ws = torch.empty(S * N * K, device=dev)
            L.ra_wgrad(ptr(dy), N, ptr(x), K, M, N, K, S, ptr(ws), None, 0, stream_ptr())

        # accuracy vs fp32
        ref = dy.float().t() @ x.float()
        sink.zero_()
        rf.wgrad_accumulate(dy, x, sink)
        torch.cuda.synchronize()
        err = ((sink - ref).norm() / ref.norm()).item()
        flop = 2.0 * M * N * K
        res = {"S_hip": L.ra_wgrad_splits(M, N, K), "S_lt": S_lt, "rel_err": err}
        for r in range(args.rounds):
            for arm, fn in (("hip", hip), ("hipblaslt", blas), ("hip_kernel", hip_kernel_only)):
                ms = timeit(fn)
                res.setdefault(arm, []).append(round(ms, 4))
        for arm in ("hip", "hipblaslt", "hip_kernel"):
            best = min(res[arm])
            res[arm + "_tflops"] = round(flop / best / 1e9, 1)
        out[name] = res
        print(name, json.dumps(res), flush=True)
    # one GPT-2 layer as ONE grouped launch (in-kernel split-K reduction) vs the four
    # per-linear hip launches (+ their slab reductions)
    import ctypes

    torch.manual_seed(0)
    prob = []
    for name, (M, N, K) in SHAPES.items():
        prob.append(((torch.rand(M, N, device=dev) * 2 - 1).bfloat16(),
                     (torch.rand(M, K, device=dev) * 2 - 1).bfloat16(),
                     torch.zeros(N, K, device=dev)))
    n = len(prob)
    M = 65536
    tiles = sum(((d.shape[1] + 255) // 256) * ((x.shape[1] + 255) // 256) for d, x, _ in prob)
    S = L.ra_wgrad_group_splits(M, tiles)
    ws = torch.empty((L.ra_wgrad_group_ws_bytes(tiles, S) + 3) // 4, device=dev)
    P, I, Lg = ctypes.c_void_p * n, ctypes.c_int * n, ctypes.c_long * n
    gargs = (n, P(*[ptr(d) for d, _, _ in prob]), Lg(*[d.stride(0) for d, _, _ in prob]),
            P(*[ptr(x) for _, x, _ in prob]), Lg(*[x.stride(0) for _, x, _ in prob]),
            P(*[ptr(s) for _, _, s in prob]), P(*[None] * n),
            I(*[d.shape[1] for d, _, _ in prob]), I(*[x.shape[1] for _, x, _ in prob]),
            I(*[2] * n), M, S, ptr(ws))

    def grouped():
        L.ra_wgrad_group(*gargs, stream_ptr())

    def per_linear():
        for d, x, s_ in prob:
            rf.wgrad_accumulate(d, x, s_)

    for _, _, s_ in prob:
        s_.zero_()
    grouped()
    torch.cuda.synchronize()
    errs = [((s_ - d.float().t() @ x.float()).norm() / (d.float().t() @ x.float()).norm()).item()
            for d, x, s_ in prob]
    g_ms, p_ms = [], []
    for r in range(args.rounds):
        g_ms.append(round(timeit(grouped), 4))
        p_ms.append(round(timeit(per_linear), 4))
    flop = sum(2.0 * M * d.shape[1] * x.shape[1] for d, x, _ in prob)
    print("layer_group", json.dumps({"S": S, "tiles": tiles, "rel_err_max": max(errs),
                                      "grouped_ms": g_ms, "per_linear_ms": p_ms,
                                      "grouped_tflops": round(flop / min(g_ms) / 1e9, 1),
                                      "per_linear_tflops": round(flop / min(p_ms) / 1e9, 1)}),
          flush=True)
    tot_h = sum(min(v["hip"]) for v in out.values())
    tot_b = sum(min(v["hipblaslt"]) for v in out.values())
    print(json.dumps({"per_layer_ms_hip": round(tot_h, 4), "per_layer_ms_hipblaslt": round(tot_b, 4),
                      "per_step_ms_hip": round(12 * tot_h, 3),
                      "per_step_ms_hipblaslt": round(12 * tot_b, 3)}))


if __name__ == "__main__":
    main()
