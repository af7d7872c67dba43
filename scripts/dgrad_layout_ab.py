"""Input-gradient GEMM layout A/B at the GPT-2 small training shapes (65536 tokens):
dX = dY @ W with W stored [out, in] (what autograd does today: TunableOp op "nn") against
dX = dY @ Wt.t() with a transposed copy Wt [in, out] (op "tn", the forward GEMMs' layout).
TunableOp runs with the committed GPT-2 file and tunes shapes it lacks (into /tmp).
Also times the transpose copy that keeping Wt current would cost per step. One JSON line.

    python scripts/dgrad_layout_ab.py
"""
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                   "tunableop", "gpt2_small_mb64_t1024.csv")


def timeit(fn, iters=20):
    for _ in range(3):
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
    dst = f"/tmp/dgrad_ab_{os.getpid()}.csv"
    shutil.copy(SRC, dst)
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(dst, insert_device_ordinal=False)
    torch.cuda.tunable.read_file(dst)
    torch.cuda.tunable.set_max_tuning_duration(20)
    M, C = 65536, 768
    # (name, out features, in features) of each Linear: dX[M, in] = dY[M, out] @ W[out, in]
    shapes = [("qkv", 3 * C, C), ("proj", C, C), ("fc", 4 * C, C), ("mlp_proj", C, 4 * C)]
    res = {}
    tot_nn = tot_tn = tot_tr = 0.0
    for name, o, i in shapes:
        dy = torch.randn(M, o, device="cuda").bfloat16()
        w = (torch.randn(o, i, device="cuda") * 0.02).bfloat16()
        wt = w.t().contiguous()
        a = dy @ w
        b = dy @ wt.t()
        err = ((a.float() - b.float()).abs().max() / a.float().abs().max()).item()
        t_nn = timeit(lambda: torch.mm(dy, w))
        t_tn = timeit(lambda: torch.mm(dy, wt.t()))
        t_tr = timeit(lambda: wt.copy_(w.t()))
        res[name] = {"nn_ms": round(t_nn, 4), "tn_ms": round(t_tn, 4),
                     "transpose_ms": round(t_tr, 4), "max_rel_diff": round(err, 6)}
        tot_nn += t_nn
        tot_tn += t_tn
        tot_tr += t_tr
    res["per_layer_ms"] = {"nn": round(tot_nn, 4), "tn": round(tot_tn, 4),
                           "transpose": round(tot_tr, 4)}
    res["per_step_saving_ms_12_layers"] = round(12 * (tot_nn - tot_tn - tot_tr), 3)
    print(json.dumps(res), flush=True)
    # the tuned entries of this process (torch 2.10 has no tunable.write_file: the
    # results table is read back instead)
    old = set(open(SRC).read().splitlines())
    rows = [",".join(str(x) for x in r) for r in torch.cuda.tunable.get_results()]
    print(json.dumps({"new_tunableop_entries": [r for r in rows if r not in old]}),
          flush=True)


if __name__ == "__main__":
    main()
