"""A/B of the attention backward prefetch variants at the GPT-2 training shape, interleaved
in one process: dK/dV (ra_knobs[11]: 0 = two Q/dO register sets, 1 = one, 2 = one + both query halves in
flight) and dQ
(ra_knobs[12], same for K/V), plus a check of every variant's dQKV against an fp32
PyTorch reference on a small batch. Prints one JSON line.

    python scripts/attn_bwd_ab.py [--B 64] [--rounds 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.ops import _lib  # noqa: E402
from ray_amd.ops._lib import ptr, stream_ptr  # noqa: E402


def ref_grads(qkv, dout, scale):
    x = qkv.float().requires_grad_()
    q, k, v = (t.transpose(1, 2) for t in x.unbind(2))
    s = q @ k.transpose(-1, -2) * scale
    T = s.shape[-1]
    s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device=s.device), 1),
                      float("-inf"))
    o = (torch.softmax(s, -1) @ v).transpose(1, 2)
    o.backward(dout.float())
    return x.grad


def run_bwd(L, qkv, out, dout, lse, delta, dqkv, B, T, H, sc):
    L.ra_attn_bwd_pre(ptr(out), ptr(dout), ptr(delta), B, T, H, stream_ptr())
    L.ra_attn_bwd_kv(ptr(qkv), ptr(dout), ptr(lse), ptr(delta), ptr(dqkv), B, T, H, 64, sc,
                     stream_ptr())
    L.ra_attn_bwd_q(ptr(qkv), ptr(dout), ptr(lse), ptr(delta), ptr(dqkv), B, T, H, 64, sc,
                    stream_ptr())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = _lib.lib()
    D = 64
    sc = D ** -0.5
    res = {}

    def alloc(B):
        qkv = torch.randn(B, a.T, 3, a.H, D, device="cuda").bfloat16()
        out = torch.empty(B, a.T, a.H, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, a.H, a.T, device="cuda")
        L.ra_attn_fwd(ptr(qkv), ptr(out), ptr(lse), B, a.T, a.H, D, sc, stream_ptr())
        dout = torch.randn(B, a.T, a.H, D, device="cuda").bfloat16()
        delta = torch.empty(B, a.H, a.T, device="cuda")
        dqkv = torch.empty_like(qkv)
        return qkv, out, dout, lse, delta, dqkv

    torch.manual_seed(3)
    qkv, out, dout, lse, delta, dqkv = alloc(2)
    ref = ref_grads(qkv, dout, sc)
    for kv in (0, 1, 2):
        for q in (0, 1):
            L.ra_set_knob(11, kv)
            L.ra_set_knob(12, q)
            run_bwd(L, qkv, out, dout, lse, delta, dqkv, 2, a.T, a.H, sc)
            torch.cuda.synchronize()
            err = ((dqkv.float() - ref).norm() / ref.norm()).item()
            res[f"kv{kv}_q{q}_rel_err"] = round(err, 5)
    torch.manual_seed(0)
    B = a.B
    qkv, out, dout, lse, delta, dqkv = alloc(B)
    L.ra_attn_bwd_pre(ptr(out), ptr(dout), ptr(delta), B, a.T, a.H, stream_ptr())
    times = {f"{k}{v}": [] for k in ("kv", "q") for v in ((0, 1, 2) if k == "kv" else (0, 1))}
    for _ in range(a.rounds):
        for v in (0, 1, 2):
            for kind in ("kv", "q"):
                if kind == "q" and v == 2:
                    continue
                L.ra_set_knob(11 if kind == "kv" else 12, v)
                f = L.ra_attn_bwd_kv if kind == "kv" else L.ra_attn_bwd_q
                args = (ptr(qkv), ptr(dout), ptr(lse), ptr(delta), ptr(dqkv), B, a.T, a.H, D,
                        sc, stream_ptr())
                f(*args)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    f(*args)
                e.record()
                torch.cuda.synchronize()
                times[f"{kind}{v}"].append(s.elapsed_time(e) / a.iters)
    for k, t in times.items():
        t = sorted(t)
        res[f"{k}_ms_median"] = round(t[len(t) // 2], 4)
    L.ra_set_knob(11, 0)
    L.ra_set_knob(12, 0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
