"""Per-step GPU timeline from a rocprofv3 SQLite trace (``*_results.db``): wall, busy union,
per-stream kernel time, and the idle gaps of each stream (steps split at the AdamW kernel).

    python scripts/rocpd_timeline.py gpurun_out/x/prof/p_results.db [--gap-us 5]

A "gap" on a stream is time between one of its kernels ending and its next kernel starting
while the step is still running: on the main (critical-path) stream it is a wait on another
stream or the host. The largest gaps are listed with the kernel that ended before each one.
"""
import argparse
import glob
import os
import sqlite3
from collections import defaultdict


def load(path):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) \
        else [path]
    rows = []
    for f in dbs:
        c = sqlite3.connect(f)
        q = ("select d.start, d.end, s.kernel_name, d.stream_id from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        rows += list(c.execute(q))
    return sorted(rows)


def short(name, n=60):
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--gap-us", type=float, default=5.0)
    a = ap.parse_args()
    ks = load(a.path)
    ends = [i for i, k in enumerate(ks) if "adamw" in k[2]]
    out = []
    for a_i, b_i in zip(ends[:-1], ends[1:]):
        step = ks[a_i + 1:b_i + 1]
        t0, t1 = step[0][0], max(k[1] for k in step)
        iv = sorted((s, e) for s, e, _, _ in step)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        per = defaultdict(int)
        by_stream = defaultdict(list)
        for s, e, n, st in step:
            per[st] += e - s
            by_stream[st].append((s, e, n))
        main_st = max(per, key=per.get)
        gaps = []
        kl = by_stream[main_st]
        for (s0, e0, n0), (s1, _, n1) in zip(kl[:-1], kl[1:]):
            if s1 - e0 > a.gap_us * 1e3:
                gaps.append(((s1 - e0) / 1e3, short(n0, 40), short(n1, 40)))
        gaps.sort(reverse=True)
        out.append(f"step wall {(t1 - t0) / 1e6:.3f} ms  busy-union {busy / 1e6:.3f}  idle "
                   f"{(t1 - t0 - busy) / 1e6:.3f}  per-stream kernel ms "
                   f"{ {k: round(v / 1e6, 2) for k, v in sorted(per.items())} }")
        out.append(f"  main stream {main_st}: {len(gaps)} gaps > {a.gap_us} us, total "
                   f"{sum(g for g, _, _ in gaps) / 1e3:.3f} ms; largest (us, after, before):")
        for g in gaps[:6]:
            out.append(f"    {g[0]:8.1f}  {g[1]} -> {g[2]}")
    print("\n".join(out))


if __name__ == "__main__":
    main()
