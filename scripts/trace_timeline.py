"""Per-step GPU timeline from a rocprofv3 kernel trace: busy union vs wall, per-stream busy,
and idle gaps (steps split at the AdamW kernel).

    python scripts/trace_timeline.py gpurun_out/x/prof/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 r["Stream_Id"]) for r in rows))
    ends = [i for i, k in enumerate(ks) if k[2].startswith("void adamw_kernel")]
    for a, b in zip(ends[:-1], ends[1:]):
        step = ks[a + 1:b + 1]
        t0, t1 = step[0][0], max(k[1] for k in step)
        iv = sorted((s, e) for s, e, _, _ in step)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        gaps = []
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                gaps.append((s - ce, s))
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        per = defaultdict(int)
        for s, e, _, st in step:
            per[st] += e - s
        big = sorted(gaps, reverse=True)[:3]
        print(f"step wall {(t1 - t0) / 1e6:.2f} ms  busy {busy / 1e6:.2f}  idle {(t1 - t0 - busy) / 1e6:.2f}"
              f"  n_gaps {len(gaps)}  sum-kernel {sum(e - s for s, e, _, _ in step) / 1e6:.2f}  "
              f"per-stream {dict((k, round(v / 1e6, 2)) for k, v in per.items())}  "
              f"largest gaps us {[round(g / 1e3, 1) for g, _ in big]}")


if __name__ == "__main__":
    main(sys.argv[1])
