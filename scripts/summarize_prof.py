#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats CSV into a markdown table.

    python scripts/summarize_prof.py gpurun_out/prof/run_kernel_stats.csv STEPS [title] > out.md
"""

import csv
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    title = sys.argv[3] if len(sys.argv) > 3 else path
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"Total GPU kernel time per step: **{tot / 1e6 / steps:.3f} ms** "
          f"({steps} profiled steps incl. warmup)\n")
    print("| ms/step | % | calls/step | kernel |")
    print("|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        name = r["Name"].replace("|", "\\|")[:120]
        print(f"| {float(r['TotalDurationNs']) / 1e6 / steps:.3f} | {float(r['Percentage']):.2f} "
              f"| {int(r['Calls']) / steps:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
