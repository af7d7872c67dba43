"""Summarise a rocprofv3 SQLite output (``*_results.db``) as a markdown kernel table.

    python scripts/rocpd_summary.py gpurun_out/prof_x [--top 25] [--title "..."]
"""

import argparse
import glob
import os
import re
import sqlite3


def summarize(path, top=25):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) \
        else [path]
    rows = {}
    for f in dbs:
        c = sqlite3.connect(f)
        q = ("select s.kernel_name, count(*), sum(d.end - d.start), s.arch_vgpr_count, "
             "s.accum_vgpr_count, s.group_segment_size from rocpd_kernel_dispatch d join "
             "rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name")
        for name, n, ns, vg, ag, lds in c.execute(q):
            r = rows.setdefault(name, [0, 0, vg, ag, lds])
            r[0] += n
            r[1] += ns
    total = sum(r[1] for r in rows.values()) or 1
    out = ["| kernel | calls | total ms | avg us | % | VGPR | AGPR | LDS |",
           "|---|---:|---:|---:|---:|---:|---:|---:|"]
    for name, (n, ns, vg, ag, lds) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:top]:
        short = re.sub(r"\.kd$", "", name)
        if len(short) > 90:
            short = short[:87] + "..."
        out.append(f"| `{short}` | {n} | {ns / 1e6:.3f} | {ns / n / 1e3:.2f} | "
                   f"{100 * ns / total:.1f} | {vg} | {ag} | {lds} |")
    out.append(f"\nTotal kernel time: {total / 1e6:.3f} ms over {sum(r[0] for r in rows.values())}"
               " dispatches")
    return "\n".join(out)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default=None)
    a = ap.parse_args()
    if a.title:
        print(f"# {a.title}\n")
    print(summarize(a.path, a.top))
