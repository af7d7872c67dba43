"""Kernel table (markdown) from a rocprofv3 SQLite result (`run_results.db`, the default
output format): ms per step = total kernel time / --steps, calls per step, short names.

    python scripts/summarize_db.py gpurun_out/r5ae/prof/run_results.db --steps 16 --title "..."
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=float, required=True)
    ap.add_argument("--title", default="kernel table")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration) from kernels group by name "
                     "order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows)
    print(f"# {a.title}\n")
    print(f"Total GPU kernel time per step: **{total / 1e6 / a.steps:.3f} ms** "
          f"({a.steps:g} profiled steps)\n")
    print("| ms/step | % | calls/step | kernel |\n|---:|---:|---:|---|")
    for name, n, dur in rows[:a.top]:
        print(f"| {dur / 1e6 / a.steps:.3f} | {100 * dur / total:.2f} | {n / a.steps:.1f} | "
              f"`{name[:120]}` |")


if __name__ == "__main__":
    main()
