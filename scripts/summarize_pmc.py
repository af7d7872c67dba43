"""Per-kernel PMC summary (markdown) from rocprofv3 `--pmc ... --output-format csv` runs.

    python scripts/summarize_pmc.py gpurun_out/r5al

Reads <dir>/{sq,fetch,write}/**/run_counter_collection.csv. Per kernel name (top by total
time): dispatches, mean duration, and per dispatch
  - MFMA TFLOP/s = SQ_VALU_MFMA_BUSY_CYCLES x 1024 FLOP / duration (bf16 32x32x16 = 32768
    FLOP per 32 busy cycles; 16x16x32 = 16384 per 16),
  - wait / active-instruction / LDS fractions of SQ_WAVE_CYCLES, LDS bank conflicts per
    LDS-active cycle,
  - HBM-side bytes (FETCH_SIZE + WRITE_SIZE, KB units) and the resulting TB/s.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[:60]


def main():
    base = sys.argv[1]
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values]
    dur = defaultdict(dict)  # kernel -> dispatch -> ns
    for sub in ("sq", "fetch", "write"):
        for r in load(os.path.join(base, sub)):
            k = short(r.get("Kernel_Name", ""))
            did = r.get("Dispatch_Id")
            try:
                ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            except (KeyError, ValueError):
                ns = 0
            if sub == "sq" and ns:
                dur[k][did] = ns
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    tot = {k: sum(v.values()) for k, v in dur.items()}
    print("| kernel | disp. | mean µs | MFMA TF/s | WAIT_ANY | ACTIVE_INST | ACTIVE_LDS | "
          "bank confl./LDS | HBM GB/disp. | TB/s |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in sorted(tot, key=lambda x: -tot[x])[:16]:
        c = per[k]
        n = len(dur[k])
        mean_ns = tot[k] / max(1, n)

        def avg(name):
            v = c.get(name)
            return sum(v) / len(v) if v else None

        wave = avg("SQ_WAVE_CYCLES") or 0
        mfma = avg("SQ_VALU_MFMA_BUSY_CYCLES")
        tf = mfma * 1024 / (mean_ns * 1e-9) / 1e12 if mfma and mean_ns else None
        f = lambda x: f"{x:.3f}" if x is not None else "–"  # noqa: E731
        fr = lambda name: f(avg(name) / wave) if wave and avg(name) is not None else "–"  # noqa
        lds = avg("SQ_ACTIVE_INST_LDS")
        bc = avg("SQ_LDS_BANK_CONFLICT")
        fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
        gb = ((fetch or 0) + (write or 0)) * 1024 / 1e9 if fetch is not None else None
        tbs = gb / (mean_ns * 1e-9) / 1e3 if gb is not None and mean_ns else None
        print(f"| `{k}` | {n} | {mean_ns / 1e3:.1f} | {f(tf) if tf else '–'} | "
              f"{fr('SQ_WAIT_ANY')} | {fr('SQ_ACTIVE_INST_ANY')} | {fr('SQ_ACTIVE_INST_LDS')} | "
              f"{f(bc / lds) if bc is not None and lds else '–'} | {f(gb) if gb is not None else '–'} | "
              f"{f(tbs) if tbs is not None else '–'} |")


if __name__ == "__main__":
    main()
