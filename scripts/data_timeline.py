"""Where the Data -> TorchTrainer ingest time goes: summarise a task timeline written by
``RAY_AMD_DATA_TIMELINE=<file> RAY_AMD_DATA_TRAINER=1 python bench.py --workload data``
over the trainer's timed window. Per task / actor-method name: calls that overlap the
window, busy seconds inside it, and the average number running at once (busy / window) —
read tasks near the CPU budget mean a producer-bound pipeline; a consumer whose
``next_block`` calls cover the window is waiting on them.

    python scripts/data_timeline.py timeline.json
"""
import collections
import json
import sys


def summarise(doc):
    w0, w1 = doc["window"]
    win = w1 - w0
    agg = collections.defaultdict(lambda: [0, 0.0])
    for ev in doc["trace"]:
        a = ev["ts"] / 1e6
        b = a + ev["dur"] / 1e6
        lo, hi = max(a, w0), min(b, w1)
        if hi <= lo:
            continue
        name = ev["name"].split(".")[-1] if "." in ev["name"] else ev["name"]
        agg[name][0] += 1
        agg[name][1] += hi - lo
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    return win, rows


def main(path):
    doc = json.load(open(path))
    win, rows = summarise(doc)
    print(f"timed window {win:.3f} s, CPU budget {doc.get('cpus')}")
    print(f"{'task / method':48s} {'calls':>6s} {'busy s':>8s} {'avg running':>11s}")
    for name, (n, busy) in rows[:25]:
        print(f"{name[:48]:48s} {n:6d} {busy:8.3f} {busy / win:11.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
