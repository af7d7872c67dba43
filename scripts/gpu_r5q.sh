#!/bin/bash
# round 5, call Q: duration of the post-process slow state and whether a cross-stream
# latency probe sees it
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5q
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
timeout -k 10 120 python scripts/stream_probe.py --duration 4 > $O/probe_0.log 2>&1 || exit 1
echo "probe before any bench:"; cat $O/probe_0.log
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_1.log 2>&1 || exit 1
echo "bench 1: $(ms $O/bench_1.log)"
timeout -k 10 120 python scripts/stream_probe.py --duration 50 --every 2 > $O/probe_1.log 2>&1 || exit 1
echo "probe after bench 1:"; cat $O/probe_1.log
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_2.log 2>&1 || exit 1
echo "bench 2 (after the probe window): $(ms $O/bench_2.log)"
exit 0
