#!/bin/bash
# round 5, call X: characterise the post-exit slow window with a two-stream probe
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 120 python scripts/stream_probe2.py > $O/probe_cold.log 2>&1 || exit 1
echo "cold:"; head -3 $O/probe_cold.log; tail -2 $O/probe_cold.log
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_1.log 2>&1 || exit 1
echo "bench: $(tail -1 $O/bench_1.log | cut -c1-160)"
timeout -k 10 120 python scripts/stream_probe2.py > $O/probe_after.log 2>&1 || exit 1
echo "after bench exit:"; cat $O/probe_after.log
exit 0
