#!/bin/bash
# round 5, call AV: closing runs of the other bench workloads (PPO, IMPALA, Data ingest,
# all-reduce) on the final tree
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5av
mkdir -p $O
for w in ppo impala data allreduce; do
  timeout -k 10 400 python bench.py --workload $w > $O/bench_$w.log 2>&1 || { echo "$w rc=$?"; tail -20 $O/bench_$w.log; exit 1; }
  echo "$w: $(tail -1 $O/bench_$w.log | cut -c1-240)"
done
exit 0
