#!/bin/bash
# GPU box: CPU-bound workload benches with / without the session-2 runtime features
# (log dedup, unhandled-error reporting) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/abwl
mkdir -p $O
for cfg in "X=1" "RAY_DEDUP_LOGS=0 RAY_IGNORE_UNHANDLED_ERRORS=1" "X=2"; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python bench.py --workload impala --steps 5 --warmup 2 > $O/impala_$tag.log 2>&1 || { echo "impala rc=$?"; exit 1; }
  echo "impala [$cfg]: $(tail -1 $O/impala_$tag.log | grep -o '"value": [0-9.]*')"
  env $cfg timeout -k 10 300 python bench.py --workload data --steps 60 --warmup 5 > $O/data_$tag.log 2>&1 || { echo "data rc=$?"; exit 1; }
  echo "data [$cfg]: $(tail -1 $O/data_$tag.log | grep -o '"value": [0-9.]*')"
done
