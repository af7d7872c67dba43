#!/bin/bash
# round 6, call F: secondary benchmarks refreshed on this tree — core microbenchmark,
# IMPALA (bf16 CPU inference now actually on), Data GPU ingest, PPO default (sync)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6f
mkdir -p $O
v() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("unit"))'; }
timeout -k 10 400 python bench.py --workload impala > $O/impala.log 2>&1 || { echo "impala rc=$?"; tail -5 $O/impala.log; exit 1; }
echo "impala: $(v $O/impala.log)"
timeout -k 10 400 python bench.py --workload ppo > $O/ppo_sync.log 2>&1 || { echo "ppo rc=$?"; tail -5 $O/ppo_sync.log; exit 1; }
echo "ppo sync: $(v $O/ppo_sync.log)"
timeout -k 10 400 python bench.py --workload data > $O/data.log 2>&1 || { echo "data rc=$?"; tail -5 $O/data.log; exit 1; }
echo "data: $(v $O/data.log)"
timeout -k 10 500 python -m ray_amd._private.ray_perf --json $O/microbench.json > $O/microbench.log 2>&1 || { echo "microbench rc=$?"; tail -5 $O/microbench.log; exit 1; }
tail -25 $O/microbench.log
exit 0
