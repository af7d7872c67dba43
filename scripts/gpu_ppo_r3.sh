#!/bin/bash
# GPU box: PPO async throughput with 1 vs 2 CPU threads per env runner.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/ppo3
mkdir -p $O
echo "nproc $(nproc) affinity $(python -c 'import os;print(len(os.sched_getaffinity(0)))')"
for c in 1 2; do
  timeout -k 10 300 env RAY_AMD_PPO_ASYNC=1 RAY_AMD_RUNNER_CPUS=$c python bench.py --workload ppo --steps 8 --warmup 2 > $O/ppo_c$c.log 2>&1 || { echo "ppo c$c rc=$?"; tail -20 $O/ppo_c$c.log; exit 1; }
  echo "cpus/runner=$c: $(tail -1 $O/ppo_c$c.log | cut -c1-140)"
done
