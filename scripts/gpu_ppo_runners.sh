#!/bin/bash
# GPU box: PPO throughput with CPU vs fractional-GPU env-runner inference, sync vs async.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ppo
for cfg in "0 0" "0 1" "0.125 0" "0.125 1"; do
  set -- $cfg
  RAY_AMD_RUNNER_GPUS=$1 RAY_AMD_PPO_ASYNC=$2 timeout -k 10 240 python bench.py --workload ppo --steps 6 --warmup 2 > gpurun_out/ppo/g$1_a$2.log 2>&1 || { echo "ppo g$1 a$2 failed rc=$?"; exit 1; }
  echo "g$1 a$2: $(tail -1 gpurun_out/ppo/g$1_a$2.log | cut -c1-200)"
done
