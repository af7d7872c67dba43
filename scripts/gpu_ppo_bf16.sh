#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ppo2
for a in 0 1; do
  RAY_AMD_PPO_ASYNC=$a timeout -k 10 240 python bench.py --workload ppo --steps 6 --warmup 2 > gpurun_out/ppo2/a$a.log 2>&1 || { echo "ppo a$a rc=$?"; tail -20 gpurun_out/ppo2/a$a.log; exit 1; }
  tail -1 gpurun_out/ppo2/a$a.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('async', $a, d['value'], d['learner'])"
done
