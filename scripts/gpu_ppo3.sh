#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
rm -rf gpurun_out/ppoprof3
timeout -k 10 300 python -u scripts/ppo_learner_bench.py > gpurun_out/ppo_learner3.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/ppoprof3" -o run -- python3 "$R/scripts/ppo_learner_bench.py" --iters 2 --warmup 1 > "$R/gpurun_out/ppoprof3.log" 2>&1 || exit $?
echo done
