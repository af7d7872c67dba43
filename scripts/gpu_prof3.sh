#!/bin/bash
# GPU box: rocprofv3 kernel trace of the bare GPT-2 step (sqlite output; summarise with
# scripts/rocpd_summary.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
rm -rf gpurun_out/prof3
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof3" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 ${BENCH_ARGS} > "$R/gpurun_out/prof3.log" 2>&1 || exit $?
echo done
