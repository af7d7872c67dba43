#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/lt_epilogue_probe.py > gpurun_out/ep_probe.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/r2_perf_bench.py --part norm > gpurun_out/norm3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_ln.log 2>&1 || exit $?
echo done
