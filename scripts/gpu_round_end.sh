#!/bin/bash
# GPU box: round-end rehearsal — GPU tests, smoke, headline bench, IMPALA + Data benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/re
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/re/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/re/gpu_tests.log; exit 1; }
tail -1 gpurun_out/re/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/re/smoke.log; exit 1; }
tail -1 gpurun_out/re/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/re/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/re/bench.log; exit 1; }
tail -1 gpurun_out/re/bench.log | cut -c1-250
timeout -k 10 300 python bench.py --workload impala --steps 5 --warmup 2 > gpurun_out/re/impala.log 2>&1 || { echo "impala rc=$?"; exit 1; }
tail -1 gpurun_out/re/impala.log | cut -c1-200
timeout -k 10 300 python bench.py --workload data --steps 60 --warmup 5 > gpurun_out/re/data.log 2>&1 || { echo "data rc=$?"; exit 1; }
tail -1 gpurun_out/re/data.log | cut -c1-200
