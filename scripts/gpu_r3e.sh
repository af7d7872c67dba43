#!/bin/bash
# GPU box: GPU tests + headline bench + data benches (after the store/iterator changes).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 python bench.py --workload data --steps 60 --warmup 5 --data-path h2d > $O/data_h2d.log 2>&1 || { echo "data h2d rc=$?"; tail -20 $O/data_h2d.log; exit 1; }
tail -1 $O/data_h2d.log | cut -c1-200
