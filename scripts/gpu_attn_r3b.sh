#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
O="$R/gpurun_out/attn3b"
mkdir -p "$O"
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "attn or attention" > "$O/test.log" 2>&1 || { echo "test rc=$?"; tail -30 "$O/test.log"; exit 1; }
tail -1 "$O/test.log"
timeout -k 10 120 python3 scripts/attn_bench3.py > "$O/bench.log" 2>&1 || { echo "bench rc=$?"; tail "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
