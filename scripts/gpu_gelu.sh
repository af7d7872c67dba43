#!/bin/bash
# GPU box: GELU backward v2 tests + bench + kernel-only trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/gelu
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gelu or colsum or flat_direct or mlp or linear" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/scripts/gelu_bwd_bench.py" > "$R/$O/prof.log" 2>&1
echo "prof rc=$?"
grep "TB/s" $R/$O/prof.log
