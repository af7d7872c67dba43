#!/bin/bash
# GPU box: LayerNorm backward v2 tests + bench + kernel-only trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/ln
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layernorm or layer_norm or flat_direct" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python scripts/ln_bwd_bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
cat $O/bench.log | grep -v amdgpu.ids
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/scripts/ln_bwd_bench.py" > "$R/$O/prof.log" 2>&1
echo "prof rc=$?"
