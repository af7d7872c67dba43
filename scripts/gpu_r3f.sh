#!/bin/bash
# GPU box: full GPU tests + headline bench (LayerNorm backward v2) + wgrad split sweep.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
for v in "RAY_AMD_WGRAD_SPLITS=8" "RAY_AMD_WGRAD_SPLITS=4" "RAY_AMD_WGRAD=lt"; do
  timeout -k 10 300 env $v python bench.py --no-ray > $O/bench_$v.log 2>&1 || { echo "bench $v rc=$?"; tail -20 $O/bench_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/bench_$v.log | cut -c1-160)"
done
timeout -k 10 300 python bench.py --no-ray > $O/bench_noray.log 2>&1 || { echo "bench noray rc=$?"; exit 1; }
echo "default --no-ray: $(tail -1 $O/bench_noray.log | cut -c1-160)"
