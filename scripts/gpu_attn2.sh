#!/bin/bash
# GPU box: attention numerics + timing, then the full bare bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -k "attention or gpt2 or flat" --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_attn.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u scripts/attn_bench.py --B 64 > gpurun_out/attn_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_attn2.log 2>&1 || exit $?
echo done
