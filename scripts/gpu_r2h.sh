#!/bin/bash
# GPU box: hipBLASLt fp32-out selector test, LT tuning run (writes profiles/tunableop/
# lt_f32out.csv into gpurun_out), then the bench with the tuned choices vs split-K.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lt_wgrad" -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_lt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_lt.log
if [ $rc -gt 1 ]; then exit $rc; fi
RAY_AMD_LT_TUNE=1 RAY_AMD_LT_FILE="$R/gpurun_out/lt_f32out.csv" timeout -k 10 600 python -u bench.py --no-ray --steps 5 --warmup 3 > gpurun_out/bench_lt_tune.log 2>&1 || exit $?
RAY_AMD_LT_FILE="$R/gpurun_out/lt_f32out.csv" timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_lt.log 2>&1 || exit $?
RAY_AMD_WGRAD=splitk timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_splitk.log 2>&1 || exit $?
echo done
