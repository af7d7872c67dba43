#!/bin/bash
# GPU box: new xent kernel + split-K 16 checks, TunableOp GEMM tuning, benches.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py tests/test_kernels_gpu.py -q -m gpu -k "lm_head or splitk or flat or gpt2" --timeout 120 --timeout-method thread > gpurun_out/t_c.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_c.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/r2_perf_bench.py --part xent,lmhead > gpurun_out/r2_perf_c.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-ray --tunableop off --steps 20 --warmup 5 > gpurun_out/bench_off.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py --no-ray --tunableop tune --steps 3 --warmup 2 > gpurun_out/bench_tune.log 2>&1 || exit $?
cp profiles/tunableop/*.csv gpurun_out/ 2>/dev/null
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_ray_tuned.log 2>&1 || exit $?
echo done
