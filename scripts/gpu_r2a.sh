#!/bin/bash
# GPU box (round 2): smoke, training GPU tests + kernel tests, the TorchTrainer headline
# bench and its bare-loop twin, then rocprofv3 kernel stats of the bare step.
# Each GPU step has its own time limit; a crash/timeout stops the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_kernels_gpu.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_ray.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_bare.log 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 ${BENCH_ARGS} > "$R/gpurun_out/prof.log" 2>&1
echo "prof rc=$?" >> "$R/gpurun_out/prof.log"
echo done
