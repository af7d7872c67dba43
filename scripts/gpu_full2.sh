#!/bin/bash
# Round-end rehearsal: smoke, the whole `pytest -m gpu` suite, the headline bench through
# TorchTrainer, and the other BASELINE workloads (PPO, IMPALA, Data) on one MI355X.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_all.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_ray.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload impala --steps 5 --warmup 2 > gpurun_out/bench_impala.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload data --steps 5 --warmup 2 > gpurun_out/bench_data.log 2>&1 || exit $?
echo done
