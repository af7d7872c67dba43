#!/bin/bash
# GPU box: smoke, full gpu test suite, then both benches. Each GPU step has its own time
# limit; a crash/timeout (rc>1 for pytest, any rc for the others) stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_gpt2.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --workload ppo --steps 3 --warmup 1 > gpurun_out/bench_ppo.log 2>&1 || exit $?
echo done
