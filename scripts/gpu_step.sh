#!/bin/bash
# all GPU kernel tests, then bench at micro-batch 16/32/64 and a rocprof of mb16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/prof
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x > gpurun_out/kt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/kt.log
if [ $rc -ne 0 ]; then exit $rc; fi
for mb in 16 32 64; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --micro-batch $mb > gpurun_out/bench_mb$mb.log 2>&1 || exit $?
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
