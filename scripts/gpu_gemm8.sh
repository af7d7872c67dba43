#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/g8
timeout -k 10 300 python scripts/gemm8_bench.py --variants ${VARIANTS:-4,0} > gpurun_out/g8/bench.log 2>&1; rc=$?
cat gpurun_out/g8/bench.log | grep -v amdgpu.ids; exit $rc
