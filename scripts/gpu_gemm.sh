#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench.json 2> gpurun_out/gemm_bench.err || exit $?
