#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/lmh
timeout -k 10 100 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 80 --timeout-method thread -k lm_head > gpurun_out/lmh/pipe0.log 2>&1; echo "pipe0 rc=$?"
tail -3 gpurun_out/lmh/pipe0.log
