#!/bin/bash
# GPU box: world-2 GPU paths on one device (TorchTrainer + RLlib learners over gloo).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_rllib_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "two_workers or two_gpu_learners or one_gpu" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log | tail -8
