#!/bin/bash
# GPU box, round 3 start: GPU tests, headline bench, kernel stats of the bare step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3d/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/r3d/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3d/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r3d/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/r3d/bench.log; exit 1; }
tail -1 gpurun_out/r3d/bench.log | cut -c1-300
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r3d/prof" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 > "$R/gpurun_out/r3d/prof.log" 2>&1
echo "prof rc=$?"
