#!/bin/bash
# GPU box: GPT-2 step tests, TorchTrainer bench, kernel trace (deferred LM-head dW).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=$R/gpurun_out/r3s3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 > "$O/prof.log" 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
cd "$R"
python scripts/summarize_prof.py $O/prof/run_kernel_stats.csv 8 "GPT-2 small mb64, one-chunk LM head, deferred dW" > $O/summary.md
python scripts/trace_timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt 2>&1
tail -4 $O/timeline.txt
