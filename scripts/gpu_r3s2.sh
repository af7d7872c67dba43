#!/bin/bash
# GPU box: TorchTrainer bench with the one-chunk LM head, then a kernel trace of the step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=$R/gpurun_out/r3s2
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-260
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 > "$O/prof.log" 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-200
cd "$R"
python scripts/summarize_prof.py $(ls $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -1) 8 "GPT-2 small mb64, one-chunk LM head" > $O/summary.md
python scripts/trace_timeline.py $(ls $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv 2>/dev/null | head -1) > $O/timeline.txt 2>&1
head -30 $O/summary.md
cat $O/timeline.txt | tail -5
