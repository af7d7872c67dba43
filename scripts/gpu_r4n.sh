#!/bin/bash
# round 4, call N: kernel statistics of the final default step (csv, small enough to copy back)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-200
find $O/prof -name "*.csv" -size +20M -delete
find $O/prof -name "*kernel_stats.csv"
exit 0
