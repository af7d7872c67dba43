#!/bin/bash
# GPU box: rocprofv3 kernel stats of the bare GPT-2 step (BENCH_ARGS appended).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/prof2"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof2" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 ${BENCH_ARGS} > "$R/gpurun_out/prof2.log" 2>&1
echo "prof rc=$?" >> "$R/gpurun_out/prof2.log"
