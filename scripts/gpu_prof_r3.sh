#!/bin/bash
# GPU box: kernel trace of the bare GPT-2 step (current kernels).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof3
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 > "$O/prof.log" 2>&1
echo "prof rc=$?"
tail -1 $O/prof.log | cut -c1-200
