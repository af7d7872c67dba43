#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/ln
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/scripts/ln_bwd_bench.py" > "$O/prof.log" 2>&1
echo "prof rc=$?"
grep -v amdgpu.ids $O/prof.log | grep "ms/call"
