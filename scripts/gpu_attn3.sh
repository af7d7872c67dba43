#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
rm -rf gpurun_out/pa_fused gpurun_out/pa_split
cd /tmp && RAY_AMD_ATTN_BWD=fused timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/pa_fused" -o run -- python3 "$R/scripts/attn_bench.py" --B 64 > "$R/gpurun_out/pa_fused.log" 2>&1 || exit $?
cd /tmp && RAY_AMD_ATTN_BWD=split timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/pa_split" -o run -- python3 "$R/scripts/attn_bench.py" --B 64 > "$R/gpurun_out/pa_split.log" 2>&1 || exit $?
echo done
