#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
for k in 1 2 3; do
rm -rf gpurun_out/pa_k$k
cd /tmp && RAY_AMD_ATTN_BWD=fused timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/pa_k$k" -o run -- python3 "$R/scripts/attn_bench.py" --B 64 --knob6 $k > "$R/gpurun_out/pa_k$k.log" 2>&1 || exit $?
done
echo done
