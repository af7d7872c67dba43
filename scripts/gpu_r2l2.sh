#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
for m in split split2 split split2; do
RAY_AMD_ATTN_BWD=$m timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 > gpurun_out/bench_$m.log 2>&1 || exit $?
tail -n1 gpurun_out/bench_$m.log | cut -c1-140
done
echo done
