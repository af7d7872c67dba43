#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
: > gpurun_out/splits.log
for s in 16 8 4 16 8; do
  echo "splits $s" >> gpurun_out/splits.log
  RAY_AMD_WGRAD_SPLITS=$s timeout -k 10 300 python -u bench.py --no-ray --steps 20 --warmup 5 >> gpurun_out/splits.log 2>&1 || exit $?
done
echo done
