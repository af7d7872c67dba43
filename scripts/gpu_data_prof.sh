#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/dataprof
mkdir -p $O
timeout -k 10 300 env RAY_AMD_DATA_TRAINER=1 RAY_AMD_DATA_PROFILE=1 python bench.py --workload data --steps 60 --warmup 5 > $O/trainer.log 2>&1 || { echo "rc=$?"; tail -20 $O/trainer.log; exit 1; }
tail -1 $O/trainer.log | cut -c1-160
