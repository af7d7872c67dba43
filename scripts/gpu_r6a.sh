#!/bin/bash
# round 6, call A: hipBLASLt GELU epilogue probe (support + speed at the GPT-2 MLP shapes)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python -u scripts/lt_epilogue_probe.py > $O/probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -40 $O/probe.log
exit $rc
