#!/bin/bash
# round 5, call AM: LM-head dW on the side stream vs the main stream, re-measured after the
# round's other changes (the r5ae timeline shows the side-stream dW holding every CU for 4.9 ms)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5am
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run side_a RAY_AMD_LMHEAD_DW_SIDE=1
run main_a RAY_AMD_LMHEAD_DW_SIDE=0
run side_b RAY_AMD_LMHEAD_DW_SIDE=1
run main_b RAY_AMD_LMHEAD_DW_SIDE=0
run side_c RAY_AMD_LMHEAD_DW_SIDE=1
run main_c RAY_AMD_LMHEAD_DW_SIDE=0
exit 0
