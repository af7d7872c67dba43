#!/bin/bash
# round 6, call B: wgrad on several side streams with a fixed split count (S = 1: no fp32
# slabs, no accumulate pass) vs the default single side stream with CU-filling split-K
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r6b
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run base RAY_AMD_X=0
run l4s1 RAY_AMD_WGRAD_LANES=4 RAY_AMD_WGRAD_S=1
run l4s2 RAY_AMD_WGRAD_LANES=4 RAY_AMD_WGRAD_S=2
run l2s2 RAY_AMD_WGRAD_LANES=2 RAY_AMD_WGRAD_S=2
run l1s2 RAY_AMD_WGRAD_S=2
run base2 RAY_AMD_X=0
exit 0
