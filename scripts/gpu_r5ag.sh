#!/bin/bash
# round 5, call AG: disjoint CU sets for the main stream and the weight-gradient side stream
# (hipExtStreamCreateWithCUMask; RAY_AMD_SIDE_CUS / RAY_AMD_MAIN_CUS, ops/cu_mask.py)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5ag
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run base RAY_AMD_X=0
run side64 RAY_AMD_SIDE_CUS=64 RAY_AMD_WGRAD_FILL=0.25
run side64_main192 RAY_AMD_SIDE_CUS=64 RAY_AMD_MAIN_CUS=-192 RAY_AMD_WGRAD_FILL=0.25
run side32_main224 RAY_AMD_SIDE_CUS=32 RAY_AMD_MAIN_CUS=-224 RAY_AMD_WGRAD_FILL=0.125
run side96_main160 RAY_AMD_SIDE_CUS=96 RAY_AMD_MAIN_CUS=-160 RAY_AMD_WGRAD_FILL=0.375
run side64_main192_full RAY_AMD_SIDE_CUS=64 RAY_AMD_MAIN_CUS=-192
run base2 RAY_AMD_X=0
exit 0
