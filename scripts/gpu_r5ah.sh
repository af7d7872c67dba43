#!/bin/bash
# round 5, call AH: wgrad fill fraction / waves re-measured outside the post-exit slow window
# (r5m's arms were all inside it); the wgrad and hipBLASLt GEMM workgroups (131 / 133 KB LDS)
# can never share a CU, so the fill decides how the chip is split while both run
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5ah
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run base RAY_AMD_X=0
run fill075 RAY_AMD_WGRAD_FILL=0.75
run fill05 RAY_AMD_WGRAD_FILL=0.5
run waves2 RAY_AMD_WGRAD_WAVES=2
run fill05_waves2 RAY_AMD_WGRAD_FILL=0.5 RAY_AMD_WGRAD_WAVES=2
run base2 RAY_AMD_X=0
exit 0
