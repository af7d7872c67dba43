#!/bin/bash
# round 5, call AU: attention backward modes in the step (split = dQ with delta, then dK/dV;
# split2 = delta pre-pass, then dQ and dK/dV concurrently on two streams; fused = one pass
# with fp32 dQ atomics), re-measured after this round's changes
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5au
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("final_loss"))'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run split_a RAY_AMD_ATTN_BWD=split
run split2_a RAY_AMD_ATTN_BWD=split2
run fused_a RAY_AMD_ATTN_BWD=fused
run split_b RAY_AMD_ATTN_BWD=split
run split2_b RAY_AMD_ATTN_BWD=split2
run fused_b RAY_AMD_ATTN_BWD=fused
exit 0
