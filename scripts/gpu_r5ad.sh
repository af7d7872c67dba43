#!/bin/bash
# round 5, call AD: host run-ahead bound (RAY_AMD_RUN_AHEAD) vs the allocator growth of the
# side-stream step; back-to-back processes to see whether the next one still starts slow
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5ad
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("hbm"), d.get("wgrad_stream_autotune"))'; }
run() { local n=$1; shift; timeout -k 10 400 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || exit 1; echo "$n: $(show $O/$n.log)"; }
run bound1_a RAY_AMD_STREAM_AUTOTUNE=0
run bound1_b RAY_AMD_STREAM_AUTOTUNE=0
run bound1_c RAY_AMD_STREAM_AUTOTUNE=0
run unbounded RAY_AMD_STREAM_AUTOTUNE=0 RAY_AMD_RUN_AHEAD=0
run after_unbounded RAY_AMD_STREAM_AUTOTUNE=0
run bound2 RAY_AMD_STREAM_AUTOTUNE=0 RAY_AMD_RUN_AHEAD=2
run autotune_default RAY_AMD_RUN_AHEAD=1
exit 0
