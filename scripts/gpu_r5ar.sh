#!/bin/bash
# round 5, call AR: c_fc / c_attn weight gradients deferred to the attention backward
# (RAY_AMD_WGRAD_DEFER=1): numerics, then step A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5ar
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_gpu.py -k "deferred or side_stream or flat_fp32" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("final_loss"))'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run now_a RAY_AMD_WGRAD_DEFER=0
run defer_a RAY_AMD_WGRAD_DEFER=1
run now_b RAY_AMD_WGRAD_DEFER=0
run defer_b RAY_AMD_WGRAD_DEFER=1
run defer_rcg RAY_AMD_WGRAD_DEFER=1 RAY_AMD_KNOBS=11=3
run now_c RAY_AMD_WGRAD_DEFER=0
run defer_c RAY_AMD_WGRAD_DEFER=1
exit 0
