#!/bin/bash
# round 5, call AP: weight-gradient kernel with a four-stage 32-token LDS ring (three stages
# in flight; ra_knobs[15] = 1): numerics, then step A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5ap
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad_kernel" > $O/wgrad_tests.log 2>&1 || { tail -30 $O/wgrad_tests.log; exit 1; }
tail -2 $O/wgrad_tests.log
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("final_loss"))'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run two_a RAY_AMD_KNOBS=15=0
run deep_a RAY_AMD_KNOBS=15=1
run two_b RAY_AMD_KNOBS=15=0
run deep_b RAY_AMD_KNOBS=15=1
mkdir -p $O/prof
RAY_AMD_KNOBS=15=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-ray --steps 13 --warmup 3 > $O/prof.log 2>&1 || exit 1
echo prof done
exit 0
