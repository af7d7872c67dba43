#!/bin/bash
# round 5, call AK: LM head in 2 chunks, cross-entropy on its own stream beside the GEMMs and
# dW_i on the wgrad side stream (pipelined form) vs the single chunk
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5ak
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_gpu.py -k "lm_head" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("final_loss"))'; }
run() { local n=$1; shift; timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run one_a
run two_a --lm-head-chunk 32768
run four_a --lm-head-chunk 16384
run one_b
run two_b --lm-head-chunk 32768
run four_b --lm-head-chunk 16384
exit 0
