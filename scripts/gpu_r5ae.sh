#!/bin/bash
# round 5, call AE: delta folded into the dQ kernel (no pre-pass): numerics + step time
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5ae
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_attention" > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
tail -2 $O/attn_tests.log
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("wgrad_stream_autotune"))'; }
run() { local n=$1; shift; timeout -k 10 400 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || exit 1; echo "$n: $(show $O/$n.log)"; }
run fold_a RAY_AMD_STREAM_AUTOTUNE=0
run pre_a RAY_AMD_STREAM_AUTOTUNE=0 RAY_AMD_KNOBS=13=1
run fold_b RAY_AMD_STREAM_AUTOTUNE=0
run pre_b RAY_AMD_STREAM_AUTOTUNE=0 RAY_AMD_KNOBS=13=1
mkdir -p $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-ray --steps 13 --warmup 3 > $O/prof.log 2>&1 || exit 1
echo prof done
exit 0
