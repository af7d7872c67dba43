#!/bin/bash
# round 5, call AJ: dK/dV kernel with row constants in registers (32 KB LDS, fits beside a
# 128 KB wgrad workgroup): numerics + step A/B against the default ILP variant
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5aj
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_attention" > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
tail -2 $O/attn_tests.log
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run ilp_a RAY_AMD_KNOBS=11=2
run rcg_a RAY_AMD_KNOBS=11=3
run pf1_a RAY_AMD_KNOBS=11=1
run ilp_b RAY_AMD_KNOBS=11=2
run rcg_b RAY_AMD_KNOBS=11=3
run pf1_b RAY_AMD_KNOBS=11=1
mkdir -p $O/prof
RAY_AMD_KNOBS=11=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-ray --steps 13 --warmup 3 > $O/prof.log 2>&1 || exit 1
echo prof done
exit 0
