#!/bin/bash
# round 5, call AT: attention forward on a 3-waves-per-SIMD register budget (ra_knobs[9] = 2):
# numerics, kernel time, step A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5at
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_attention" > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
tail -2 $O/attn_tests.log
timeout -k 10 120 python scripts/attn_bench.py --B 64 > $O/attn_qb1.log 2>&1 || { tail -5 $O/attn_qb1.log; exit 1; }
RAY_AMD_KNOBS=9=2 timeout -k 10 120 python scripts/attn_bench.py --B 64 > $O/attn_wpe3.log 2>&1 || { tail -5 $O/attn_wpe3.log; exit 1; }
echo "qb1: $(tail -1 $O/attn_qb1.log)"
echo "wpe3: $(tail -1 $O/attn_wpe3.log)"
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() { local n=$1; shift; timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(show $O/$n.log)"; }
run qb1_a RAY_AMD_KNOBS=9=0
run wpe3_a RAY_AMD_KNOBS=9=2
run qb1_b RAY_AMD_KNOBS=9=0
run wpe3_b RAY_AMD_KNOBS=9=2
exit 0
