#!/bin/bash
# round 5, call O: Tensile stream-K grid knobs for the main-stream hipBLASLt GEMMs. The
# persistent SK3 kernels launch one workgroup per CU, so a side-stream wgrad workgroup on a
# CU stalls a whole GEMM slice (r5e: dgrad GEMMs 2-5x slower while overlapped).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5o
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
run() {  # name env...
  local n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(ms $O/bench_$n.log) load=$(cut -d' ' -f1 /proc/loadavg)"
}
run base_a X=1
run dp TENSILE_STREAMK_DATA_PARALLEL=1
run gm2 TENSILE_STREAMK_GRID_MULTIPLIER=2
run maxcu192 TENSILE_STREAMK_MAX_CUS=192
run gm4 TENSILE_STREAMK_GRID_MULTIPLIER=4
run perlin_inkernel RAY_AMD_WGRAD_GROUP=1 RAY_AMD_WGRAD_GROUP_TILES=1
run dp_perlin_inkernel TENSILE_STREAMK_DATA_PARALLEL=1 RAY_AMD_WGRAD_GROUP=1 RAY_AMD_WGRAD_GROUP_TILES=1
run base_b X=1
exit 0
