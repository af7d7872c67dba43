#!/bin/bash
# round 5, call S: r5o's stream-K grid A/B again, with 35 s between processes (outside the
# post-process slow window, profiles/r5/r5p) and the autotune off so each arm runs the
# mode it names
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5s
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() {  # name env...
  local n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(ms $O/bench_$n.log) load=$(cut -d' ' -f1 /proc/loadavg)"
  sleep 35
}
run base_a X=1
run dp TENSILE_STREAMK_DATA_PARALLEL=1
run gm2 TENSILE_STREAMK_GRID_MULTIPLIER=2
run maxcu224 TENSILE_STREAMK_MAX_CUS=224
run perlin_inkernel RAY_AMD_WGRAD_GROUP=1 RAY_AMD_WGRAD_GROUP_TILES=1
run fill05 RAY_AMD_WGRAD_FILL=0.5
run serial RAY_AMD_WGRAD_STREAM=0
run base_b X=1
exit 0
