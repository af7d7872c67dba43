#!/bin/bash
# round 5, call W: TunableOp GEMM selection. profiles/ stopped being uploaded this round, so
# every r5 bench ran hipBLASLt's heuristic; the tuned files now live in ray_amd/tuned/.
# A/B: heuristic vs the r4 file vs a file re-tuned on the current code (35 s apart).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5w
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["gemm_selection"])'; }
run() {
  local n=$1; shift
  timeout -k 10 900 python bench.py --no-ray "$@" > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(show $O/bench_$n.log)"
  sleep 35
}
run heuristic --steps 30 --warmup 5 --tunableop off
run r4file --steps 30 --warmup 5 --tunableop auto
run tune --steps 5 --warmup 5 --tunableop tune
cp ray_amd/tuned/gpt2_small_mb64_t1024.csv $O/gpt2_small_mb64_t1024.csv
run retuned --steps 30 --warmup 5 --tunableop auto
run heuristic2 --steps 30 --warmup 5 --tunableop off
exit 0
