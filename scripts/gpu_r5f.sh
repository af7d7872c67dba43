#!/bin/bash
# round 5, call F: main/side stream scheduling A/B on the GPT-2 step — per-linear wgrad on
# the side stream (baseline), step on a high-priority stream, shorter-lived wgrad
# workgroups (2 waves), and no side stream at all (serial)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5f
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
run() {  # name env...
  local n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(ms $O/bench_$n.log)"
}
for i in 1 2; do
  run base_$i RAY_AMD_WGRAD_GROUP=0
  run prio_$i RAY_AMD_MAIN_PRIO=1
  run waves2_$i RAY_AMD_WGRAD_WAVES=2
  run prio_waves2_$i RAY_AMD_MAIN_PRIO=1 RAY_AMD_WGRAD_WAVES=2
  run serial_$i RAY_AMD_WGRAD_STREAM=0
done
exit 0
