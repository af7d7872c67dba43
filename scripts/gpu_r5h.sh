#!/bin/bash
# round 5, call H: repeat of the r5g step A/B (erratic timings there) with GPU state
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5h
mkdir -p $O
rocm-smi --showuse --showpower --showclocks --showtemp > $O/smi_before.txt 2>&1 || true
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
run() {  # name env...
  local n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(ms $O/bench_$n.log)"
}
for i in 1 2 3; do
  run side_hip_$i RAY_AMD_LMHEAD_DW=hip
  run main_torch_$i RAY_AMD_LMHEAD_DW=torch RAY_AMD_LMHEAD_DW_SIDE=0
done
rocm-smi --showuse --showpower --showclocks --showtemp > $O/smi_after.txt 2>&1 || true
exit 0
