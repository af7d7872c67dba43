#!/bin/bash
# round 5, call G: LM-head dW on the side stream through the hip wgrad kernel (S = 3 at
# 591 tiles) — numerics, step A/B against the main-stream torch.addmm path, kernel stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or lm_head or flat" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 $O/tests.log
[ $rc -eq 0 ] || exit 1
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
run() {  # name env...
  local n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(ms $O/bench_$n.log)"
}
for i in 1 2; do
  run side_hip_$i RAY_AMD_LMHEAD_DW=hip
  run main_hip_$i RAY_AMD_LMHEAD_DW=hip RAY_AMD_LMHEAD_DW_SIDE=0
  run main_torch_$i RAY_AMD_LMHEAD_DW=torch RAY_AMD_LMHEAD_DW_SIDE=0
  run side_lt_$i RAY_AMD_LMHEAD_DW=lt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*.csv" -size +20M -delete
exit 0
