#!/bin/bash
# round 5, call E: grouped wgrad (one launch per layer, in-kernel split-K reduction) —
# numerics, kernel bench, step A/B, kernel stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/wgrad_bench.py --rounds 3 > $O/wgrad_bench.log 2>&1 || { echo "wbench rc=$?"; tail -20 $O/wgrad_bench.log; exit 1; }
grep -E "layer_group|per_layer" $O/wgrad_bench.log
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
for i in 1 2; do
  for g in 1 0; do
    timeout -k 10 300 env RAY_AMD_WGRAD_GROUP=$g python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_g${g}_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_g${g}_$i.log; exit 1; }
    echo "group=$g $i: $(ms $O/bench_g${g}_$i.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*.csv" -size +20M -delete
exit 0
