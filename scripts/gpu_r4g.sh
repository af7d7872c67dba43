#!/bin/bash
# round 4, call G: GPU tests, then interleaved A/B arms of the GPT-2 no-ray step
# (base vs transposed-weight dgrad; DDP hooks off vs on at world 1) and the dgrad layout A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_train_predictors.py -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 $O/gpu_tests.log
case $rc in 0|1) ;; *) exit 1;; esac
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])'; }
for i in 1 2 3; do
  for arm in base wt; do
    ex=""; [ $arm = wt ] && ex="RAY_AMD_DGRAD_WT=1"
    timeout -k 10 300 env $ex python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_${arm}_$i.log 2>&1 || { echo "bench $arm rc=$?"; tail -30 $O/bench_${arm}_$i.log; exit 1; }
    echo "$arm $i: $(ms $O/bench_${arm}_$i.log)"
  done
done
for i in 1 2 3; do
  for arm in auto always; do
    timeout -k 10 300 python bench.py --no-ray --ddp-hooks $arm --steps 30 --warmup 5 > $O/bench_hooks_${arm}_$i.log 2>&1 || { echo "bench hooks rc=$?"; tail -30 $O/bench_hooks_${arm}_$i.log; exit 1; }
    echo "hooks $arm $i: $(ms $O/bench_hooks_${arm}_$i.log)"
  done
done
timeout -k 10 300 python scripts/dgrad_layout_ab.py > $O/dgrad_layout.log 2>&1 || { echo "dgrad ab rc=$?"; tail -20 $O/dgrad_layout.log; exit 1; }
tail -2 $O/dgrad_layout.log | cut -c1-600
exit 0
