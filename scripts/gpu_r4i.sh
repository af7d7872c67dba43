#!/bin/bash
# round 4, call I: kernel + train GPU tests (incl. the LDS transpose), the GPT-2 step with
# the new transpose (dgrad-wt on) vs dgrad-wt off, interleaved; TorchTrainer; kernel-stats
# profile of the new default; kernel trace of the hooks-always step (timeline)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
for i in 1 2 3; do
  for wt in 1 0; do
    timeout -k 10 300 env RAY_AMD_DGRAD_WT=$wt python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_wt${wt}_$i.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench_wt${wt}_$i.log; exit 1; }
    echo "dgrad-wt=$wt $i: $(ms $O/bench_wt${wt}_$i.log)"
  done
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $O/bench_tt_$i.log 2>&1 || { echo "bench tt rc=$?"; tail -30 $O/bench_tt_$i.log; exit 1; }
  echo "tt $i: $(ms $O/bench_tt_$i.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_hooks -o run -- python bench.py --no-ray --ddp-hooks always --steps 10 --warmup 3 > $O/prof_hooks.log 2>&1 || { echo "prof hooks rc=$?"; tail -20 $O/prof_hooks.log; exit 1; }
echo "profiles done"
exit 0
