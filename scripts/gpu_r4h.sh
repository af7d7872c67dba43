#!/bin/bash
# round 4, call H: the full GPU test suite, TorchTrainer with the default vs a 50 ms
# dispatcher poll (interleaved), the driver's default bench, and a kernel-stats profile
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
for i in 1 2; do
  for p in 10 50; do
    timeout -k 10 300 env RAY_AMD_POLL_MS=$p python bench.py --steps 30 --warmup 5 > $O/bench_tt_poll${p}_$i.log 2>&1 || { echo "bench tt rc=$?"; tail -30 $O/bench_tt_poll${p}_$i.log; exit 1; }
    echo "tt poll $p $i: $(ms $O/bench_tt_poll${p}_$i.log)"
  done
done
for i in 1 2; do
  for arm in auto:32 always:32 always:64; do
    h=${arm%%:*}; mb=${arm##*:}
    timeout -k 10 300 python bench.py --no-ray --ddp-hooks $h --bucket-mb $mb --steps 30 --warmup 5 > $O/bench_hooks_${h}_${mb}_$i.log 2>&1 || { echo "bench hooks rc=$?"; tail -30 $O/bench_hooks_${h}_${mb}_$i.log; exit 1; }
    echo "hooks $h bucket $mb $i: $(ms $O/bench_hooks_${h}_${mb}_$i.log)"
  done
done
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "bench default rc=$?"; tail -30 $O/bench_default.log; exit 1; }
echo "default: $(ms $O/bench_default.log)"
for pin in 0 1; do
  timeout -k 10 400 env RAY_AMD_DATA_GPU_ACTORS=2 RAY_AMD_DATA_PIN_STORE=$pin RAY_AMD_DATA_TRAINER=1 python bench.py --workload data --steps 300 --warmup 20 > $O/data_trainer_a2_pin$pin.log 2>&1 || { echo "data rc=$?"; tail -20 $O/data_trainer_a2_pin$pin.log; exit 1; }
  echo "data trainer a2 pin=$pin: $(ms $O/data_trainer_a2_pin$pin.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
exit 0
