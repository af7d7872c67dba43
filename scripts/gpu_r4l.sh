#!/bin/bash
# round 4, call L: dK/dV ILP variant as default — full GPU suite, smoke,
# the driver's default bench twice, no-ray and hooks-always steps
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_default_$i.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench_default_$i.log; exit 1; }
  echo "default $i: $(ms $O/bench_default_$i.log)"
done
for i in 1 2 3; do
  for k in 2 0; do
    timeout -k 10 300 env RAY_AMD_KNOBS=11=$k python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_noray_k${k}_$i.log 2>&1 || { echo "noray rc=$?"; exit 1; }
    echo "no-ray dkdv knob=$k $i: $(ms $O/bench_noray_k${k}_$i.log)"
  done
done
timeout -k 10 300 python bench.py --no-ray --ddp-hooks always --steps 30 --warmup 5 > $O/bench_hooks.log 2>&1 || { echo "hooks rc=$?"; exit 1; }
echo "hooks always: $(ms $O/bench_hooks.log)"
exit 0
