#!/bin/bash
# round 6, call C: new bench-shape gradient test, full GPU suite, smoke, default bench
# (TorchTrainer over the memfd object store), bare-loop bench, kernel profile
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 240 --timeout-method thread -k bench_path -s > $O/gradcheck.log 2>&1 || { echo "gradcheck rc=$?"; tail -30 $O/gradcheck.log; exit 1; }
grep -E "max rel|passed|failed" $O/gradcheck.log | tail -3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"), d.get("ranks_in_sync"))'; }
sleep 5
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_default.log; exit 1; }
echo "default: $(ms $O/bench_default.log)"
grep -c "destroy_process_group" $O/bench_default.log || true
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_noray.log 2>&1 || { echo "noray rc=$?"; exit 1; }
echo "noray: $(ms $O/bench_noray.log)"
exit 0
