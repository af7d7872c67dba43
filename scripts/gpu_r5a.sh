#!/bin/bash
# round 5, call A: baseline health check on a fresh box — GPU suite, smoke, default bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench_default.log; exit 1; }
echo "default: $(ms $O/bench_default.log)"
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_noray.log 2>&1 || { echo "noray rc=$?"; exit 1; }
echo "no-ray: $(ms $O/bench_noray.log)"
exit 0
