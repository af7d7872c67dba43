#!/bin/bash
# round 6, call H: validation after the API-parity work: full GPU suite, smoke, default
# bench (TorchTrainer), bare-loop bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"), d.get("ranks_in_sync"))'; }
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_default.log; exit 1; }
echo "default: $(ms $O/bench_default.log)"
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_noray.log 2>&1 || { echo "noray rc=$?"; exit 1; }
echo "noray: $(ms $O/bench_noray.log)"
exit 0
