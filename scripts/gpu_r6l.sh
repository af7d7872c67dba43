#!/bin/bash
# round 6, call L: validation near the end of round 6 (tracing hooks in the core worker, module work): full GPU suite,
# smoke, default bench, and the PPO bench with its new default (in-process policy server)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_default.log; exit 1; }
echo "default: $(ms $O/bench_default.log)"
timeout -k 10 400 python bench.py --workload ppo > $O/ppo_default.log 2>&1 || { echo "ppo rc=$?"; tail -20 $O/ppo_default.log; exit 1; }
echo "ppo default: $(tail -1 $O/ppo_default.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["env_runner_inference"], d["config"]["sample_async"])') load=$(cut -d' ' -f1 /proc/loadavg)"
timeout -k 10 400 python bench.py --workload impala > $O/impala.log 2>&1 || { echo "impala rc=$?"; tail -20 $O/impala.log; exit 1; }
echo "impala: $(tail -1 $O/impala.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
exit 0
