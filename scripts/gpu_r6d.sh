#!/bin/bash
# round 6, call D: pruned kernels (full GPU suite incl. GPU env-runner tests), smoke,
# default GPT-2 bench; PPO with env-runner inference on CPU vs the MI355X (HIP graph)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rllib_gpu_runner.py -x -v --timeout 120 --timeout-method thread > $O/gpu_runner.log 2>&1 || { echo "gpu_runner rc=$?"; tail -30 $O/gpu_runner.log; exit 1; }
tail -2 $O/gpu_runner.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"), d.get("ranks_in_sync"))'; }
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_default.log; exit 1; }
echo "default: $(ms $O/bench_default.log)"
run() { local n=$1; shift; timeout -k 10 400 env "$@" python bench.py --workload ppo > $O/$n.log 2>&1 || { echo "$n failed"; tail -8 $O/$n.log; exit 1; }; echo "$n: $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["learner"].get("sample_time_s"), d["learner"].get("sample_wait_s"))') load=$(cut -d' ' -f1 /proc/loadavg)"; }
run ppo_gpu_async RAY_AMD_RUNNER_GPUS=0.125 RAY_AMD_PPO_ASYNC=1
run ppo_gpu_sync RAY_AMD_RUNNER_GPUS=0.125
run ppo_cpu_async RAY_AMD_PPO_ASYNC=1
run ppo_cpu_sync RAY_AMD_X=0

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-ray --steps 8 --warmup 3 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof ok"
exit 0
