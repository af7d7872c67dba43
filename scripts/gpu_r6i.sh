#!/bin/bash
# round 6, call I: PPO with the in-process policy server (local learner) vs CPU inference,
# sync and async; GPU runner tests incl. the server in both forms
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rllib_gpu_runner.py -x -v --timeout 200 --timeout-method thread > $O/gpu_runner.log 2>&1 || { echo "gpu_runner rc=$?"; tail -30 $O/gpu_runner.log; exit 1; }
tail -2 $O/gpu_runner.log
run() { local n=$1; shift; timeout -k 10 400 env "$@" python bench.py --workload ppo > $O/$n.log 2>&1 || { echo "$n failed"; tail -8 $O/$n.log; exit 1; }; echo "$n: $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["learner"].get("sample_time_s"), d["learner"].get("sample_wait_s"), d["learner"].get("learn_time_s"))') load=$(cut -d' ' -f1 /proc/loadavg)"; }
run srv_async RAY_AMD_POLICY_SERVER_GPUS=0.5 RAY_AMD_PPO_ASYNC=1
run srv_sync RAY_AMD_POLICY_SERVER_GPUS=0.5
run cpu_async RAY_AMD_PPO_ASYNC=1
run srv_async_b RAY_AMD_POLICY_SERVER_GPUS=0.5 RAY_AMD_PPO_ASYNC=1
exit 0
