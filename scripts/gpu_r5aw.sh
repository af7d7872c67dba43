#!/bin/bash
# round 5, call AW: PPO throughput spread (r5av 28.1k vs r5n 33.6k): repeats, plus the
# separate epoll thread (RAY_AMD_IO_THREAD=1) and no task pipelining as checks
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5aw
mkdir -p $O
run() { local n=$1; shift; timeout -k 10 400 env "$@" python bench.py --workload ppo > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n: $(tail -1 $O/$n.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])') load=$(cut -d' ' -f1 /proc/loadavg)"; }
run default_a RAY_AMD_X=0
run io_thread RAY_AMD_IO_THREAD=1
run no_pipeline RAY_AMD_PIPELINE_DEPTH=1
run default_b RAY_AMD_X=0
exit 0
