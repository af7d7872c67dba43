#!/bin/bash
# round 5, call Z: is the back-to-back slow state a hardware-queue effect? The bench uses 8
# HIP hardware queues per process; try 2 right after an 8-queue process, and back to back
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5z
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
run() { local n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || exit 1
  echo "$n: $(ms $O/bench_$n.log)"; }
run a_q8 RAY_AMD_HW_QUEUES=8
run b_q2 RAY_AMD_HW_QUEUES=2
run c_q2 RAY_AMD_HW_QUEUES=2
run d_q2 RAY_AMD_HW_QUEUES=2
sleep 35
run e_q8 RAY_AMD_HW_QUEUES=8
run f_q8 RAY_AMD_HW_QUEUES=8
exit 0
