#!/bin/bash
# GPU box: LM-head pipeline test + A/B of the GPT-2 step (interleaved runs).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread -k lm_head > gpurun_out/r3c/test.log 2>&1 || { echo "test rc=$?"; tail -30 gpurun_out/r3c/test.log; exit 1; }
tail -1 gpurun_out/r3c/test.log
run() {
  local name=$1; shift
  timeout -k 10 240 env "$@" python bench.py --no-ray --steps 12 --warmup 4 > gpurun_out/r3c/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 gpurun_out/r3c/$name.log; return 1; }
  tail -1 gpurun_out/r3c/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], d['value'])" | tee -a gpurun_out/r3c/sweep.log
}
run pipe1 RAY_AMD_LMHEAD_PIPE=1 && run pipe0 RAY_AMD_LMHEAD_PIPE=0 && run pipe1b RAY_AMD_LMHEAD_PIPE=1 && run pipe0b RAY_AMD_LMHEAD_PIPE=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r3c/prof" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 > "$R/gpurun_out/r3c/prof.log" 2>&1
echo "prof rc=$?"
