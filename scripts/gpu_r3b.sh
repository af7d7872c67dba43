#!/bin/bash
# GPU box: GPT-2 step sweep over wgrad partial caps, attention-bwd mode, LM-head chunk.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
cp profiles/tunableop/lt_f32out.csv gpurun_out/r3b/lt_f32out.csv
export RAY_AMD_LT_FILE=$R/gpurun_out/r3b/lt_f32out.csv
run() {  # name, env..., -- args
  local name=$1; shift
  echo "== $name" >> gpurun_out/r3b/sweep.log
  timeout -k 10 240 env "$@" python bench.py --no-ray --steps 10 --warmup 4 > gpurun_out/r3b/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -5 gpurun_out/r3b/$name.log; return 1; }
  tail -1 gpurun_out/r3b/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'], d['value'])" | tee -a gpurun_out/r3b/sweep.log
}
run tune64 RAY_AMD_LT_TUNE=1 RAY_AMD_WGRAD_PART_MB=64 &&
run tune32 RAY_AMD_LT_TUNE=1 RAY_AMD_WGRAD_PART_MB=32 &&
run base RAY_AMD_WGRAD_PART_MB=4096 &&
run p64 RAY_AMD_WGRAD_PART_MB=64 &&
run p32 RAY_AMD_WGRAD_PART_MB=32 &&
run p16 RAY_AMD_LT_TUNE=1 RAY_AMD_WGRAD_PART_MB=16 &&
run base_b RAY_AMD_WGRAD_PART_MB=4096 &&
run p64_split2 RAY_AMD_WGRAD_PART_MB=64 RAY_AMD_ATTN_BWD=split2 &&
run p64_nostream RAY_AMD_WGRAD_PART_MB=64 RAY_AMD_WGRAD_STREAM=0 &&
run p64_b RAY_AMD_WGRAD_PART_MB=64
