#!/bin/bash
# GPU box: interleaved A/B of wgrad stream / split knobs with the one-chunk LM head.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ab4
mkdir -p $O
for rep in 1 2; do
  for cfg in "X=default" "RAY_AMD_WGRAD_STREAM=0" "RAY_AMD_WGRAD_SPLITS=8" "RAY_AMD_LMHEAD_PIPE=0"; do
    env $cfg timeout -k 10 200 python bench.py --no-ray --steps 20 --warmup 5 > "$O/${cfg}_$rep.log" 2>&1 || { echo "$cfg rc=$?"; tail -5 "$O/${cfg}_$rep.log"; exit 1; }
    echo "$cfg rep$rep: $(grep -o '"ms_per_step": [0-9.]*' "$O/${cfg}_$rep.log")"
  done
done
