#!/bin/bash
# GPU box: interleaved A/B of wgrad split rules on the bare GPT-2 step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/splits3
mkdir -p $O
for rep in 1 2; do
  for v in "X=default" "RAY_AMD_WGRAD_TILES=256" "RAY_AMD_WGRAD_SPLITS=8"; do
    timeout -k 10 300 env $v python bench.py --no-ray > $O/b_${v}_$rep.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/b_${v}_$rep.log; exit 1; }
    echo "$rep $v: $(tail -1 $O/b_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
