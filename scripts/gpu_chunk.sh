#!/bin/bash
# GPU box: LM-head chunk-size sweep (bench.py --no-ray), new GEMM shapes tuned on first use.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/chunk
mkdir -p $O
for c in 8192 16384 32768 65536; do
  timeout -k 10 600 python bench.py --no-ray --steps 20 --warmup 6 --lm-head-chunk $c --tunableop tune > $O/tune_c$c.log 2>&1 || { echo "c$c rc=$?"; tail -20 $O/tune_c$c.log; exit 1; }
  echo "tune c$c: $(grep -o '"ms_per_step": [0-9.]*' $O/tune_c$c.log)"
done
cp profiles/tunableop/*.csv $O/
for c in 8192 16384 32768 65536; do
  timeout -k 10 300 python bench.py --no-ray --steps 20 --warmup 5 --lm-head-chunk $c > $O/c$c.log 2>&1 || { echo "c$c rc=$?"; exit 1; }
  echo "c$c: $(grep -o '"ms_per_step": [0-9.]*' $O/c$c.log)"
done
