#!/bin/bash
# round 5, call T: LM-head chunking again, spaced 35 s apart (r5k ran inside the post-
# process slow window): one chunk vs 2 / 4 chunks on the two-stream pipelined path
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5t
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
for ch in 65536 32768 16384 32768 65536; do
  timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 --lm-head-chunk $ch > $O/bench_$ch.log 2>&1 || { echo "bench $ch rc=$?"; tail -20 $O/bench_$ch.log; exit 1; }
  echo "chunk=$ch: $(ms $O/bench_$ch.log)"
  sleep 35
done
exit 0
