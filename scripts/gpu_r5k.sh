#!/bin/bash
# round 5, call K: LM-head chunk size A/B (65536 = one chunk, dW on the side stream; smaller
# chunks = the two-stream pipelined path, logits chunks that fit the 256 MB Infinity Cache)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5k
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
for i in 1 2; do
  for ch in 65536 16384 8192 4096; do
    timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 --lm-head-chunk $ch > $O/bench_${ch}_$i.log 2>&1 || { echo "bench $ch rc=$?"; tail -20 $O/bench_${ch}_$i.log; exit 1; }
    echo "chunk=$ch $i: $(ms $O/bench_${ch}_$i.log) load=$(cut -d' ' -f1 /proc/loadavg)"
  done
done
exit 0
