#!/bin/bash
# round 6, call E: solo memory-bound passes at the bench shapes; LM-head token-chunk sweep
# (logits chunk resident in the Infinity Cache between GEMM -> cross-entropy -> dh GEMM,
# one side-stream dW over all tokens)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread -k "side_stream or bench_path" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python scripts/membound_bench.py > $O/membound.log 2>&1 || { echo "membound rc=$?"; tail -5 $O/membound.log; exit 1; }
cat $O/membound.log | grep pass
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
i=0
for c in 65536 8192 4096 2048 65536; do
  i=$((i+1)); f=$O/chunk_${i}_$c.log
  timeout -k 10 300 python bench.py --no-ray --steps 20 --warmup 5 --lm-head-chunk $c > $f 2>&1 || { echo "chunk $c rc=$?"; tail -5 $f; exit 1; }
  echo "chunk $c: $(ms $f)"
done
exit 0
