#!/bin/bash
# round 5, call D: W^T refreshed inside AdamW — tests, step A/B (flat W^T views vs the old
# per-weight side-stream transposes), kernel stats
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 $O/tests.log
[ $rc -eq 0 ] || exit 1
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_wt_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_wt_$i.log; exit 1; }
  echo "flat W^T $i: $(ms $O/bench_wt_$i.log)"
  timeout -k 10 300 env RAY_AMD_FLAT_WT=0 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_nowt_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_nowt_$i.log; exit 1; }
  echo "side-stream transposes $i: $(ms $O/bench_nowt_$i.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*.csv" -size +20M -delete
exit 0
