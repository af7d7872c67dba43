#!/bin/bash
# round 5, call U: fused embedding backward (numerics + step), autotune sanity, profile
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "embedding or flat or autotune or lm_head" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
sleep 30
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("wgrad_stream_autotune"))'; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$i.log 2>&1 || { echo "rc=$?"; tail -5 $O/bench_$i.log; exit 1; }
  echo "bench $i: $(show $O/bench_$i.log)"
  sleep 35
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 5 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
echo "profiled: $(show $O/prof.log)"
find $O/prof -name "*.csv" -size +20M -delete
exit 0
