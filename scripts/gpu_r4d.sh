#!/bin/bash
# round 4, call D: attention forward variant A/B (v1, v2 family), kernel GPU tests, bench at
# the new defaults, then the two ops/lt-only LM-head hang arms (per-stream vs shared
# workspace; the shared arm is the LAST step: it may hang and is bounded by its watchdog)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 200 python scripts/attn_fwd_ab.py > $O/attn_ab.log 2>&1 || { echo "attn ab rc=$?"; tail -20 $O/attn_ab.log; exit 1; }
tail -1 $O/attn_ab.log
timeout -k 10 200 python scripts/attn_bwd_ab.py > $O/attn_bwd_ab.log 2>&1 || { echo "attn bwd ab rc=$?"; tail -20 $O/attn_bwd_ab.log; exit 1; }
tail -1 $O/attn_bwd_ab.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 $O/gpu_tests.log
case $rc in 0|1) ;; *) exit 1;; esac
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-ray --steps 20 --warmup 5 > $O/bench_noray_$i.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench_noray_$i.log; exit 1; }
  echo "no-ray: $(tail -1 $O/bench_noray_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 300 env RAY_AMD_DATA_TRAINER=1 RAY_AMD_DATA_TIMELINE=$O/data_timeline.json python bench.py --workload data --steps 60 --warmup 5 > $O/data_trainer.log 2>&1 || { echo "data rc=$?"; tail -20 $O/data_trainer.log; exit 1; }
tail -1 $O/data_trainer.log | cut -c1-200
python scripts/data_timeline.py $O/data_timeline.json > $O/data_timeline.txt 2>&1; head -20 $O/data_timeline.txt
timeout -k 10 300 python bench.py --workload data --steps 60 --warmup 5 > $O/data_direct.log 2>&1 || { echo "data direct rc=$?"; tail -20 $O/data_direct.log; exit 1; }
tail -1 $O/data_direct.log | cut -c1-200
timeout -k 10 120 python scripts/lmhead_hang_repro.py 10 40 lt2 > $O/lmhead_lt2.log 2>&1; rc=$?
echo "lt2 rc=$rc: $(tail -1 $O/lmhead_lt2.log)"
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/lmhead_hang_repro.py 10 40 lt2shared > $O/lmhead_lt2shared.log 2>&1; rc=$?
echo "lt2shared rc=$rc: $(tail -1 $O/lmhead_lt2shared.log)"
exit 0
