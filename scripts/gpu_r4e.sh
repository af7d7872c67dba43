#!/bin/bash
# round 4, call E: GPU tests, attention forward baseline and backward ILP variants, and
# GPT-2 step arms (no-ray x2, TorchTrainer, transposed-weight dgrad, overlapped AdamW,
# wgrad split counts) plus the dgrad layout A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 $O/gpu_tests.log
case $rc in 0|1) ;; *) exit 1;; esac
timeout -k 10 200 python scripts/attn_fwd_ab.py > $O/attn_fwd.log 2>&1 || { echo "attn fwd rc=$?"; tail -20 $O/attn_fwd.log; exit 1; }
tail -1 $O/attn_fwd.log
timeout -k 10 300 python scripts/attn_bwd_ab.py > $O/attn_bwd_ab.log 2>&1 || { echo "attn bwd ab rc=$?"; tail -20 $O/attn_bwd_ab.log; exit 1; }
tail -1 $O/attn_bwd_ab.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-ray --steps 20 --warmup 5 > $O/bench_noray_$i.log 2>&1 || { echo "bench rc=$?"; tail -30 $O/bench_noray_$i.log; exit 1; }
  echo "no-ray: $(tail -1 $O/bench_noray_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 300 python bench.py --no-ray --ddp-hooks always --steps 20 --warmup 5 > $O/bench_noray_hooks.log 2>&1 || { echo "bench hooks rc=$?"; tail -30 $O/bench_noray_hooks.log; exit 1; }
echo "no-ray ddp-hooks always: $(tail -1 $O/bench_noray_hooks.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_tt.log 2>&1 || { echo "bench tt rc=$?"; tail -30 $O/bench_tt.log; exit 1; }
echo "torchtrainer: $(tail -1 $O/bench_tt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
for i in 1 2; do
  timeout -k 10 300 env RAY_AMD_DGRAD_WT=1 python bench.py --no-ray --steps 20 --warmup 5 > $O/bench_noray_wt_$i.log 2>&1 || { echo "bench wt rc=$?"; tail -30 $O/bench_noray_wt_$i.log; exit 1; }
  echo "no-ray dgrad-wt: $(tail -1 $O/bench_noray_wt_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
for sp in 4 8; do
  timeout -k 10 300 env RAY_AMD_WGRAD_SPLITS=$sp RAY_AMD_LT_TUNE=1 python bench.py --no-ray --steps 20 --warmup 5 > $O/bench_noray_splits$sp.log 2>&1 || { echo "bench splits rc=$?"; tail -30 $O/bench_noray_splits$sp.log; exit 1; }
  echo "no-ray wgrad splits=$sp: $(tail -1 $O/bench_noray_splits$sp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 300 python scripts/dgrad_layout_ab.py > $O/dgrad_layout.log 2>&1 || { echo "dgrad ab rc=$?"; tail -20 $O/dgrad_layout.log; exit 1; }
tail -1 $O/dgrad_layout.log
exit 0
