#!/bin/bash
# round 4, call E: forward v1 restored (GPU tests + A/B baseline), backward ILP variants,
# bench, Data ingest with 1 vs 2 preprocessing actors (300 steps, timeline), PPO with 5 vs
# 20 envs per runner, then the LM-head hang arms: per-stream handles (expect drain), shared
# workspace, shared handle (expected to hang: LAST step, bounded by its watchdog)
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
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_tt.log 2>&1 || { echo "bench tt rc=$?"; tail -30 $O/bench_tt.log; exit 1; }
echo "torchtrainer: $(tail -1 $O/bench_tt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
for i in 1 2; do
  timeout -k 10 300 env RAY_AMD_DGRAD_WT=1 python bench.py --no-ray --steps 20 --warmup 5 > $O/bench_noray_wt_$i.log 2>&1 || { echo "bench wt rc=$?"; tail -30 $O/bench_noray_wt_$i.log; exit 1; }
  echo "no-ray dgrad-wt: $(tail -1 $O/bench_noray_wt_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
for i in 1 2; do
  timeout -k 10 300 env RAY_AMD_OPT_OVERLAP=1 python bench.py --no-ray --steps 20 --warmup 5 > $O/bench_noray_optov_$i.log 2>&1 || { echo "bench optov rc=$?"; tail -30 $O/bench_noray_optov_$i.log; exit 1; }
  echo "no-ray opt-overlap: $(tail -1 $O/bench_noray_optov_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
for sp in 4 8; do
  timeout -k 10 300 env RAY_AMD_WGRAD_SPLITS=$sp RAY_AMD_LT_TUNE=1 python bench.py --no-ray --steps 20 --warmup 5 > $O/bench_noray_splits$sp.log 2>&1 || { echo "bench splits rc=$?"; tail -30 $O/bench_noray_splits$sp.log; exit 1; }
  echo "no-ray wgrad splits=$sp: $(tail -1 $O/bench_noray_splits$sp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 300 python scripts/dgrad_layout_ab.py > $O/dgrad_layout.log 2>&1 || { echo "dgrad ab rc=$?"; tail -20 $O/dgrad_layout.log; exit 1; }
tail -1 $O/dgrad_layout.log
for cfg in a1 a2 a1pin; do
  a=${cfg:1:1}; pin=0; [ "$cfg" = a1pin ] && pin=1
  timeout -k 10 400 env RAY_AMD_DATA_GPU_ACTORS=$a RAY_AMD_DATA_PIN_STORE=$pin RAY_AMD_DATA_TRAINER=1 RAY_AMD_DATA_TIMELINE=$O/data_timeline_$cfg.json python bench.py --workload data --steps 300 --warmup 20 > $O/data_trainer_$cfg.log 2>&1 || { echo "data rc=$?"; tail -20 $O/data_trainer_$cfg.log; exit 1; }
  echo "trainer $cfg: $(tail -1 $O/data_trainer_$cfg.log | cut -c1-120)"
  python scripts/data_timeline.py $O/data_timeline_$cfg.json > $O/data_timeline_$cfg.txt 2>&1; head -8 $O/data_timeline_$cfg.txt
  timeout -k 10 400 env RAY_AMD_DATA_GPU_ACTORS=$a RAY_AMD_DATA_PIN_STORE=$pin python bench.py --workload data --steps 300 --warmup 20 > $O/data_direct_$cfg.log 2>&1 || { echo "data direct rc=$?"; tail -20 $O/data_direct_$cfg.log; exit 1; }
  echo "direct $cfg: $(tail -1 $O/data_direct_$cfg.log | cut -c1-120)"
done
for e in 5 20; do
  timeout -k 10 400 env RAY_AMD_RUNNER_ENVS=$e RAY_AMD_PPO_ASYNC=1 python bench.py --workload ppo --steps 8 --warmup 2 > $O/ppo_envs$e.log 2>&1 || { echo "ppo rc=$?"; tail -20 $O/ppo_envs$e.log; exit 1; }
  echo "ppo envs=$e: $(tail -1 $O/ppo_envs$e.log | cut -c1-120)"
done
timeout -k 10 120 python scripts/lmhead_hang_repro.py 10 40 lt2 > $O/lmhead_lt2.log 2>&1; rc=$?
echo "lt2 rc=$rc: $(tail -1 $O/lmhead_lt2.log)"
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/lmhead_hang_repro.py 10 40 lt2shared > $O/lmhead_lt2shared.log 2>&1; rc=$?
echo "lt2shared rc=$rc: $(tail -1 $O/lmhead_lt2shared.log)"
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python scripts/lmhead_hang_repro.py 10 40 lt2h > $O/lmhead_lt2h.log 2>&1; rc=$?
echo "lt2h rc=$rc: $(tail -1 $O/lmhead_lt2h.log)"
exit 0
