#!/bin/bash
# round 4, call F: Data ingest (1 vs 2 preprocessing actors, pinned store pages; 300
# steps with timelines), PPO with 5 vs 20 envs per runner, then the LM-head hang arms:
# per-stream handles (expect drain), shared workspace, shared handle (expected to hang:
# LAST step, bounded by its watchdog)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4f
mkdir -p $O
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
