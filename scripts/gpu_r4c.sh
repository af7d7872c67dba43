#!/bin/bash
# round 4, call C: attention fwd v1/v2 A/B + occupancy PMC, whole-step HIP graph A/B
# (no-ray and TorchTrainer), kernel trace of the graphed step, GPU tests
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 150 python scripts/attn_fwd_ab.py > $O/attn_ab.log 2>&1 || { echo "attn ab rc=$?"; tail -20 $O/attn_ab.log; exit 1; }
tail -1 $O/attn_ab.log
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_occ -o run \
  --pmc SQ_WAVES SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
  -- python3 scripts/attn_bench3.py --iters 3 > $O/pmc_occ.log 2>&1
rc=$?; echo "pmc occ rc=$rc"
case $rc in 0|1|2) ;; *) tail -5 $O/pmc_occ.log; exit 1;; esac
for g in on off on off; do
  timeout -k 10 300 python bench.py --no-ray --steps 20 --warmup 5 --step-graph $g > $O/bench_noray_$g.log 2>&1 || { echo "bench $g rc=$?"; tail -30 $O/bench_noray_$g.log; exit 1; }
  echo "no-ray graph=$g: $(tail -1 $O/bench_noray_$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("step_graph"), d["final_loss"])')"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_tt.log 2>&1 || { echo "bench tt rc=$?"; tail -30 $O/bench_tt.log; exit 1; }
tail -1 $O/bench_tt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_graph -o p -- python3 bench.py --no-ray --steps 6 --warmup 3 > $O/prof_graph.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof_graph.log; exit 1; }
tail -1 $O/prof_graph.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -6 $O/gpu_tests.log
exit 0
