#!/bin/bash
# round 4, call A: GPU tests, the stream-K probe, bench with DDP hooks off/on, rocprof of hooks-on
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -8 $O/gpu_tests.log
case $rc in 0|1) ;; *) exit 1;; esac
tail -3 $O/gpu_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/skprobe -o sk -- python3 scripts/lmhead_sk_probe.py > $O/skprobe.log 2>&1 || { echo "probe rc=$?"; tail -20 $O/skprobe.log; exit 1; }
grep rows= $O/skprobe.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_off.log 2>&1 || { echo "bench off rc=$?"; tail -20 $O/bench_off.log; exit 1; }
tail -1 $O/bench_off.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ddp-hooks always > $O/bench_on.log 2>&1 || { echo "bench on rc=$?"; tail -20 $O/bench_on.log; exit 1; }
tail -1 $O/bench_on.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_on -o p -- python3 bench.py --no-ray --steps 6 --warmup 2 --ddp-hooks always > $O/prof_on.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof_on.log; exit 1; }
tail -1 $O/prof_on.log
# LAST step: bounded repro of the removed side-stream-dW LM-head layout (may hang -> exit 3)
timeout -k 10 120 python -u scripts/lmhead_hang_repro.py 20 40 > $O/hang_repro.log 2>&1; echo "hang repro rc=$?"; tail -3 $O/hang_repro.log
