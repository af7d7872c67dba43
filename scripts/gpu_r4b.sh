#!/bin/bash
# round 4, call B: PMC counters of the attention kernels (two passes, kernel-trace only),
# then the LM-head hang root-cause arms (serial first, then ops/lt side stream LAST: it may hang)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 120 python scripts/attn_bench3.py > $O/attn_plain.log 2>&1 || { echo "attn bench rc=$?"; tail $O/attn_plain.log; exit 1; }
tail -1 $O/attn_plain.log
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/pmc1 -o run \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES \
  -- python3 scripts/attn_bench3.py --iters 3 > $O/pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"
case $rc in 0) ;; *) tail -5 $O/pmc1.log; exit 1;; esac
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/pmc2 -o run \
  --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM \
  -- python3 scripts/attn_bench3.py --iters 3 > $O/pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
case $rc in 0|1|2) ;; *) tail -5 $O/pmc2.log; exit 1;; esac
timeout -k 10 90 python -u scripts/lmhead_hang_repro.py 10 30 serial > $O/hang_serial.log 2>&1; rc=$?
echo "serial rc=$rc"; tail -2 $O/hang_serial.log
[ $rc -eq 0 ] || exit 1
# LAST step: may hang (exit 3 after the 30 s watchdog)
timeout -k 10 90 python -u scripts/lmhead_hang_repro.py 10 30 lt > $O/hang_lt.log 2>&1; rc=$?
echo "lt rc=$rc"; tail -2 $O/hang_lt.log
exit 0
