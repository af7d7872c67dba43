#!/bin/bash
# round 5, call AL: PMC counters of the GPT-2 step's kernels (3 passes, each its own run;
# counters only with --kernel-trace, never with trace domains)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5al
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d $O/sq -o run -- python bench.py --no-ray --steps 2 --warmup 1 > $O/sq.log 2>&1 || { echo "sq rc=$?"; tail -20 $O/sq.log; exit 1; }
echo sq done
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/fetch -o run -- python bench.py --no-ray --steps 2 --warmup 1 > $O/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -20 $O/fetch.log; exit 1; }
echo fetch done
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/write -o run -- python bench.py --no-ray --steps 2 --warmup 1 > $O/write.log 2>&1 || { echo "write rc=$?"; tail -20 $O/write.log; exit 1; }
echo write done
ls -R $O | head -30
exit 0
