#!/bin/bash
# GPU box: component microbenchmarks (wgrad / LM head / xent) + attention PMC passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out/pmc
timeout -k 10 400 python -u scripts/r2_perf_bench.py > gpurun_out/r2_perf.log 2>&1 || exit $?
cd /tmp
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/a" -o run \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES \
  -- python3 "$R/scripts/attn_bench.py" --B 64 > "$R/gpurun_out/pmc/a.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/b" -o run \
  --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -- python3 "$R/scripts/attn_bench.py" --B 64 > "$R/gpurun_out/pmc/b.log" 2>&1
echo "pmc b rc=$?" >> "$R/gpurun_out/pmc/b.log"
echo done
