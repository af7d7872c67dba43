#!/bin/bash
# GPU box: step kernel stats + attention PMC passes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p "$R/gpurun_out/prof3" "$R/gpurun_out/pmc3"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof3" -o run -- python3 "$R/bench.py" --no-ray --steps 5 --warmup 3 > "$R/gpurun_out/prof3.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc3/a" -o run \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES \
  -- python3 "$R/scripts/attn_bench.py" --B 64 > "$R/gpurun_out/pmc3/a.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc3/b" -o run \
  --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -- python3 "$R/scripts/attn_bench.py" --B 64 > "$R/gpurun_out/pmc3/b.log" 2>&1
echo "pmc rc=$?" >> "$R/gpurun_out/pmc3/b.log"
