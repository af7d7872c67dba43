#!/bin/bash
# PMC counters for the attention kernels (kernel-trace only; no runtime/sys trace)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/pmc"
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1
export PYTHONPATH="$R"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/a" -o run \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES \
  -- python3 "$R/scripts/attn_bench.py" > "$R/gpurun_out/pmc/a.log" 2>&1
echo "rc=$?" >> "$R/gpurun_out/pmc/a.log"
