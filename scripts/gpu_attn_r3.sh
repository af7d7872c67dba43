#!/bin/bash
# GPU box: attention timings + PMC passes (kernel-trace only, one pass per counter group).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp PYTHONPATH="$R"
O="$R/gpurun_out/attn3"
mkdir -p "$O"
cd /tmp
timeout -k 10 120 python3 "$R/scripts/attn_bench3.py" > "$O/bench.log" 2>&1 || { echo "bench rc=$?"; tail "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
timeout -k 10 60 rocprofv3 -L > "$O/counters.txt" 2>&1
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$O/p$i" -o run --pmc $grp -- python3 "$R/scripts/attn_bench3.py" --iters 3 > "$O/p$i.log" 2>&1 || { echo "pmc pass $i rc=$?"; tail -3 "$O/p$i.log"; }
done
echo done
