#!/bin/bash
# GPU box: data-ingest stage probes + data benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/data3
mkdir -p $O
[ -x scripts/probes/shm_fault ] || gcc -O2 -o scripts/probes/shm_fault scripts/probes/shm_fault.c
timeout -k 5 60 scripts/probes/shm_fault > $O/shm_fault.log 2>&1; cat $O/shm_fault.log
timeout -k 10 200 python scripts/probes/task_put.py > $O/task_put.log 2>&1; tail -5 $O/task_put.log
timeout -k 10 300 python scripts/data_probe.py > $O/data_probe.log 2>&1 || { echo "probe rc=$?"; tail -20 $O/data_probe.log; exit 1; }
grep -v amdgpu.ids $O/data_probe.log
timeout -k 10 300 python bench.py --workload data --steps 60 --warmup 5 > $O/data.log 2>&1 || { echo "data rc=$?"; tail -20 $O/data.log; exit 1; }
tail -1 $O/data.log | cut -c1-200
timeout -k 10 300 env RAY_AMD_DATA_TRAINER=1 python bench.py --workload data --steps 60 --warmup 5 > $O/data_trainer.log 2>&1 || { echo "data trainer rc=$?"; tail -20 $O/data_trainer.log; exit 1; }
tail -1 $O/data_trainer.log | cut -c1-200
