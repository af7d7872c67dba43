#!/bin/bash
# GPU box: workload benches (data via TorchTrainer ingest, IMPALA, PPO) at N = 1.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/wl3
mkdir -p $O
timeout -k 10 300 env RAY_AMD_DATA_TRAINER=1 python bench.py --workload data --steps 60 --warmup 5 > $O/data_trainer.log 2>&1 || { echo "data trainer rc=$?"; tail -20 $O/data_trainer.log; exit 1; }
tail -1 $O/data_trainer.log | cut -c1-300
timeout -k 10 300 python bench.py --workload data --steps 60 --warmup 5 > $O/data.log 2>&1 || { echo "data rc=$?"; tail -20 $O/data.log; exit 1; }
tail -1 $O/data.log | cut -c1-300




