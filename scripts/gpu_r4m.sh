#!/bin/bash
# round 4, call M: 8 vs 16 hardware queues per process (TorchTrainer and the bare loop)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4m
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
for i in 1 2; do
  for q in 8 16; do
    timeout -k 10 300 env RAY_AMD_HW_QUEUES=$q python bench.py --steps 30 --warmup 5 > $O/tt_q${q}_$i.log 2>&1 || { echo "tt rc=$?"; tail -20 $O/tt_q${q}_$i.log; exit 1; }
    echo "tt hwq=$q $i: $(ms $O/tt_q${q}_$i.log)"
    timeout -k 10 300 env RAY_AMD_HW_QUEUES=$q python bench.py --no-ray --steps 30 --warmup 5 > $O/noray_q${q}_$i.log 2>&1 || { echo "noray rc=$?"; exit 1; }
    echo "no-ray hwq=$q $i: $(ms $O/noray_q${q}_$i.log)"
  done
done
exit 0
