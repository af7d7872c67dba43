#!/bin/bash
# round 4, call J: is the hooks-on / TorchTrainer overhead hardware-queue sharing? More
# streams than GPU_MAX_HW_QUEUES (4) makes streams share a hardware queue, where one
# stream's event wait blocks the other's kernels. Arms interleaved: default vs 8 queues.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r4j
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])'; }
for i in 1 2; do
  for q in 4 8; do
    timeout -k 10 300 env GPU_MAX_HW_QUEUES=$q python bench.py --no-ray --ddp-hooks always --steps 30 --warmup 5 > $O/hooks_q${q}_$i.log 2>&1 || { echo "hooks rc=$?"; tail -30 $O/hooks_q${q}_$i.log; exit 1; }
    echo "hooks always hwq=$q $i: $(ms $O/hooks_q${q}_$i.log)"
    timeout -k 10 300 env GPU_MAX_HW_QUEUES=$q python bench.py --steps 30 --warmup 5 > $O/tt_q${q}_$i.log 2>&1 || { echo "tt rc=$?"; tail -30 $O/tt_q${q}_$i.log; exit 1; }
    echo "tt hwq=$q $i: $(ms $O/tt_q${q}_$i.log)"
    timeout -k 10 300 env GPU_MAX_HW_QUEUES=$q python bench.py --no-ray --steps 30 --warmup 5 > $O/noray_q${q}_$i.log 2>&1 || { echo "noray rc=$?"; tail -30 $O/noray_q${q}_$i.log; exit 1; }
    echo "no-ray hwq=$q $i: $(ms $O/noray_q${q}_$i.log)"
  done
done
exit 0
