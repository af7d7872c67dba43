#!/bin/bash
# round 5, call M: fraction of the CUs the side-stream wgrad fills (fewer, longer workgroups)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5m
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
for i in 1 2; do
  for f in 1.0 0.5 0.75 0.25; do
    timeout -k 10 300 env RAY_AMD_WGRAD_FILL=$f python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_${f}_$i.log 2>&1 || { echo "bench $f rc=$?"; tail -20 $O/bench_${f}_$i.log; exit 1; }
    echo "fill=$f $i: $(ms $O/bench_${f}_$i.log) load=$(cut -d' ' -f1 /proc/loadavg)"
  done
done
exit 0
