#!/bin/bash
# round 5, call C: GPT-2 step A/B — hand-written wgrad (RAY_AMD_WGRAD=hip) vs hipBLASLt split-K
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5c
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))'; }
for i in 1 2 3; do
  for wg in hip lt-splitk; do
    timeout -k 10 300 env RAY_AMD_WGRAD=$wg python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_${wg}_$i.log 2>&1 || { echo "bench $wg rc=$?"; tail -20 $O/bench_${wg}_$i.log; exit 1; }
    echo "wgrad=$wg $i: $(ms $O/bench_${wg}_$i.log)"
  done
done
timeout -k 10 300 env RAY_AMD_WGRAD=hip rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-ray --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*.csv" -size +20M -delete
find $O/prof -name "*kernel_stats.csv"
exit 0
