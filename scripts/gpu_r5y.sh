#!/bin/bash
# round 5, call Y: does free HBM return gradually after a big process exits? bench (big
# allocation) -> free-memory timeline -> bench; then bench -> bench back to back
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5y
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_1.log 2>&1 || exit 1
echo "bench 1: $(ms $O/bench_1.log)"
timeout -k 10 120 python scripts/mem_settle_probe.py 40 > $O/mem.log 2>&1 || exit 1
echo "free HBM after bench 1 exit:"; grep free_gb $O/mem.log | awk 'NR%4==1'
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_2.log 2>&1 || exit 1
echo "bench 2 (after the 40 s timeline): $(ms $O/bench_2.log)"
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_3.log 2>&1 || exit 1
echo "bench 3 (immediately): $(ms $O/bench_3.log)"
exit 0
