#!/bin/bash
# round 5, call AC: caching-allocator counters of the side-stream vs single-stream step
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5ac
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("hbm"))'; }
timeout -k 10 400 python bench.py --no-ray --steps 30 --warmup 5 > $O/side.log 2>&1 || exit 1
echo "side: $(show $O/side.log)"
timeout -k 10 400 env RAY_AMD_WGRAD_STREAM=0 python bench.py --no-ray --steps 30 --warmup 5 > $O/serial.log 2>&1 || exit 1
echo "serial: $(show $O/serial.log)"
timeout -k 10 400 env PYTORCH_HIP_ALLOC_CONF=garbage_collection_threshold:0.5 python bench.py --no-ray --steps 30 --warmup 5 > $O/gc05.log 2>&1 || exit 1
echo "gc0.5: $(show $O/gc05.log)"
exit 0
