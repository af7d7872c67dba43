#!/bin/bash
# round 5, call AA: HBM footprint side-stream vs single-stream (the back-to-back slow state
# coincides with the previous process still holding 267 GB in KFD teardown, r5p smi)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
export RAY_AMD_STREAM_AUTOTUNE=0
O=gpurun_out/r5aa
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("hbm"))'; }
timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_side.log 2>&1 || exit 1
echo "side: $(show $O/bench_side.log)"
rocm-smi --showpids > $O/smi_after_side.txt 2>&1 || true
grep -E "^[0-9]+ " $O/smi_after_side.txt | awk '$4>0' || true
sleep 40
timeout -k 10 300 env RAY_AMD_WGRAD_STREAM=0 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_serial.log 2>&1 || exit 1
echo "serial: $(show $O/bench_serial.log)"
exit 0
