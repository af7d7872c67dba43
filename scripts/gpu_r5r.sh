#!/bin/bash
# round 5, call R (+ S): the side-stream autotune back to back (the second and third processes
# start inside the post-process slow window), plus the default Ray TorchTrainer bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5r
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("wgrad_stream_autotune"))'; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_noray_$i.log 2>&1 || { echo "rc=$?"; tail -5 $O/bench_noray_$i.log; exit 1; }
  echo "noray $i: $(show $O/bench_noray_$i.log)"
done
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { echo "rc=$?"; tail -5 $O/bench_default.log; exit 1; }
echo "default (TorchTrainer): $(show $O/bench_default.log)"
sleep 35
bash scripts/gpu_r5s.sh
