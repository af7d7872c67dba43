#!/bin/bash
# round 5, call AB: back-to-back benches with the HBM-teardown settle guard and the end-of-
# run HBM release; an expandable-segments arm for the side-stream cache bloat (95 GB
# reserved vs 28 GB allocated, r5aa)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5ab
mkdir -p $O
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "settle", d.get("gpu_settle_wait_s"), "hbm", d.get("hbm"), d.get("wgrad_stream_autotune",{}) and d["wgrad_stream_autotune"].get("chosen"))'; }
for n in 1 2; do
  timeout -k 10 400 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_noray_$n.log 2>&1 || { tail -5 $O/bench_noray_$n.log; exit 1; }
  echo "noray $n: $(show $O/bench_noray_$n.log)"
done
timeout -k 10 400 env PYTORCH_HIP_ALLOC_CONF=expandable_segments:True python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_expseg.log 2>&1 || { tail -5 $O/bench_expseg.log; exit 1; }
echo "expandable_segments: $(show $O/bench_expseg.log)"
timeout -k 10 500 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
echo "default (TorchTrainer): $(show $O/bench_default.log)"
exit 0
