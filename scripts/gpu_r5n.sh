#!/bin/bash
# round 5, call N: the other BASELINE workloads on one MI355X (PPO, IMPALA, Data ingest),
# plus the all-reduce sweep at world 1
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5n
mkdir -p $O
rocm-smi --showpids --showpower --showclocks --showuse > $O/smi_0.txt 2>&1 || true
for w in ppo impala data; do
  timeout -k 10 400 python -u bench.py --workload $w > $O/bench_$w.log 2>&1 || { echo "$w rc=$?"; tail -20 $O/bench_$w.log; exit 1; }
  echo "$w: $(tail -1 $O/bench_$w.log | cut -c1-400)"
  rocm-smi --showpids --showpower --showclocks --showuse > $O/smi_$w.txt 2>&1 || true
done
for i in 1 2; do
  rocm-smi --showpids --showpower --showclocks --showuse > $O/smi_gpt2_pre$i.txt 2>&1 || true
  timeout -k 10 300 python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_gpt2_$i.log 2>&1 || { echo "gpt2 rc=$?"; exit 1; }
  echo "gpt2 $i: $(tail -1 $O/bench_gpt2_$i.log | cut -c1-200) load=$(cut -d' ' -f1 /proc/loadavg)"
done
exit 0
