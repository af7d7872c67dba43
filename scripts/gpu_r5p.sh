#!/bin/bash
# round 5, call P: why every bench process after the first in a call runs ~3x slower
# (r5g-r5o). Probes: a pause between processes, HW queue counts, a single-stream step,
# the same step under rocprofv3, and the KFD process list / GPU state between runs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5p
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])'; }
state() {
  echo "  kfd procs: $(ls /sys/class/kfd/kfd/proc 2>/dev/null | tr '\n' ' ')"
  rocm-smi --showpids --showuse --showpower --showclocks > $O/smi_$1.txt 2>&1 || true
  grep -E "GPU use|Power|sclk" $O/smi_$1.txt | tr -s ' ' | head -4 | sed 's/^/  /'
}
run() {  # name env...
  local n=$1; shift
  state $n
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(ms $O/bench_$n.log) ms load=$(cut -d' ' -f1 /proc/loadavg)"
}
run first X=1
run second X=1
sleep 30
run after_sleep30 X=1
run hwq4 RAY_AMD_HW_QUEUES=4
run serial RAY_AMD_WGRAD_STREAM=0
state prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo "under rocprofv3: $(ms $O/bench_prof.log) ms"
find $O/prof -name "*.csv" -size +20M -delete
run last X=1
exit 0
