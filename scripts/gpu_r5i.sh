#!/bin/bash
# round 5, call I: step timing vs host CPU load (r5g/r5h: first run ~62.5 ms, later runs
# 118-188 ms); eager vs whole-step HIP graph, with the load average logged per run
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5i
mkdir -p $O
ms() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"), d["config"].get("step_graph"))'; }
run() {  # name env...
  local n=$1; shift
  local la=$(cut -d' ' -f1-3 /proc/loadavg)
  timeout -k 10 300 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/bench_$n.log 2>&1 || { echo "bench $n rc=$?"; tail -20 $O/bench_$n.log; exit 1; }
  echo "$n: $(ms $O/bench_$n.log) load=[$la] -> [$(cut -d' ' -f1-3 /proc/loadavg)]"
}
echo "nproc=$(nproc) cpus_allowed=$(grep Cpus_allowed_list /proc/self/status)"
for i in 1 2 3; do
  run eager_$i RAY_AMD_STEP_GRAPH=0
  run graph_$i RAY_AMD_STEP_GRAPH=1
done
exit 0
