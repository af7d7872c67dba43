#!/bin/bash
# round 6, call M: IMPALA repeat (r6l measured 50.7k at box load 36 against 62.9k in r6k)
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r6m
mkdir -p $O
for i in 1 2; do
  echo "load before run $i: $(cut -d' ' -f1 /proc/loadavg) nproc=$(nproc)"
  timeout -k 10 400 python bench.py --workload impala > $O/impala_$i.log 2>&1 || { echo "impala rc=$?"; tail -20 $O/impala_$i.log; exit 1; }
  echo "impala $i: $(tail -1 $O/impala_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
exit 0
