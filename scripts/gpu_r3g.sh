#!/bin/bash
# GPU box: GELU backward v2 + fixed-S split-K accumulate: tests, kernel bench, step bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gelu or colsum or flat_direct or linear or splitk or layernorm" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 "$R/scripts/gelu_bwd_bench.py" > "$R/$O/prof.log" 2>&1
echo "prof rc=$?"
grep "TB/s" $R/$O/prof.log
cd "$R"
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
echo "trainer: $(tail -1 $O/bench.log | cut -c1-170)"
timeout -k 10 300 python bench.py --no-ray > $O/bench_noray.log 2>&1 || { echo "bench noray rc=$?"; exit 1; }
echo "no-ray: $(tail -1 $O/bench_noray.log | cut -c1-170)"
