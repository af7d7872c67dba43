#!/bin/bash
# round 5, call AF: LayerNorm-backward column sums by in-kernel atomics into the fp32 flat
# gradient (no partial slabs, no colsum launches): numerics + step A/B (ra_knobs[14])
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp
export PYTHONPATH="$R"
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm or flat_direct or flash_attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
show() { tail -1 "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("wgrad_stream_autotune"))'; }
run() { local n=$1; shift; timeout -k 10 400 env "$@" python bench.py --no-ray --steps 30 --warmup 5 > $O/$n.log 2>&1 || exit 1; echo "$n: $(show $O/$n.log)"; }
run atom_a RAY_AMD_STREAM_AUTOTUNE=0
run slabs_a RAY_AMD_STREAM_AUTOTUNE=0 RAY_AMD_KNOBS=14=1
run atom_b RAY_AMD_STREAM_AUTOTUNE=0
run slabs_b RAY_AMD_STREAM_AUTOTUNE=0 RAY_AMD_KNOBS=14=1
run default
exit 0
