#!/bin/bash
# GPU box: compiled-DAG GPU tensors, Data GPU ingest tests, image_normalize bandwidth,
# data bench (hbm + h2d paths), rocprof of the image_normalize microbench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
export TMPDIR=/tmp PYTHONPATH="$R"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_compiled_dag_gpu.py tests/test_data_gpu.py "tests/test_kernels_gpu.py::test_image_normalize" "tests/test_kernels_gpu.py::test_image_normalize_vector_path" -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_r2f.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_r2f.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/r2_perf_bench.py --part imgnorm > gpurun_out/imgnorm.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload data --data-path hbm --steps 30 --warmup 5 > gpurun_out/data_hbm.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload data --data-path h2d --steps 30 --warmup 5 > gpurun_out/data_h2d.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_imgnorm -o run -- python3 scripts/r2_perf_bench.py --part imgnorm > gpurun_out/prof_imgnorm.log 2>&1 || exit $?
echo done
