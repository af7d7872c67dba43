cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc1 -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -- python scripts/hip_gemm_bench.py --only fc2_fwd,qkv_fwd --variant 1 --iters 3 --no-epi > gpurun_out/pmc1.log 2>&1
echo rc=$?
