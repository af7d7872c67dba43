#!/bin/bash
# Run GPU calls one after another (each through gpurun_retry.sh); stop at the first that
# fails for a reason other than "no box". Usage: scripts/gpu_chain.sh NAME [NAME...] runs
# scripts/gpu_NAME.sh with log gpurun_out/NAME_call.log.
for n in "$@"; do
  scripts/gpurun_retry.sh "gpurun_out/${n}_call.log" 1200 bash "scripts/gpu_${n}.sh" || exit $?
done
