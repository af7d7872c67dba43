#!/bin/bash
# round 6: calls D and E in one box session
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/gpu_r6d.sh && bash scripts/gpu_r6e.sh
