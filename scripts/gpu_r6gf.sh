#!/bin/bash
# round 6: calls G and F in one box session
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
bash scripts/gpu_r6g.sh && bash scripts/gpu_r6f.sh
