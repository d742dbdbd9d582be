#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo} && tools/gpu_ab_env2.sh r03_flatall 2 "PF_FLAT_SPLIT=0" "PF_FLAT_SPLIT=1" && NO_TESTS=1 tools/gpu_ab_env2.sh r03_flatall_wide 1 "PF_FLAT_SPLIT=0" "PF_FLAT_SPLIT=1" -- --workload wide
