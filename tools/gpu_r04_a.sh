#!/bin/bash
# r04 first GPU call: the step-count experiment, then the 4-wave executor validation + A/B.
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
tools/gpu_r04_steps.sh r04_steps && tools/gpu_r04_exec3.sh r04_exec3
