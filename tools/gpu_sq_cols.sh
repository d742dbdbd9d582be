#!/bin/bash
# SQ instruction counts per kernel for column subsets of the SF1 file (which page kinds cost what).
cd ${GRAFT_REPO_ROOT:-/root/repo} || exit 1
for spec in "comment:15" "dictstr:8,9,13,14" "dictfix:2,3,4,6,7,10,11,12" "plainfix:0,1,5"; do
  name=${spec%%:*}; cols=${spec#*:}
  echo "== $name ($cols)"
  tools/gpu_sq_wl.sh r03_sqc_$name 'k_' --columns $cols | grep -v rocprim | grep -v k_enc || exit 1
done
