#!/bin/bash
# PMC passes (one counter group per pass) over the extraction kernel; run on the GPU box.
# Usage: tools/pmc_extract.sh <tag> "<group1>" "<group2>" ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o p -- python3 $R/tools/diag_extract.py 1000 > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
echo PMC_DONE
