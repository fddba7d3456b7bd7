#!/bin/bash
# A/B of library variants at 100k / 12.5k clips (no tests), then stamps of stamp-build variants:
#   bash tools/r05_ab2.sh TAG "v1 v2 ..." "stampvariant1 ..."
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05x}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
for clips in 100000 12500; do
  timeout -k 10 600 bash tools/ab_bench.sh $clips $2 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt || exit 1
done
[ -n "$3" ] && { timeout -k 10 400 bash tools/stamps_seq.sh $T $3 > $O/stamps.txt 2>&1; cat $O/stamps.txt; }
echo R05X_DONE
