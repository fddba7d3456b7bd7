#!/bin/bash
# tools/kinfo.sh [hipcc flags...]: code bytes, VGPRs, spills and scratch of the extraction kernels
# (device-only compile of extract.hip with the given -D flags)
cd "$(dirname "$0")/../dsp-audioreclabs_amd/csrc"
O=/tmp/kinfo_$$.o
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../include -Wno-unused-function -mllvm -amdgpu-use-amdgpu-trackers=1 \
    --offload-device-only --no-gpu-bundle-output -c extract.hip -o $O "$@" -Rpass-analysis=kernel-resource-usage 2>&1 |
    grep -E "Function Name|VGPRs:|Spill|ScratchSize" | sed 's/.*remark: *//' | sed 's/ \[-Rpass.*\]//' | paste - - - - - | sed 's/_ZN3dsp14//'
/opt/rocm/lib/llvm/bin/llvm-readelf -s $O | awk '$4 == "FUNC" {print "code bytes", $3, $8}'
rm -f $O
