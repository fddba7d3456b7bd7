#!/bin/bash
# tools/buildvar.sh NAME [extra hipcc flags...]: build the current sources as
# dsp-audioreclabs_amd/lib/libdsp_audiorec_NAME.so (A/B variants for tools/ab.sh)
set -e
cd "$(dirname "$0")/../dsp-audioreclabs_amd/csrc"
n=$1; shift
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -I../../include -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form "$@" extract.hip general.hip knn.hip -o ../lib/libdsp_audiorec_$n.so
