#!/bin/bash
# tools/buildvar.sh NAME [extra hipcc flags...]: build extract.hip with the extra flags and link it
# with the product objects of general.hip / knn.hip (make first) as
# dsp-audioreclabs_amd/lib/libdsp_audiorec_NAME.so (A/B variants for tools/ab_bench.sh)
set -e
cd "$(dirname "$0")/../dsp-audioreclabs_amd/csrc"
n=$1; shift
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -I../../include -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form -mllvm -amdgpu-use-amdgpu-trackers=1"
/opt/rocm/bin/hipcc $F "$@" -c extract.hip -o ../lib/obj/extract_$n.o
/opt/rocm/bin/hipcc $F -shared ../lib/obj/extract_$n.o ../lib/obj/general.o ../lib/obj/knn.o ../lib/obj/wav_io.o -o ../lib/libdsp_audiorec_$n.so
