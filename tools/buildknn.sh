#!/bin/bash
# tools/buildknn.sh NAME [extra hipcc flags...]: build knn.hip with the extra flags and link it with
# the product objects of extract.hip / general.hip as lib/libdsp_audiorec_NAME.so (KNN A/B variants)
set -e
cd "$(dirname "$0")/../dsp-audioreclabs_amd/csrc"
n=$1; shift
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -I../../include -Wall -Wno-unused-function -mllvm -amdgpu-mfma-vgpr-form"
/opt/rocm/bin/hipcc $F "$@" -c knn.hip -o ../lib/obj/knn_$n.o
/opt/rocm/bin/hipcc $F -shared ../lib/obj/extract.o ../lib/obj/general.o ../lib/obj/knn_$n.o ../lib/obj/wav_io.o -o ../lib/libdsp_audiorec_$n.so
