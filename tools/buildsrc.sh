#!/bin/bash
# tools/buildsrc.sh NAME SRC [extra hipcc flags...]: build an extract.hip variant from another source
# file (a patched copy, for A/B of code changes that have no switch) and link it with the product
# objects of general.hip / knn.hip / wav_io.cpp (make first) as lib/libdsp_audiorec_NAME.so
set -e
cd "$(dirname "$0")/../dsp-audioreclabs_amd/csrc"
n=$1; src=$2; shift 2
F="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -I../../include -I. -Wall -Wno-unused-function -mllvm -amdgpu-use-amdgpu-trackers=1"
/opt/rocm/bin/hipcc $F "$@" -c "$src" -o ../lib/obj/extract_$n.o
/opt/rocm/bin/hipcc $F -shared ../lib/obj/extract_$n.o ../lib/obj/general.o ../lib/obj/knn.o ../lib/obj/wav_io.o -o ../lib/libdsp_audiorec_$n.so
