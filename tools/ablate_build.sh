#!/bin/bash
# Ablation variants of the extraction kernel (diagnostic: outputs are wrong) for instruction and
# time deltas per phase: lib/libdsp_audiorec_abl<mask>.so.  usage: tools/ablate_build.sh mask...
cd "$(dirname "$0")/.."
for m in "$@"; do bash tools/buildvar.sh abl$m -DDSP_ABL=$m 2>&1 | grep -v "argument unused"; done
