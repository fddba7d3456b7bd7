# A/B timing of library variants on one box: tools/ab.sh name1 name2 ... (lib/libdsp_audiorec_<name>.so; "base" = default)
for rep in 1 2; do
for v in "$@"; do
  lib=$PWD/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$PWD/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  DSP_LIB_PATH=$lib DIAG_VARIANTS=vad_hamming timeout -k 10 100 python tools/diag_extract.py 1000 | grep '"ms"' | sed "s/^/$v /"
done
done
