# A/B timing on one box: tools/ab.sh spec ...   spec = lib name (lib/libdsp_audiorec_<name>.so, "base" =
# default lib) optionally with :v3 / :v4 to force the kernel variant
for rep in 1 2 3; do
for spec in "$@"; do
  v=${spec%%:*}; var=${spec#*:}; [ "$var" = "$spec" ] && var=""
  lib=$PWD/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$PWD/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  DSP_EXTRACT_VARIANT=$var DSP_LIB_PATH=$lib DIAG_VARIANTS=vad_hamming,novad_hamming timeout -k 10 100 python tools/diag_extract.py 1000 | grep '"ms"' | tr -d '\n' | sed "s/^/$spec /"; echo
done
done
