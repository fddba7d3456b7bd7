#!/bin/bash
# KNN at the rank shape (12 500 x 100 000) and the full self-query: seed-sample / warm-up variants
# (lib/libdsp_audiorec_<v>.so) and a forced split sweep of the diagnostic build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/knn_libs_ab.sh base "$@"
bash tools/knn_split_sweep.sh 12500 4 6 8 10 12 16 20 25 32
