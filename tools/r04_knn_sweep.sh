#!/bin/bash
# KNN at the rank shape (12 500 x 100 000) and the full self-query: the model's split pick against
# forced split counts of the diagnostic build (DSP_KNN_NSPLIT), optionally library variants first.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
[ $# -gt 0 ] && bash tools/knn_libs_ab.sh base "$@"
bash tools/knn_split_sweep.sh 12500 8 9 10 11 12 13 14
bash tools/knn_split_sweep.sh 100000 3 4 5 6 7 8 10
