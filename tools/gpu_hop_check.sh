#!/bin/bash
# GPU box: parity tests, hop-vs-generic bench timing, hop-kernel phase stamps
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_hop.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/gt_hop.log
for k in hop generic; do
  if [ $k = generic ]; then export DSP_EXTRACT_KERNEL=generic; fi
  timeout -k 10 120 python3 bench.py --no-cpu > gpurun_out/b_$k.json 2> gpurun_out/b_$k.err || { echo "bench $k failed"; tail -5 gpurun_out/b_$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/b_$k.json').read().strip().splitlines()[-1]); print('$k', d['roofline']['kernel_avg_ms'], d['ms_per_step'], d['roofline']['frac'])"
done
unset DSP_EXTRACT_KERNEL
DSP_LIB_PATH=$PWD/dsp-audioreclabs_amd/lib/libdsp_audiorec_stamps.so timeout -k 10 60 python3 tools/hop_stamps.py 1000 2>/dev/null
