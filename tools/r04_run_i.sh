set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04i_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04i_gpu_tests.log
bash tools/r04_kt.sh r04i r03 base c1 c2 q1c1
