set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stock_4k.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/s31_4k.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E |Error" gpurun_out/s31_4k.log | head -20; tail -5 gpurun_out/s31_4k.log; exit 1; }
tail -2 gpurun_out/s31_4k.log
