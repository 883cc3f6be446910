set -o pipefail
mkdir -p gpurun_out/s40
PYTORCH_NO_HIP_MEMORY_CACHING=1 timeout -k 10 200 python3 tools/alloc_cycle.py 42 10 > gpurun_out/s40/alloc42.jsonl 2> gpurun_out/s40/alloc.err || { echo FAIL1; tail -5 gpurun_out/s40/alloc.err; exit 1; }
cat gpurun_out/s40/alloc42.jsonl
timeout -k 10 300 python3 tools/mem_cycle.py init --reps 12 --spp 2 > gpurun_out/s40/mem_cached.jsonl 2> gpurun_out/s40/mem.err || { echo FAIL2; tail -5 gpurun_out/s40/mem.err; exit 1; }
cat gpurun_out/s40/mem_cached.jsonl
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_stock.py tests/test_gpu_stock_4k.py > gpurun_out/s40/tests.log 2>&1 || { echo FAIL3; tail -20 gpurun_out/s40/tests.log; exit 1; }
tail -2 gpurun_out/s40/tests.log
