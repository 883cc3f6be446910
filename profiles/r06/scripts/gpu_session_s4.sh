set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stock.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s4_stock_tests.log 2>&1 || { echo STOCKFAIL; grep -E "^FAILED|^E " gpurun_out/s4_stock_tests.log | head -20; tail -5 gpurun_out/s4_stock_tests.log; exit 1; }
tail -1 gpurun_out/s4_stock_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/s4_suite.log 2>&1 || { echo SUITEFAIL; grep -E "^FAILED|^E " gpurun_out/s4_suite.log | head -20; exit 1; }
tail -1 gpurun_out/s4_suite.log
timeout -k 10 600 python tools/session_rate.py init --reps 2 "stock_random=0" "stock_random=1" > gpurun_out/s4_init.jsonl 2> gpurun_out/s4_init.err || { echo FAIL1; tail -3 gpurun_out/s4_init.err; exit 1; }
tail -1 gpurun_out/s4_init.jsonl
timeout -k 10 300 python tools/session_rate.py c5 --reps 1 "" > gpurun_out/s4_c5.jsonl 2> gpurun_out/s4_c5.err || { echo FAIL2; exit 1; }
tail -1 gpurun_out/s4_c5.jsonl
timeout -k 10 300 python tools/session_rate.py init --reps 1 "log=1" > /dev/null 2> gpurun_out/s4_init_log.txt || exit 1
