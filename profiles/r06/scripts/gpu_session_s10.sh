set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "finish_tail" -x -q --timeout 120 --timeout-method thread > gpurun_out/s10_tests.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/s10_tests.log | head -20; tail -5 gpurun_out/s10_tests.log; exit 1; }
tail -1 gpurun_out/s10_tests.log
timeout -k 10 600 python tools/session_rate.py init --reps 2 "finish_coop=0" "finish_coop=1" > gpurun_out/s10_init.jsonl 2> gpurun_out/s10_init.err || { echo FAIL1; tail -3 gpurun_out/s10_init.err; exit 1; }
tail -1 gpurun_out/s10_init.jsonl
