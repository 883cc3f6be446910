set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/s15_suite.log 2>&1 || { echo SUITEFAIL; grep -E "^FAILED|^E " gpurun_out/s15_suite.log | head -20; exit 1; }
tail -1 gpurun_out/s15_suite.log
timeout -k 10 900 python tools/session_rate.py c5 --reps 2 "" "async_grid_pct=0,async_fused_below=0" > gpurun_out/s15_c5.jsonl 2> gpurun_out/s15_c5.err || { echo FAIL1; tail -3 gpurun_out/s15_c5.err; exit 1; }
tail -1 gpurun_out/s15_c5.jsonl
timeout -k 10 600 python tools/session_rate.py init --reps 3 "" "async_grid_pct=0,async_fused_below=0" > gpurun_out/s15_init.jsonl 2> gpurun_out/s15_init.err || { echo FAIL2; tail -3 gpurun_out/s15_init.err; exit 1; }
tail -1 gpurun_out/s15_init.jsonl
