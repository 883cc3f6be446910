set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/session_rate.py c5 --reps 2 "" "async_fused_below=67108864" "async_fused_below=67108864,async_grid_pct=100" "async_grid_pct=100" > gpurun_out/s14_c5.jsonl 2> gpurun_out/s14_c5.err || { echo FAIL1; tail -3 gpurun_out/s14_c5.err; exit 1; }
tail -1 gpurun_out/s14_c5.jsonl
timeout -k 10 600 python tools/session_rate.py init --reps 2 "" "async_fused_below=67108864,async_grid_pct=100" "async_grid_pct=100" > gpurun_out/s14_init.jsonl 2> gpurun_out/s14_init.err || { echo FAIL2; tail -3 gpurun_out/s14_init.err; exit 1; }
tail -1 gpurun_out/s14_init.jsonl
