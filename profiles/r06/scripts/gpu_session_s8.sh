set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py init --reps 2 "" "async_grid_pct=25" "async_grid_pct=40" "async_grid_pct=60" "async_grid_pct=40,async_prio=1" > gpurun_out/s8_init.jsonl 2> gpurun_out/s8_init.err || { echo FAIL1; tail -3 gpurun_out/s8_init.err; exit 1; }
tail -1 gpurun_out/s8_init.jsonl
timeout -k 10 600 python tools/session_rate.py c5 --reps 1 "" "async_grid_pct=40" "async_grid_pct=60" > gpurun_out/s8_c5.jsonl 2> gpurun_out/s8_c5.err || { echo FAIL2; tail -3 gpurun_out/s8_c5.err; exit 1; }
tail -1 gpurun_out/s8_c5.jsonl
