set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python tools/session_rate.py c5 --reps 2 "" "trace_grid_pct=60" "trace_grid_pct=90" "async_prio=1" "stock_ahead=32" "small_lanes=1" > gpurun_out/s16_c5.jsonl 2> gpurun_out/s16_c5.err || { echo FAIL1; tail -3 gpurun_out/s16_c5.err; exit 1; }
tail -1 gpurun_out/s16_c5.jsonl
timeout -k 10 600 python tools/session_rate.py init --reps 2 "" "finish_below=131072" "finish_below=524288" "trace_grid_pct=60" "async_prio=1" > gpurun_out/s16_init.jsonl 2> gpurun_out/s16_init.err || { echo FAIL2; tail -3 gpurun_out/s16_init.err; exit 1; }
tail -1 gpurun_out/s16_init.jsonl
