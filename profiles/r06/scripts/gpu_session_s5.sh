set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py init --reps 2 "stock_random=0" "stock_random=1,async_prio=1" "stock_random=0,async_prio=1" "stock_random=1,async_prio=1,stock_lanes=3" > gpurun_out/s5_init.jsonl 2> gpurun_out/s5_init.err || { echo FAIL1; tail -3 gpurun_out/s5_init.err; exit 1; }
tail -1 gpurun_out/s5_init.jsonl
