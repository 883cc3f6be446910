set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/session_rate.py c5 --reps 1 "" "stock_lanes=3" > gpurun_out/s18_c5_q4.jsonl 2> gpurun_out/s18_c5_q4.err || { echo FAIL0; tail -3 gpurun_out/s18_c5_q4.err; exit 1; }
tail -1 gpurun_out/s18_c5_q4.jsonl
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python tools/session_rate.py c5 --reps 2 "" "stock_lanes=3" "stock_lanes=4" > gpurun_out/s18_c5.jsonl 2> gpurun_out/s18_c5.err || { echo FAIL1; tail -3 gpurun_out/s18_c5.err; exit 1; }
tail -1 gpurun_out/s18_c5.jsonl
timeout -k 10 600 python tools/session_rate.py init --reps 2 "" "stock_lanes=3" > gpurun_out/s18_init.jsonl 2> gpurun_out/s18_init.err || { echo FAIL2; tail -3 gpurun_out/s18_init.err; exit 1; }
tail -1 gpurun_out/s18_init.jsonl
timeout -k 10 600 python tools/session_rate.py c3 --reps 2 "" > gpurun_out/s18_c3.jsonl 2> gpurun_out/s18_c3.err || { echo FAIL3; tail -3 gpurun_out/s18_c3.err; exit 1; }
tail -1 gpurun_out/s18_c3.jsonl
