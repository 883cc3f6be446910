set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py init --reps 2 "" "stock_floor=1" "stock_floor=2" "stock_floor=3" "stock_floor=2,fill=1" > gpurun_out/s3_init.jsonl 2> gpurun_out/s3_init.err || { echo FAIL1; tail -3 gpurun_out/s3_init.err; exit 1; }
tail -1 gpurun_out/s3_init.jsonl
timeout -k 10 300 python tools/session_rate.py c5 --reps 1 "" "stock_floor=2" > gpurun_out/s3_c5.jsonl 2> gpurun_out/s3_c5.err || { echo FAIL2; exit 1; }
tail -1 gpurun_out/s3_c5.jsonl
timeout -k 10 300 python tools/session_rate.py init --reps 1 "stock_floor=2,log=1" > /dev/null 2> gpurun_out/s3_init_log_floor2.txt || exit 1
timeout -k 10 300 python tools/session_rate.py init --reps 1 "stock_floor=2,fill=1,log=1" > /dev/null 2> gpurun_out/s3_init_log_floor2_fill.txt || exit 1
