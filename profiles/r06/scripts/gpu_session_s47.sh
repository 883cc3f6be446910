set -o pipefail
timeout -k 10 600 python tools/session_rate.py init --reps 6 "" "stock_ahead=40" "stock_ahead=32,stock_extra=16" "stock_ahead=40,stock_extra=16" > gpurun_out/s47_init.jsonl 2> gpurun_out/s47_init.err || { echo FAIL2; tail -3 gpurun_out/s47_init.err; exit 1; }
tail -1 gpurun_out/s47_init.jsonl
timeout -k 10 600 python tools/session_rate.py c5 --reps 3 "stock_ahead=40" "stock_ahead=40,stock_extra=16" > gpurun_out/s47_c5.jsonl 2> gpurun_out/s47_c5.err || { echo FAIL1; tail -3 gpurun_out/s47_c5.err; exit 1; }
tail -1 gpurun_out/s47_c5.jsonl
