set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/session_rate.py c5 --reps 2 "" "stock_ahead=16" "stock_ahead=32" "stock_extra=16" "stock_every=3" > gpurun_out/s36_c5.jsonl 2> gpurun_out/s36_c5.err || { echo FAIL1; tail -3 gpurun_out/s36_c5.err; exit 1; }
tail -1 gpurun_out/s36_c5.jsonl
timeout -k 10 900 python tools/session_rate.py init --reps 3 "" "stock_ahead=16" "stock_extra=16" "stock_every=3" > gpurun_out/s36_init.jsonl 2> gpurun_out/s36_init.err || { echo FAIL2; tail -3 gpurun_out/s36_init.err; exit 1; }
tail -1 gpurun_out/s36_init.jsonl
