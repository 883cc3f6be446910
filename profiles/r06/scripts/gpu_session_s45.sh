set -o pipefail
timeout -k 10 600 python tools/session_rate.py c5 --reps 3 "" "stock_every=4" "stock_ahead=32" > gpurun_out/s45_c5.jsonl 2> gpurun_out/s45_c5.err || { echo FAIL1; tail -3 gpurun_out/s45_c5.err; exit 1; }
tail -1 gpurun_out/s45_c5.jsonl
timeout -k 10 600 python tools/session_rate.py init --reps 5 "" "stock_every=4" "stock_ahead=32" > gpurun_out/s45_init.jsonl 2> gpurun_out/s45_init.err || { echo FAIL2; tail -3 gpurun_out/s45_init.err; exit 1; }
tail -1 gpurun_out/s45_init.jsonl
