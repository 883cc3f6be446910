set -o pipefail
timeout -k 10 600 python tools/session_rate.py c5 --reps 3 "" "stock_lanes=3" "stock_ahead=36" "stock_ahead=44" > gpurun_out/s50_c5.jsonl 2> gpurun_out/s50_c5.err || { echo FAIL1; tail -3 gpurun_out/s50_c5.err; exit 1; }
tail -1 gpurun_out/s50_c5.jsonl
timeout -k 10 600 python tools/session_rate.py init --reps 4 "" "stock_lanes=3" > gpurun_out/s50_init.jsonl 2> gpurun_out/s50_init.err || { echo FAIL2; tail -3 gpurun_out/s50_init.err; exit 1; }
tail -1 gpurun_out/s50_init.jsonl
