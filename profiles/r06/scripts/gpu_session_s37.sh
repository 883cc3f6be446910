set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/session_rate.py init --reps 2 "stock_every=3,log=1" > gpurun_out/s37_init.jsonl 2> gpurun_out/s37_log.txt || { echo FAIL1; tail -3 gpurun_out/s37_log.txt; exit 1; }
tail -1 gpurun_out/s37_init.jsonl
