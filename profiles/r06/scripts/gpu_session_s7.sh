set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/session_rate.py init --reps 1 "stock=0,log=1" "log=1" > gpurun_out/s7_init.jsonl 2> gpurun_out/s7_init_log.txt || { echo FAIL1; tail -3 gpurun_out/s7_init_log.txt; exit 1; }
cat gpurun_out/s7_init.jsonl
