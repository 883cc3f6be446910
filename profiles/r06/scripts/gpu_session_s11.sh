set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py init --reps 2 "finish_coop=0" "finish_coop=1" "finish_below=16384,finish_coop=0" "finish_below=16384,finish_coop=1" "finish_below=65536,finish_coop=1" > gpurun_out/s11_init.jsonl 2> gpurun_out/s11_init.err || { echo FAIL1; tail -3 gpurun_out/s11_init.err; exit 1; }
tail -1 gpurun_out/s11_init.jsonl
