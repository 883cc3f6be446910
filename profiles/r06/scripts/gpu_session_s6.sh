set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py init --reps 2 "async_cus=0" "async_cus=16" "async_cus=32" "async_cus=64" > gpurun_out/s6_init.jsonl 2> gpurun_out/s6_init.err || { echo FAIL1; tail -3 gpurun_out/s6_init.err; exit 1; }
tail -1 gpurun_out/s6_init.jsonl
timeout -k 10 600 python tools/session_rate.py c5 --reps 1 "async_cus=0" "async_cus=16" "async_cus=32" > gpurun_out/s6_c5.jsonl 2> gpurun_out/s6_c5.err || { echo FAIL2; tail -3 gpurun_out/s6_c5.err; exit 1; }
tail -1 gpurun_out/s6_c5.jsonl
