set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py init --reps 2 "" "fill=1" > gpurun_out/s24_init_q4.jsonl 2> gpurun_out/s24_init_q4.err || { echo FAIL0; tail -3 gpurun_out/s24_init_q4.err; exit 1; }
tail -1 gpurun_out/s24_init_q4.jsonl
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python tools/session_rate.py init --reps 2 "" "fill=1" > gpurun_out/s24_init_q8.jsonl 2> gpurun_out/s24_init_q8.err || { echo FAIL1; tail -3 gpurun_out/s24_init_q8.err; exit 1; }
tail -1 gpurun_out/s24_init_q8.jsonl
