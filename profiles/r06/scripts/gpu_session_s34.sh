set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/session_rate.py init --reps 8 "" "finish_every=3" > gpurun_out/s34_init.jsonl 2> gpurun_out/s34_init.err || { echo FAIL1; tail -3 gpurun_out/s34_init.err; exit 1; }
tail -1 gpurun_out/s34_init.jsonl
