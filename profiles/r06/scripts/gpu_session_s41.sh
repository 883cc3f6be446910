set -o pipefail
bash tools/gpu_final.sh r06c || exit 1
timeout -k 10 600 python tools/session_rate.py init --reps 3 "" "stock_every=3" "async_grid_pct=60" "finish_every=6" > gpurun_out/s41_init.jsonl 2> gpurun_out/s41_init.err || { echo FAIL2; tail -3 gpurun_out/s41_init.err; exit 1; }
tail -1 gpurun_out/s41_init.jsonl
