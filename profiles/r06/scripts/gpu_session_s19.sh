set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/session_rate.py c3 --reps 2 "" "pixel_tile=4" "pixel_tile=16" "pixel_tile=32" > gpurun_out/s19_c3.jsonl 2> gpurun_out/s19_c3.err || { echo FAIL1; tail -3 gpurun_out/s19_c3.err; exit 1; }
tail -1 gpurun_out/s19_c3.jsonl
