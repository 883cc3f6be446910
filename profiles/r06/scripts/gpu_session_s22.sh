set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/session_rate.py c2 --reps 3 "" "pixel_tile=4" > gpurun_out/s22_c2.jsonl 2> gpurun_out/s22_c2.err || { echo FAIL1; tail -3 gpurun_out/s22_c2.err; exit 1; }
tail -1 gpurun_out/s22_c2.jsonl
timeout -k 10 900 python tools/session_rate.py museum --reps 3 "" "pixel_tile=4" > gpurun_out/s22_museum.jsonl 2> gpurun_out/s22_museum.err || { echo FAIL2; tail -3 gpurun_out/s22_museum.err; exit 1; }
tail -1 gpurun_out/s22_museum.jsonl
