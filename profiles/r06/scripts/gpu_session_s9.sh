set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python tools/session_rate.py c3 --reps 2 "" "fused=1" "fused=1,trace_grid_pct=50" > gpurun_out/s9_c3.jsonl 2> gpurun_out/s9_c3.err || { echo FAIL1; tail -3 gpurun_out/s9_c3.err; exit 1; }
tail -1 gpurun_out/s9_c3.jsonl
