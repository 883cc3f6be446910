set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/session_rate.py c5 --reps 1 "" "grid_pct=75" "grid_pct=100" "fused_below=67108864" "fused_below=67108864,trace_grid_pct=100" "small_lanes=1" > gpurun_out/s12_c5.jsonl 2> gpurun_out/s12_c5.err || { echo FAIL1; tail -3 gpurun_out/s12_c5.err; exit 1; }
tail -1 gpurun_out/s12_c5.jsonl
