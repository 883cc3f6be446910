set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python tools/session_rate.py c3 --reps 5 "" "refill=10" "refill=14" "refill_sh=12" "refill_sh=20" "grid_pct=45" "grid_pct=55" > gpurun_out/s28_c3.jsonl 2> gpurun_out/s28_c3.err || { echo FAIL1; tail -3 gpurun_out/s28_c3.err; exit 1; }
tail -1 gpurun_out/s28_c3.jsonl
