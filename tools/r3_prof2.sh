#!/bin/bash
# Round-3 C3 profile (kernel trace + PMC passes), then C5-shaped sessions
# with PNEE vs uniform NEE on both halves (the PNEE light pick's price).
set -o pipefail
bash tools/profile.sh r03 || exit 1
for t in "2 2" "1 1"; do
  timeout -k 10 300 python tools/c5_types.py $t > gpurun_out/c5t.json 2>gpurun_out/c5t.err || { echo C5TFAIL; tail -3 gpurun_out/c5t.err; exit 1; }
  cat gpurun_out/c5t.json
done
echo prof2-done
