#!/bin/bash
# Round-3 C3 profile (kernel trace + SQ / FETCH_SIZE / WRITE_SIZE / TCC
# passes), summarised on the box (the raw traces exceed gpurun_out's limit):
# profiles/r03/c3_{kernel_stats.csv,pmc_summary.json,trace.log,args.txt} and
# profiles/traffic_c3.json, copied to gpurun_out/collected/.
set -o pipefail
bash tools/profile.sh r03 || exit 1
python3 tools/collect_profile.py gpurun_out/prof_r03 r03 c3 134217728 64 bvh2 4 > gpurun_out/collect.log 2>&1 || { tail -5 gpurun_out/collect.log; exit 1; }
mkdir -p gpurun_out/collected
cp profiles/r03/c3_* profiles/traffic_c3.json gpurun_out/collected/
rm -rf gpurun_out/prof_r03
ls gpurun_out/collected
echo prof3-done
