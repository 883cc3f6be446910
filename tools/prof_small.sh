#!/bin/bash
# Kernel traces of the small-batch workloads: C5 (one step) and the init-default session.
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-serial-step > gpurun_out/prof_c5.log 2>&1 || { echo C5FAIL; tail -5 gpurun_out/prof_c5.log; exit 1; }
python3 tools/timeline.py gpurun_out/prof_c5 > gpurun_out/timeline_c5.json && head -12 gpurun_out/timeline_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ds -o run --output-format csv -- python3 tools/default_session_rate.py 3 > gpurun_out/prof_ds.log 2>&1 || { echo DSFAIL; tail -5 gpurun_out/prof_ds.log; exit 1; }
python3 tools/timeline.py gpurun_out/prof_ds > gpurun_out/timeline_ds.json && head -12 gpurun_out/timeline_ds.json
echo prof-done
