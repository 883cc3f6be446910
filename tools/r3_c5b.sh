#!/bin/bash
# C5 / init-default session after the round-planning changes (tiled error
# estimate + hierarchical min/max, segment sum on the host), then a kernel
# trace of one C5 step for the timeline.
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adaptive or init_defaults or pnee or multirank or finish" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 1 --no-serial-step > gpurun_out/c5_$r.json 2>gpurun_out/c5_$r.err || { echo C5FAIL; tail -3 gpurun_out/c5_$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5_$r.json'));print('c5',round(d['value']),round(d['ms_per_step'],1),d['kernel_busy_ms_per_step'])"
  timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds_$r.json 2>gpurun_out/ds_$r.err || { echo DSFAIL; tail -3 gpurun_out/ds_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds_$r.json'));print('default', round(d['Mray/s']), round(d['s'],3))"
done
rm -rf gpurun_out/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step --no-secondary > gpurun_out/prof_c5.log 2>&1 || { echo PROFFAIL; tail -5 gpurun_out/prof_c5.log; exit 1; }
python3 tools/timeline.py gpurun_out/prof_c5 > gpurun_out/timeline_c5.json && head -4 gpurun_out/timeline_c5.json
echo c5b-done
