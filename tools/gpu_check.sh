#!/bin/bash
# GPU check used during development: parity suite, then C3 bench lines for the
# given library variants ("" = the product build). Usage: tools/gpu_check.sh [variant ...]
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in "" "$@"; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/b_$v.json 2>gpurun_out/b_$v.err || { echo BENCHFAIL $v; tail gpurun_out/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_$v.json'));print('[$v]',round(d['value']),round(d['ms_per_step'],2),d['kernel_busy_ms_per_step'],d['work'])"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --opt lanes=1 > gpurun_out/b_l1.json 2>gpurun_out/b_l1.err && python -c "import json;d=json.load(open('gpurun_out/b_l1.json'));print('lanes1',round(d['value']),d['ms_per_step'],d['kernel_launch_ms_per_step'])"
