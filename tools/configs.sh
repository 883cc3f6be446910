#!/bin/bash
# Bench lines of the other configs on one GPU (no CPU baseline): C1, C2, museum, C5, C4.
set -o pipefail
for c in ${@:-c1 c2 museum c5 c4}; do
  steps=3; [ $c == c4 ] && steps=1; [ $c == c1 ] && steps=20
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps $steps --warmup 1 > gpurun_out/cfg_$c.json 2> gpurun_out/cfg_$c.err || { echo FAIL $c; tail -5 gpurun_out/cfg_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/cfg_$c.json').read().strip().splitlines()[-1]);print('$c', round(d['value']), 'Mray/s', round(d['ms_per_step'],2), 'ms/step', d['kernel_busy_ms_per_step'])"
done
