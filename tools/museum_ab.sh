#!/bin/bash
# Same-session A/B of the museum scene (scene 0) bench line. Arguments are
# library variants ("" = the product build). Usage: tools/museum_ab.sh "" tc
set -o pipefail
for v in "$@"; do
  WPT_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config museum --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/m_$v.json 2> gpurun_out/m_$v.err || { echo FAIL $v; tail -3 gpurun_out/m_$v.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/m_$v.json').read().strip().splitlines()[-1]);print('museum [$v]', round(d['value']), round(d['ms_per_step'],1), d['kernel_busy_ms_per_step'])"
done
