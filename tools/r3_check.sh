#!/bin/bash
# GPU suite, then the default bench line (C3 + cpu baseline + secondary configs).
set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head -20; tail -3 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo BENCHFAIL; tail -5 gpurun_out/bench_full.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_full.json'))
print('C3', round(d['value']), round(d['ms_per_step'],2), d['kernel_busy_ms_per_step'], d.get('parity'))
for k,v in d.get('secondary',{}).items(): print(k, round(v['value']), round(v['ms_per_step'],1), v['parity'])
print('secondary_s', d.get('secondary_s'))"
echo check-done
