#!/bin/bash
# GPU suite, then the init-default session at several k_finish thresholds and C5.
set -o pipefail
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head -20; tail -3 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for fb in 0 16384 65536 131072 524288; do
  timeout -k 10 200 python tools/default_session_rate.py 3 finish_below=$fb > gpurun_out/ds_fb$fb.json 2>gpurun_out/ds_fb$fb.err || { echo DSFAIL; tail -3 gpurun_out/ds_fb$fb.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds_fb$fb.json'));print('fb $fb', round(d['Mray/s']), round(d['s'],3))"
done
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 1 --no-serial-step > gpurun_out/c5.json 2>gpurun_out/c5.err || { echo C5FAIL; tail -3 gpurun_out/c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5.json'));print('c5',round(d['value']),round(d['ms_per_step'],1),d['kernel_busy_ms_per_step'])"
echo ab-done
