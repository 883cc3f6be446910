#!/bin/bash
# C5: product (PNEE shade at 6 waves) vs pnee5 variant; init defaults at larger k_finish thresholds.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pnee or adaptive or photon or finish or init_defaults" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
for v in "" pnee5 "" pnee5; do
  WPT_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 1 --no-serial-step > gpurun_out/c5_$v.json 2>gpurun_out/c5_$v.err || { echo C5FAIL; tail -3 gpurun_out/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5_$v.json'));print('c5 [$v]',round(d['value']),round(d['ms_per_step'],1),d['kernel_busy_ms_per_step'])"
done
for fb in 524288 1048576 2097152 4194304; do
  timeout -k 10 200 python tools/default_session_rate.py 3 finish_below=$fb > gpurun_out/ds_fb$fb.json 2>gpurun_out/ds_fb$fb.err || { echo DSFAIL; tail -3 gpurun_out/ds_fb$fb.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds_fb$fb.json'));print('fb $fb', round(d['Mray/s']), round(d['s'],3))"
done
echo ab2-done
