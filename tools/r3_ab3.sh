#!/bin/bash
# Branch-free leaf accept (product) vs branchy (acc0); k_finish tracing each
# bounce's shadow ray with the next extension ray (product) vs one after the
# other (fin1).
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "finish or image_parity or closest_hit or shadow or c3_full or init_defaults or adaptive" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
AB_STEPS=10 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh base= acc0=WPT_LIB_VARIANT=acc0 base2= acc02=WPT_LIB_VARIANT=acc0 || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step" bash tools/ab.sh c5=--config=c5 c5acc0=WPT_LIB_VARIANT=acc0,--config=c5 || exit 1
for v in "" fin1 "" fin1; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3), d['finish_paths'], d['finish_max_bounces'])"
done
echo ab3-done
