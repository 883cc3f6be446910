#!/bin/bash
# fused k_trace forced to 7 waves/SIMD (12 B scratch, SGPR spills) vs the
# compiler's 6: C5 and the init-default session.
set -o pipefail
WPT_LIB_VARIANT=kt7 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused or adaptive or init_defaults" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
AB_STEPS=1 AB_ARGS="--no-serial-step --config c5" bash tools/ab.sh base= kt7=WPT_LIB_VARIANT=kt7 base2= kt72=WPT_LIB_VARIANT=kt7 || exit 1
for v in "" kt7 "" kt7; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3))"
done
echo kt7-done
