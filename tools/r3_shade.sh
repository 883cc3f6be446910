#!/bin/bash
# k_shade: the hit normal's loads issued with the material's and the light
# records from LDS (product) vs the previous commit ("head"): C3, C5, museum.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
AB_STEPS=10 AB_ARGS="--no-secondary" bash tools/ab.sh base= head=WPT_LIB_VARIANT=head base2= head2=WPT_LIB_VARIANT=head || exit 1
python3 -c "
import json
for n in ('base','head'):
    d=json.load(open('gpurun_out/ab_'+n+'.json')); print(n, 'serial', d['kernel_serial_ms_per_step'])"
AB_STEPS=1 AB_ARGS="--no-serial-step --config c5" bash tools/ab.sh c5= c5head=WPT_LIB_VARIANT=head || exit 1
AB_STEPS=2 AB_ARGS="--no-serial-step --config museum" bash tools/ab.sh mus= mushead=WPT_LIB_VARIANT=head || exit 1
echo shade-done
