#!/bin/bash
# 48 B triangle records (WPT_PRIM48 variant) vs the 64 B product records:
# parity of the variant, then C3 and C5 same-session A/B.
set -o pipefail
WPT_LIB_VARIANT=p48 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "closest_hit or shadow or image_parity or c3_full" > gpurun_out/t_p48.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_p48.log | head; exit 1; }
tail -1 gpurun_out/t_p48.log
AB_STEPS=10 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh base= p48=WPT_LIB_VARIANT=p48 base2= p482=WPT_LIB_VARIANT=p48 || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step" bash tools/ab.sh c5=--config=c5 c5p48=WPT_LIB_VARIANT=p48,--config=c5 || exit 1
echo p48-done
