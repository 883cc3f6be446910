#!/bin/bash
# PNEE neighbour cells from the precomputed per-leaf table (product) vs the
# seven integer walks (notab): C5 and the init-default session.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pnee or photon or adaptive or init_defaults or finish or light_debug" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
AB_STEPS=1 AB_ARGS="--no-serial-step --config c5" bash tools/ab.sh base= notab=WPT_LIB_VARIANT=notab base2= notab2=WPT_LIB_VARIANT=notab || exit 1
for v in "" notab "" notab; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3))"
done
echo tab-done
