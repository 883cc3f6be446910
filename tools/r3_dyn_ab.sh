#!/bin/bash
# Work feed: static share + per-XCD claimed blocks (dyn: 75 % static, dyn50:
# 50 %) vs the static wave-interleaved feed (base); museum kernels at 6 waves
# (any6). Parity subset on dyn first.
export TMPDIR=/tmp
set -o pipefail
WPT_LIB_VARIANT=dyn timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_comm.py tests/test_gpu_bvh_build.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_dyn.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_dyn.log | head; exit 1; }
tail -1 gpurun_out/t_dyn.log
AB_STEPS=8 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh base= dyn=WPT_LIB_VARIANT=dyn dyn50=WPT_LIB_VARIANT=dyn50 base2= dyn2=WPT_LIB_VARIANT=dyn || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5=--config=c5 c5dyn=WPT_LIB_VARIANT=dyn,--config=c5 c5dyn50=WPT_LIB_VARIANT=dyn50,--config=c5 c5dyn50g75=WPT_LIB_VARIANT=dyn50,--config=c5,--opt=trace_grid_pct=75 || exit 1
AB_STEPS=2 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh mus=--config=museum mus_any6=WPT_LIB_VARIANT=any6,--config=museum mus_dyn=WPT_LIB_VARIANT=dyn,--config=museum || exit 1
for v in "" dyn50 "" dyn50; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3))"
done
echo dyn-done
