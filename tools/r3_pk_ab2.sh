#!/bin/bash
# Round 2 of the no-SLP A/B: pair layout (bf8) vs node layout (abf8), both
# with the branch-free triangle test and 8-wave traversal kernels; *f: the
# fused k_trace at 8 waves too. aos = the round's starting point.
export TMPDIR=/tmp
set -o pipefail
WPT_LIB_VARIANT=abf8f timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "image_parity or closest_hit or shadow or museum or finish or adaptive" > gpurun_out/t_pk_abf8f.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_pk_abf8f.log | head; exit 1; }
tail -1 gpurun_out/t_pk_abf8f.log
AB_STEPS=8 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh aos=WPT_LIB_VARIANT=aos bf8=WPT_LIB_VARIANT=bf8 abf8=WPT_LIB_VARIANT=abf8 aos2=WPT_LIB_VARIANT=aos bf82=WPT_LIB_VARIANT=bf8 abf82=WPT_LIB_VARIANT=abf8 || exit 1
AB_STEPS=2 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh mus_aos=WPT_LIB_VARIANT=aos,--config=museum mus_abf8=WPT_LIB_VARIANT=abf8,--config=museum || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5aos=WPT_LIB_VARIANT=aos,--config=c5 c5bf8=WPT_LIB_VARIANT=bf8,--config=c5 c5bf8f=WPT_LIB_VARIANT=bf8f,--config=c5 c5abf8=WPT_LIB_VARIANT=abf8,--config=c5 c5abf8f=WPT_LIB_VARIANT=abf8f,--config=c5 || exit 1
for v in aos abf8 abf8f aos abf8f; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3))"
done
echo ab2-done
