#!/bin/bash
# Register-resident stack top (rt) vs the stack wholly in LDS (rt0): parity
# subset on rt, then C3 / C5 / museum / init-default session A/B.
export TMPDIR=/tmp
set -o pipefail
WPT_LIB_VARIANT=rt timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c4" > gpurun_out/t_rt.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_rt.log | head; exit 1; }
tail -1 gpurun_out/t_rt.log
AB_STEPS=8 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh rt0=WPT_LIB_VARIANT=rt0 rt=WPT_LIB_VARIANT=rt rt02=WPT_LIB_VARIANT=rt0 rt2=WPT_LIB_VARIANT=rt || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5rt0=WPT_LIB_VARIANT=rt0,--config=c5 c5rt=WPT_LIB_VARIANT=rt,--config=c5 || exit 1
AB_STEPS=2 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh mus_rt0=WPT_LIB_VARIANT=rt0,--config=museum mus_rt=WPT_LIB_VARIANT=rt,--config=museum || exit 1
for v in rt0 rt rt0 rt; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3))"
done
echo rt-done
