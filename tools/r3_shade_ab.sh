#!/bin/bash
# k_shade's persistent grid from the launched variant's own occupancy (shv)
# vs the smallest occupancy of all variants (shv0); shv8: + NEE shade forced
# to 8 waves; shb128: 128-thread shade blocks (old grid rule).
export TMPDIR=/tmp
set -o pipefail
WPT_LIB_VARIANT=shv timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "image_parity or museum or adaptive or finish or lanes" > gpurun_out/t_shv.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_shv.log | head; exit 1; }
tail -1 gpurun_out/t_shv.log
AB_STEPS=8 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh shv0=WPT_LIB_VARIANT=shv0 shv=WPT_LIB_VARIANT=shv shv8=WPT_LIB_VARIANT=shv8 shb128=WPT_LIB_VARIANT=shb128 shv02=WPT_LIB_VARIANT=shv0 shv2=WPT_LIB_VARIANT=shv || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5shv0=WPT_LIB_VARIANT=shv0,--config=c5 c5shv=WPT_LIB_VARIANT=shv,--config=c5 || exit 1
AB_STEPS=2 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh mus_shv0=WPT_LIB_VARIANT=shv0,--config=museum mus_shv=WPT_LIB_VARIANT=shv,--config=museum || exit 1
for v in shv0 shv shv0 shv; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3))"
done
echo shade-done
