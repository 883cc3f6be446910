#!/bin/bash
# Packed-f32 check, parity subset on the pair-layout build without SLP
# vectorisation, then same-session C3 / C5 A/B of the node layout (aos / soa)
# x SLP vectoriser (on / ns = -fno-slp-vectorize), 8 waves (soans8) and the
# branch-free triangle test (bf, bf8).
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 60 ./tools/pk_denorm_check || { echo PKFAIL; exit 1; }
for v in soans bf; do
WPT_LIB_VARIANT=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "image_parity or closest_hit or shadow or museum or finish" > gpurun_out/t_pk_$v.log 2>&1 || { echo TESTFAIL $v; grep -E "^FAILED|^E " gpurun_out/t_pk_$v.log | head; exit 1; }
echo $v; tail -1 gpurun_out/t_pk_$v.log
done
AB_STEPS=8 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh aos=WPT_LIB_VARIANT=aos aosns=WPT_LIB_VARIANT=aosns soa=WPT_LIB_VARIANT=soa soans=WPT_LIB_VARIANT=soans soans8=WPT_LIB_VARIANT=soans8 bf=WPT_LIB_VARIANT=bf bf8=WPT_LIB_VARIANT=bf8 aos2=WPT_LIB_VARIANT=aos soans2=WPT_LIB_VARIANT=soans || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5aos=WPT_LIB_VARIANT=aos,--config=c5 c5soans=WPT_LIB_VARIANT=soans,--config=c5 c5soans8=WPT_LIB_VARIANT=soans8,--config=c5 c5bf=WPT_LIB_VARIANT=bf,--config=c5 c5bf8=WPT_LIB_VARIANT=bf8,--config=c5 || exit 1
echo pk-done
