#!/bin/bash
# C5 and the init-default session: fused k_trace (small batches, default) vs
# the separate 7-wave extend/shadow kernels with 2-4 lanes.
set -o pipefail
AB_STEPS=1 AB_ARGS="--no-serial-step --config c5" bash tools/ab.sh base= nf=--opt=fused_below=0 nf4=--opt=fused_below=0,--opt=small_lanes=4 nf3=--opt=fused_below=0,--opt=small_lanes=3 base2= nf4b=--opt=fused_below=0,--opt=small_lanes=4 || exit 1
for o in "" "fused_below=0" "fused_below=0 small_lanes=4" "fused_below=0 small_lanes=3"; do
  timeout -k 10 200 python tools/default_session_rate.py 3 $o > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$o]', round(d['Mray/s']), round(d['s'],3))"
done
echo c5ab2-done
