# Parity subsets on variants pk (packed box test, pair-friendly node layout)
# and pt3 (pk + packed triangle test), then a same-session A/B, C3 and C5.
set -o pipefail
for v in pk pt3; do
  timeout -k 10 300 env WPT_LIB_VARIANT=$v python -u -m pytest tests/test_gpu_parity.py -x -q -k "closest_hit or shadow_query or image_parity or c5_settings" --timeout 250 --timeout-method thread > gpurun_out/t_$v.log 2>&1 || { echo TESTFAIL $v; grep -E "^FAILED|^E " gpurun_out/t_$v.log | head; exit 1; }
  echo $v $(tail -1 gpurun_out/t_$v.log)
done
AB_STEPS=4 AB_ARGS=--no-secondary bash tools/ab.sh base= pk=WPT_LIB_VARIANT=pk pt3=WPT_LIB_VARIANT=pt3 base2= pk2=WPT_LIB_VARIANT=pk pt32=WPT_LIB_VARIANT=pt3 c5=--config=c5 c5k=WPT_LIB_VARIANT=pk,--config=c5 c5t=WPT_LIB_VARIANT=pt3,--config=c5 || exit 1
for f in base pk pt3 base2 pk2 pt32 c5 c5k c5t; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
