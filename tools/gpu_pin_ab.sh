# Parity subset on the variants, then a same-session A/B (C3, C5, museum via
# the secondary block of the base lines): pt = tuple pinning, s2 = pt + step2.
set -o pipefail
for v in pt s2; do
  timeout -k 10 300 env WPT_LIB_VARIANT=$v python -u -m pytest tests/test_gpu_parity.py -x -q -k "closest_hit or shadow_query or image_parity" --timeout 250 --timeout-method thread > gpurun_out/t_$v.log 2>&1 || { echo TESTFAIL $v; grep -E "^FAILED|^E " gpurun_out/t_$v.log | head; exit 1; }
  echo $v $(tail -1 gpurun_out/t_$v.log)
done
AB_STEPS=4 bash tools/ab.sh base= pt=WPT_LIB_VARIANT=pt s2=WPT_LIB_VARIANT=s2 base2= pt2=WPT_LIB_VARIANT=pt s22=WPT_LIB_VARIANT=s2 c5=--config=c5 c5s=WPT_LIB_VARIANT=s2,--config=c5 || exit 1
for f in base pt s2 base2 pt2 s22 c5 c5s; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
