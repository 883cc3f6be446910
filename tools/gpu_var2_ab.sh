# Parity subset on variant $V, then a same-session C3 A/B: product, $V, the
# product without the LDS treelet; twice each.
set -o pipefail
timeout -k 10 300 env WPT_LIB_VARIANT=$V python -u -m pytest tests/test_gpu_parity.py -x -q -k "closest_hit or shadow_query or image_parity or c5_settings" --timeout 250 --timeout-method thread > gpurun_out/t_$V.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_$V.log | head; exit 1; }
echo $V $(tail -1 gpurun_out/t_$V.log)
AB_STEPS=4 AB_ARGS=--no-secondary bash tools/ab.sh base= v=WPT_LIB_VARIANT=$V nt=--opt=treelet=0 base2= v2=WPT_LIB_VARIANT=$V nt2=--opt=treelet=0 || exit 1
for f in base v nt base2 v2 nt2; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
