# Parity subset on variant $V (all three traversals), then a same-session A/B
# against the product: C3 twice, C5 once. Usage: V=name bash tools/gpu_var_ab.sh
set -o pipefail
timeout -k 10 300 env WPT_LIB_VARIANT=$V python -u -m pytest tests/test_gpu_parity.py -x -q -k "closest_hit or shadow_query or image_parity or c5_settings" --timeout 250 --timeout-method thread > gpurun_out/t_$V.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_$V.log | head; exit 1; }
echo $V $(tail -1 gpurun_out/t_$V.log)
AB_STEPS=4 bash tools/ab.sh base= v=WPT_LIB_VARIANT=$V base2= v2=WPT_LIB_VARIANT=$V c5=--config=c5 c5v=WPT_LIB_VARIANT=$V,--config=c5 || exit 1
for f in base v base2 v2 c5 c5v; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'],{k:round(x['value']) for k,x in (d.get('secondary') or {}).items()})"; done
