# Museum (tori, WPT_TRI_ONLY off) parity subset and A/B for variant $V.
set -o pipefail
timeout -k 10 300 env WPT_LIB_VARIANT=$V python -u -m pytest tests/test_gpu_parity.py -x -q -k "(closest_hit or shadow_query or image_parity) and 0" --timeout 250 --timeout-method thread > gpurun_out/t_$V.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_$V.log | head; exit 1; }
echo $V $(tail -1 gpurun_out/t_$V.log)
AB_STEPS=2 AB_ARGS=--no-secondary bash tools/ab.sh m=--config=museum mv=WPT_LIB_VARIANT=$V,--config=museum m2=--config=museum mv2=WPT_LIB_VARIANT=$V,--config=museum || exit 1
for f in m mv m2 mv2; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
