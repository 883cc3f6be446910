# Parity subset for variant $V, then a same-session A/B: C2 (no BVH: the
# linear scan) and C3, twice each.
set -o pipefail
timeout -k 10 300 env WPT_LIB_VARIANT=$V python -u -m pytest tests/test_gpu_parity.py -x -q -k "closest_hit or shadow_query or image_parity" --timeout 250 --timeout-method thread > gpurun_out/t_$V.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_$V.log | head; exit 1; }
echo $V $(tail -1 gpurun_out/t_$V.log)
AB_STEPS=3 AB_ARGS=--no-secondary bash tools/ab.sh c2=--config=c2 c2v=WPT_LIB_VARIANT=$V,--config=c2 base= v=WPT_LIB_VARIANT=$V c22=--config=c2 c2v2=WPT_LIB_VARIANT=$V,--config=c2 base2= v2=WPT_LIB_VARIANT=$V || exit 1
for f in c2 c2v base v c22 c2v2 base2 v2; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
