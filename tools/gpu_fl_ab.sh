# Parity subset on variant fl (one flat load site for treelet and global node
# pairs), then a same-session A/B: C3 (plus refill 10 / 14 on the product) and C5.
set -o pipefail
timeout -k 10 300 env WPT_LIB_VARIANT=fl python -u -m pytest tests/test_gpu_parity.py -x -q -k "closest_hit or shadow_query or image_parity or c5_settings" --timeout 250 --timeout-method thread > gpurun_out/t_fl.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_fl.log | head; exit 1; }
echo fl $(tail -1 gpurun_out/t_fl.log)
AB_STEPS=4 AB_ARGS=--no-secondary bash tools/ab.sh base= fl=WPT_LIB_VARIANT=fl r10=--opt=refill=10 base2= fl2=WPT_LIB_VARIANT=fl r14=--opt=refill=14 c5=--config=c5 c5f=WPT_LIB_VARIANT=fl,--config=c5 || exit 1
for f in base fl r10 base2 fl2 r14 c5 c5f; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
