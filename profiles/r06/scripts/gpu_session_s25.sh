set -o pipefail
mkdir -p gpurun_out
for V in glds glds7; do
timeout -k 10 300 env WPT_LIB_VARIANT=$V python -u -m pytest tests/test_gpu_parity.py -x -q -k "image_parity or c5_settings or finish_tail" --timeout 250 --timeout-method thread > gpurun_out/t_$V.log 2>&1 || { echo TESTFAIL $V; grep -E "^FAILED|^E " gpurun_out/t_$V.log | head; exit 1; }
echo $V $(tail -1 gpurun_out/t_$V.log)
done
AB_STEPS=8 AB_ARGS="--no-secondary" bash tools/ab.sh base= v=WPT_LIB_VARIANT=glds v7=WPT_LIB_VARIANT=glds7 base2= v2=WPT_LIB_VARIANT=glds v72=WPT_LIB_VARIANT=glds7 || exit 1
for f in base v v7 base2 v2 v72; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
