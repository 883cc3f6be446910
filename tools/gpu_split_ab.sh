# GPU suite, then a same-session A/B of the split traversal step (product) vs
# the combined step (variant old, WPT_SPLIT_STEP=0), C3 and C5.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/t_split.log 2>&1; rc=$?
tail -1 gpurun_out/t_split.log; grep -E "^FAILED|^E " gpurun_out/t_split.log | head -20
[ $rc -eq 0 ] || exit 1
AB_STEPS=4 bash tools/ab.sh new= old=WPT_LIB_VARIANT=old new2= old2=WPT_LIB_VARIANT=old c5=--config=c5 c5old=WPT_LIB_VARIANT=old,--config=c5
for f in new old new2 old2 c5 c5old; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'])"; done
