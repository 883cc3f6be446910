#!/bin/bash
# Init-default session: k_finish at 5 waves (fin5) vs the compiler's 4, and
# the k_finish threshold re-tuned on the 8-wave build.
export TMPDIR=/tmp
set -o pipefail
WPT_LIB_VARIANT=fin5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "finish or init_defaults or adaptive" > gpurun_out/t_fin5.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_fin5.log | head; exit 1; }
tail -1 gpurun_out/t_fin5.log
run() {
  WPT_LIB_VARIANT=$1 timeout -k 10 200 python tools/default_session_rate.py 3 $2 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$1 $2]', round(d['Mray/s']), round(d['s'],3), d['finish_paths'], d['finish_max_bounces'])"
}
run "" "" && run fin5 "" && run "" "" && run fin5 "" && run "" finish_below=131072 && run "" finish_below=524288 && run fin5 finish_below=524288 && run "" "" || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5=--config=c5 c5sep=--config=c5,--opt=fused_below=0 c5fin5=WPT_LIB_VARIANT=fin5,--config=c5 || exit 1
echo fin-done
