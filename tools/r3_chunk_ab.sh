#!/bin/bash
# Adaptive rounds: the error copy in 4 pieces summed as they land (product)
# vs one copy then one sum (head = the previous commit). Adaptive / init-
# default parity tests first.
export TMPDIR=/tmp
set -o pipefail
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_comm.py -m gpu -x -q --timeout 300 --timeout-method thread -k "adaptive or init_defaults or random_halves or multirank or transport" > gpurun_out/t_chunk.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_chunk.log | head; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/t_chunk.log
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5head=WPT_LIB_VARIANT=head,--config=c5 c5=--config=c5 c5head2=WPT_LIB_VARIANT=head,--config=c5 c52=--config=c5 || exit 1
for v in head "" head ""; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v]', round(d['Mray/s']), round(d['s'],3))"
done
echo chunk-done
