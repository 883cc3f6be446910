#!/bin/bash
# init-default session: k_finish occupancy (compiler 4 waves vs 5 / 6 forced
# with spills) and the threshold 2^18 vs 2^19.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "finish or init_defaults" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
for r in 1 2; do
for v in "" fw5 fw6; do
  for fb in 524288 262144; do
    WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 finish_below=$fb > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('default [$v] fb $fb', round(d['Mray/s']), round(d['s'],3), d['finish_paths'], d['finish_max_bounces'])"
  done
done
done
echo fin-done
