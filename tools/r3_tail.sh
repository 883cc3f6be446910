#!/bin/bash
# k_finish tail statistics of the init-default session at a few thresholds.
set -o pipefail
for fb in 524288 262144 131072; do
  timeout -k 10 200 python tools/default_session_rate.py 3 finish_below=$fb > gpurun_out/ds.json 2>gpurun_out/ds.err || { echo DSFAIL; tail -3 gpurun_out/ds.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ds.json'));print('fb $fb', round(d['Mray/s']), round(d['s'],3), d['finish_paths'], d['finish_max_bounces'])"
done
echo tail-done
