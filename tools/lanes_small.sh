#!/bin/bash
# Same-session A/B on the small-batch workloads (C5 adaptive rounds and the
# init-default session). Each argument is NAME=ENV (space-separated
# assignments, e.g. "sl2=WPT_SMALL_LANES=2"); "base=" runs the product as is.
set -o pipefail
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-serial-step --steps 2 --warmup 1 > gpurun_out/c5_$name.json 2> gpurun_out/c5_$name.err || { echo FAIL c5 $name; tail -5 gpurun_out/c5_$name.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c5_$name.json').read().strip().splitlines()[-1]);print('c5 $name', round(d['value']), 'Mray/s', round(d['ms_per_step'],1), 'ms/step')"
  env $envs timeout -k 10 300 python tools/default_session_rate.py 4 > gpurun_out/ds_$name.json 2> gpurun_out/ds_$name.err || { echo FAIL ds $name; tail -5 gpurun_out/ds_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ds_$name.json'));print('init-defaults $name', round(d['Mray/s']), 'Mray/s')"
done
