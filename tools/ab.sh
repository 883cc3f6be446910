#!/bin/bash
# Same-session A/B of C3 bench lines. Each argument is NAME=SPEC, SPEC a
# comma-separated list of env assignments (WPT_LIB_VARIANT=<v>: an experiment
# build, csrc/Makefile `variant`) and bench options (--opt=traversal=bvh4,
# --config=c5, ...); "base=" runs the product as is.
# Usage: tools/ab.sh [--tests] base= name=SPEC ...   (AB_STEPS, AB_ARGS: extra bench args for all)
set -o pipefail
if [ "$1" == "--tests" ]; then
  shift
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head -20; exit 1; }
  tail -1 gpurun_out/t.log
fi
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}
  envs=(); bargs=()
  IFS=',' read -ra toks <<< "$rest"
  for t in "${toks[@]}"; do
    [ -z "$t" ] && continue
    if [[ $t == --* ]]; then bargs+=("${t%%=*}" "${t#*=}"); else envs+=("$t"); fi
  done
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${AB_STEPS:-5} $AB_ARGS "${bargs[@]}" > gpurun_out/ab_$name.json 2>gpurun_out/ab_$name.err || { echo BENCHFAIL $name; tail -5 gpurun_out/ab_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));w=d['work'];print('$name',round(d['value']),round(d['ms_per_step'],2),d['kernel_busy_ms_per_step'],'visits/ray %.2f steps/ray %.2f live %.2f sh %.2f/%.2f'%(w['node_visits_per_ray'],w['ext_steps_per_ray'],w['ext_loop_live_frac'],w['sh_steps_per_ray'],w['sh_loop_live_frac']))"
done
