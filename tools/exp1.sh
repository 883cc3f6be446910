# A/B runs of bench.py: tools/exp1.sh "label ENV=val ..." ...
set -e
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
for spec in "$@"; do
  set -- $spec
  label=$1; shift
  echo "== $label"
  env "$@" timeout -k 10 200 $B 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.readlines()[-1]); w=d['work']; ms=d['ms_per_step']
print(round(d['value'],1), 'Mray/s', round(ms,1), 'ms/step', d['kernel_busy_ms_per_step'],
      'ext_live', round(w['ext_loop_live_frac'],3), 'sh_live', round(w['sh_loop_live_frac'],3))"
done
