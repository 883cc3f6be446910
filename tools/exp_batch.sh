set -e
for b in 33554432 67108864 134217728; do
  echo "== batch $b"
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch $b 2>/dev/null | python3 -c "
import json,sys
d=json.loads(sys.stdin.readlines()[-1]); ms=d['ms_per_step']
print(round(d['value'],1), 'Mray/s', round(ms,1), 'ms/step', d['kernel_busy_ms_per_step'])"
done
