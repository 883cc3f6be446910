# Round 5, thirty-sixth GPU session: the fused k_trace's grid at 75 % of the
# resident capacity as the default (variant tg75; session 32: +1 % on C5 in
# one run): C5 three times each and the C3 line (secondary: C5, init defaults).
set -o pipefail
AB_STEPS=4 bash tools/ab.sh c5=--config=c5 t1=WPT_LIB_VARIANT=tg75,--config=c5 c5b=--config=c5 t2=WPT_LIB_VARIANT=tg75,--config=c5 c5c=--config=c5 t3=WPT_LIB_VARIANT=tg75,--config=c5 base= v=WPT_LIB_VARIANT=tg75 || exit 1
mkdir -p gpurun_out/r05/tg75
for n in c5 t1 c5b t2 c5c t3 base v; do cp gpurun_out/ab_$n.json gpurun_out/r05/tg75/; done
python -c "
import json
for n in ['base','v']:
    d=json.load(open('gpurun_out/r05/tg75/ab_'+n+'.json')); print(n, round(d['value']), {k:round(x['value']) for k,x in (d.get('secondary') or {}).items()})
"
