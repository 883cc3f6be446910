# Round 5, twenty-first GPU session: the device error sum with the chunks the
# host walk re-sums packed on the device (k_sum_pack) instead of copying all
# errors; on-demand copies for any other. The GPU suite, then C5 twice and the
# C3 line (secondary: C5, init defaults) against variant hsum (host sum).
set -o pipefail
mkdir -p gpurun_out/r05/dsum2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/dsum2/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/dsum2/tests.log; exit 1; }
tail -1 gpurun_out/r05/dsum2/tests.log
AB_STEPS=4 bash tools/ab.sh c5=--config=c5 c5h=WPT_LIB_VARIANT=hsum,--config=c5 c5b=--config=c5 c5hb=WPT_LIB_VARIANT=hsum,--config=c5 base= h=WPT_LIB_VARIANT=hsum || exit 1
for n in c5 c5h c5b c5hb base h; do cp gpurun_out/ab_$n.json gpurun_out/r05/dsum2/; done
python -c "
import json
for n in ['base','h']:
    d=json.load(open('gpurun_out/r05/dsum2/ab_'+n+'.json')); print(n, round(d['value']), {k:round(x['value']) for k,x in (d.get('secondary') or {}).items()})
"
