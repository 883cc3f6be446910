# Round 5, thirty-third GPU session: k_finish (the RR-only tails of the
# reference's init-default session) reads the PNEE octree's child array from
# LDS like k_shade (product) instead of global memory (variant foct0). The GPU
# suite, then C3 lines with their secondary block (init defaults) alternating.
set -o pipefail
mkdir -p gpurun_out/r05/foct
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/foct/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/foct/tests.log; exit 1; }
tail -1 gpurun_out/r05/foct/tests.log
AB_STEPS=3 bash tools/ab.sh base= v=WPT_LIB_VARIANT=foct0 base2= v2=WPT_LIB_VARIANT=foct0 || exit 1
for n in base v base2 v2; do cp gpurun_out/ab_$n.json gpurun_out/r05/foct/; done
python -c "
import json
for n in ['base','v','base2','v2']:
    d=json.load(open('gpurun_out/r05/foct/ab_'+n+'.json')); print(n, round(d['value']), {k:round(x['value']) for k,x in (d.get('secondary') or {}).items()})
"
