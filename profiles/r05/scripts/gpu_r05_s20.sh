# Round 5, twentieth GPU session: the adaptive rounds' error sum from chunk
# effects computed on the GPU (k_sum_*) and walked on the host, the errors'
# copy overlapping those kernels. The GPU suite (test_gpu_seqsum.py and the
# adaptive parity tests), then C5 and the C3 line (its secondary block holds
# C5 and the init-default session) against variant hsum (the host sum alone).
set -o pipefail
mkdir -p gpurun_out/r05/dsum
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/dsum/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/dsum/tests.log; exit 1; }
tail -1 gpurun_out/r05/dsum/tests.log
AB_STEPS=4 bash tools/ab.sh c5=--config=c5 c5h=WPT_LIB_VARIANT=hsum,--config=c5 c5b=--config=c5 c5hb=WPT_LIB_VARIANT=hsum,--config=c5 base= h=WPT_LIB_VARIANT=hsum || exit 1
for n in c5 c5h c5b c5hb base h; do cp gpurun_out/ab_$n.json gpurun_out/r05/dsum/; done
python -c "
import json
for n in ['base','h']:
    d=json.load(open('gpurun_out/r05/dsum/ab_'+n+'.json')); print(n, round(d['value']), {k:round(x['value']) for k,x in (d.get('secondary') or {}).items()})
"
