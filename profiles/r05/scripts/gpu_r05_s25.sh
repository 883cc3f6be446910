# Round 5, twenty-fifth GPU session: an adaptive round's batch returns
# without waiting for its lanes (its counts are read at the next host sync):
# the next round's planning is queued behind it. The GPU suite, then C5 twice
# and the C3 line against variant sb (every batch waits at its end).
# (Session 24 counted the next round's path count as a batch's rays: the planning reused
# the lanes' pinned count words; fixed with a word of its own, and the probe
# test now checks an adaptive session's ray counts.)
set -o pipefail
mkdir -p gpurun_out/r05/defer2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/defer2/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/defer2/tests.log; exit 1; }
tail -1 gpurun_out/r05/defer2/tests.log
AB_STEPS=4 bash tools/ab.sh c5=--config=c5 c5s=WPT_LIB_VARIANT=sb,--config=c5 c5b=--config=c5 c5sb=WPT_LIB_VARIANT=sb,--config=c5 base= s=WPT_LIB_VARIANT=sb || exit 1
for n in c5 c5s c5b c5sb base s; do cp gpurun_out/ab_$n.json gpurun_out/r05/defer2/; done
python -c "
import json
for n in ['base','s']:
    d=json.load(open('gpurun_out/r05/defer2/ab_'+n+'.json')); print(n, round(d['value']), {k:round(x['value']) for k,x in (d.get('secondary') or {}).items()})
"
