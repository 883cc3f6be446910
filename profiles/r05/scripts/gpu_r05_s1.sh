# Round 5, first GPU session: the GPU suite on the round's changes, the wave
# probe of C5 and C3 launches, the traversal A/B on C5 / museum / C3
# (tools/gpu_trav_scenes.sh), the inline-leaf variant A/B, the PMC counter
# list and a PC-sampling attempt.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r05/s1_tests.log 2>&1 || { echo TESTFAIL; tail -5 gpurun_out/r05/s1_tests.log; grep -E "^FAILED|^E " gpurun_out/r05/s1_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r05/s1_tests.log
timeout -k 10 300 python tools/probe_tails.py c5 1500 > gpurun_out/r05/probe_c5.json 2> gpurun_out/r05/probe_c5.err || { echo PROBEFAIL; tail -5 gpurun_out/r05/probe_c5.err; exit 1; }
timeout -k 10 200 python tools/probe_tails.py c3 1500 > gpurun_out/r05/probe_c3.json 2> gpurun_out/r05/probe_c3.err || { echo PROBEFAIL3; tail -5 gpurun_out/r05/probe_c3.err; exit 1; }
python -c "
import json
for c in ('c5','c3'):
    d=json.load(open('gpurun_out/r05/probe_%s.json'%c))
    for k,v in d['kernels'].items(): print(c,k,{a:(round(b,3) if isinstance(b,float) else b) for a,b in v.items() if a!='by_bounce'})
"
bash tools/gpu_trav_scenes.sh || exit 1
V=inl bash tools/gpu_var_ab.sh || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/r05/counters_list.txt 2>&1; echo list rc=$?
bash tools/pc_sample.sh
