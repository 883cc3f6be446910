# Round 5, second GPU session: the GPU suite after the fast tree's removal
# (auto traversal), the variant A/Bs (leaf peel, sincos at 6 / 7 NEE-shade
# waves), the wave probe of C5 / C3 with the GPU-wide timeline, the museum
# default, and the full-residency counter passes of the traversal kernels.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r05/s2_tests.log 2>&1 || { echo TESTFAIL; tail -5 gpurun_out/r05/s2_tests.log; grep -E "^FAILED|^E " gpurun_out/r05/s2_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r05/s2_tests.log
timeout -k 10 300 python tools/probe_tails.py c5 1500 > gpurun_out/r05/probe2_c5.json 2> gpurun_out/r05/probe2_c5.err || { echo PROBEFAIL; tail -5 gpurun_out/r05/probe2_c5.err; exit 1; }
timeout -k 10 200 python tools/probe_tails.py c3 1500 > gpurun_out/r05/probe2_c3.json 2> gpurun_out/r05/probe2_c3.err || { echo PROBEFAIL3; exit 1; }
python -c "
import json
for c in ('c5','c3'):
    d=json.load(open('gpurun_out/r05/probe2_%s.json'%c)); print(c, 'gpu_wide', d['gpu_wide'])
"
for V in peel sc sc7; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
AB_STEPS=3 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh musauto=--config=museum mus2=--config=museum,--opt=traversal=bvh2,--opt=traversal_sh=bvh2 || exit 1
bash tools/pmc_extend.sh ext
