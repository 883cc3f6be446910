# End-of-round evidence on one MI355X: the GPU suite, the default bench line,
# then tools/profile.sh (kernel trace + PMC passes) of the same workload.
# Usage on the box: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/final_tests.log | head -20; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo SMOKEFAIL; tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { echo BENCHFAIL; tail -5 gpurun_out/final_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final_bench.json'));print(round(d['value'],1),d['ms_per_step'],d['roofline'],d['cpu_baseline']['value'])"
bash tools/profile.sh $TAG
