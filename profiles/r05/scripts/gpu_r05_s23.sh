# Round 5, twenty-third GPU session: evidence for the final build (leaf
# batching, device error sum): the GPU suite, the default bench line, then the
# C3 kernel trace + PMC passes (tools/profile.sh) of the same workload.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05/final2_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|^E " gpurun_out/r05/final2_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r05/final2_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r05/c3_bench_line_final.json 2> gpurun_out/r05/c3_bench_line_final.err || { echo BENCHFAIL; tail -5 gpurun_out/r05/c3_bench_line_final.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05/c3_bench_line_final.json'));print(round(d['value'],1),d['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic'],d['cpu_baseline']['value'],d['parity']['bit_exact_frac'],{k:round(v['value']) for k,v in d['secondary'].items()})"
bash tools/profile.sh r05final2 || exit 1
