# Round 5, twenty-seventh GPU session: the final build's evidence: GPU suite,
# default bench line, C5 kernel stats + counters (production and counting
# k_trace keyed apart).
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05/final3_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|^E " gpurun_out/r05/final3_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r05/final3_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r05/c3_bench_line_final3.json 2> gpurun_out/r05/c3_bench_line_final3.err || { echo BENCHFAIL; tail -5 gpurun_out/r05/c3_bench_line_final3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05/c3_bench_line_final3.json'));print(round(d['value'],1),d['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic'],d['cpu_baseline']['value'],d['parity']['bit_exact_frac'],{k:round(v['value']) for k,v in d['secondary'].items()})"
bash tools/profile_c5_small.sh r05final || exit 1
