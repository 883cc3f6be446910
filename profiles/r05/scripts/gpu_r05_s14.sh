# Round 5, fourteenth GPU session: the final build's GPU suite and default
# bench line (C3 + roofline + cpu_baseline + secondary), as the driver runs them.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05/final_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|^E " gpurun_out/r05/final_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r05/final_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r05/c3_bench_line.json 2> gpurun_out/r05/c3_bench_line.err || { echo BENCHFAIL; tail -5 gpurun_out/r05/c3_bench_line.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05/c3_bench_line.json'));print(round(d['value'],1),d['ms_per_step'],d['roofline'],d['cpu_baseline']['value'],{k:round(v['value']) for k,v in d['secondary'].items()})"
