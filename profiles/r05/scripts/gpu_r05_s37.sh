# Round 5, last GPU session: the committed tree with the fused grid at 75 %:
# the GPU suite, smoke() and the default bench line.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/last_suite.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/last_suite.log; exit 1; }
tail -1 gpurun_out/r05/last_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05/last_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r05/last_smoke.log; exit 1; }
tail -1 gpurun_out/r05/last_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r05/c3_bench_line_last.json 2> gpurun_out/r05/c3_bench_line_last.err || { echo BENCHFAIL; tail -5 gpurun_out/r05/c3_bench_line_last.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05/c3_bench_line_last.json'));print(round(d['value'],1),d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'],d['parity']['bit_exact_frac'],{k:(round(v['value']),v.get('parity',{}).get('bit_exact_frac')) for k,v in d['secondary'].items()})"
