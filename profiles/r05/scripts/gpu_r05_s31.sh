# Round 5, thirty-first GPU session: with the torus test free of scratch, the
# museum's traversal kernels at 5 / 4 waves (variants any5 / any4, no scratch)
# against the product's 6 (80 VGPRs forced, 80-112 B scratch); then the
# final build's default bench line.
set -o pipefail
mkdir -p gpurun_out/r05/waves2
for V in any5 any4; do
  timeout -k 10 600 env WPT_LIB_VARIANT=$V python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/waves2/t_$V.log 2>&1 || { echo TESTFAIL $V; tail -20 gpurun_out/r05/waves2/t_$V.log; exit 1; }
  echo $V $(tail -1 gpurun_out/r05/waves2/t_$V.log)
done
bash tools/museum_ab.sh "" any5 any4 "" any5 any4 || exit 1
cp gpurun_out/m_.json gpurun_out/m_any5.json gpurun_out/m_any4.json gpurun_out/r05/waves2/
timeout -k 10 600 python bench.py > gpurun_out/r05/c3_bench_line_final4.json 2> gpurun_out/r05/c3_bench_line_final4.err || { echo BENCHFAIL; tail -5 gpurun_out/r05/c3_bench_line_final4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05/c3_bench_line_final4.json'));print(round(d['value'],1),d['ms_per_step'],d['roofline']['frac'],d['cpu_baseline']['value'],d['parity']['bit_exact_frac'],{k:(round(v['value']),v.get('parity',{}).get('bit_exact_frac')) for k,v in d['secondary'].items()})"
