set -o pipefail
for k in 1 2; do
timeout -k 10 400 python bench.py > gpurun_out/s44_bench$k.json 2> gpurun_out/s44_bench$k.err || { echo BENCHFAIL; tail -5 gpurun_out/s44_bench$k.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/s44_bench$k.json'));print(round(d['value'],1),{k:round(v['value'],1) for k,v in d['secondary'].items()})"
done
