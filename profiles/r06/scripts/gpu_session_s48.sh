set -o pipefail
bash tools/gpu_final.sh r06e || exit 1
timeout -k 10 400 python bench.py > gpurun_out/s48_bench2.json 2> gpurun_out/s48_bench2.err || { echo BENCHFAIL; tail -5 gpurun_out/s48_bench2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/s48_bench2.json'));print(round(d['value'],1),{k:round(v['value'],1) for k,v in d['secondary'].items()})"
