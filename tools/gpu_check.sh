set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
for v in "" sb512 sb256; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/b1_$v.json 2>gpurun_out/b1_$v.err || { echo BENCHFAIL $v; tail gpurun_out/b1_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b1_$v.json'));print('$v',round(d['value']),d['ms_per_step'],d['kernel_busy_ms_per_step'],d['kernel_launch_ms_per_step'])"
done
WPT_LANES=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > gpurun_out/b1_l1.json 2>gpurun_out/b1_l1.err && python -c "import json;d=json.load(open('gpurun_out/b1_l1.json'));print('lanes1',round(d['value']),d['ms_per_step'],d['kernel_busy_ms_per_step'],d['kernel_launch_ms_per_step'])"
