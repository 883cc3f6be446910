#!/bin/bash
# Round-3 evidence run: whole GPU suite, the default bench line (C3 + CPU
# baseline + secondary configs), rocprof kernel stats of C3, C5 and
# init-default timelines, C4 strong scaling at N=1 and as 2 gloo ranks.
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/r3/gpu_tests.log | head; tail -3 gpurun_out/r3/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r3/c3_bench_line.json 2> gpurun_out/r3/c3_bench.err || { echo BENCHFAIL; tail -5 gpurun_out/r3/c3_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r3/c3_bench_line.json'));print('c3',round(d['value']),round(d['ms_per_step'],2),d['parity']['rel_l2'],d['parity'].get('bit_exact_frac'));[print(k,v.get('Mray/s'),v.get('ms_per_step'),v.get('bit_exact')) for k,v in d.get('secondary',{}).items() if isinstance(v,dict)]"
rm -rf gpurun_out/r3/prof_c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/r3/prof_c3.log 2>&1 || { echo PROFFAIL; tail -5 gpurun_out/r3/prof_c3.log; exit 1; }
tail -c 300 gpurun_out/r3/prof_c3.log; echo
rm -rf gpurun_out/r3/prof_c5 gpurun_out/r3/prof_ds
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step > gpurun_out/r3/prof_c5.log 2>&1 || { echo C5FAIL; tail -5 gpurun_out/r3/prof_c5.log; exit 1; }
python3 tools/timeline.py gpurun_out/r3/prof_c5 > gpurun_out/r3/timeline_c5.json && head -4 gpurun_out/r3/timeline_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_ds -o run --output-format csv -- python3 tools/default_session_rate.py 3 > gpurun_out/r3/prof_ds.log 2>&1 || { echo DSFAIL; tail -5 gpurun_out/r3/prof_ds.log; exit 1; }
python3 tools/timeline.py gpurun_out/r3/prof_ds > gpurun_out/r3/timeline_ds.json && head -4 gpurun_out/r3/timeline_ds.json
timeout -k 10 300 python3 bench.py --config c4 --scaling strong --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step > gpurun_out/r3/c4_strong_n1.json 2> gpurun_out/r3/c4_strong_n1.err || { echo C4FAIL; tail -5 gpurun_out/r3/c4_strong_n1.err; exit 1; }
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --config c4 --scaling strong --backend gloo --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step > gpurun_out/r3/c4_strong_gloo2.json 2> gpurun_out/r3/c4_strong_gloo2.err || { echo C4G2FAIL; tail -5 gpurun_out/r3/c4_strong_gloo2.err; exit 1; }
python3 -c "
import json
for f in ('c4_strong_n1','c4_strong_gloo2'):
    d=json.load(open('gpurun_out/r3/'+f+'.json')); print(f, round(d['value']), round(d['ms_per_step'],1))"
echo full-done
