#!/bin/bash
# Round-3 evidence: kernel traces of C5 and the init-default session (timeline
# breakdown), C4 strong scaling at N=1 and as a 2-rank gloo rehearsal on one GPU.
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step > gpurun_out/prof_c5.log 2>&1 || { echo C5FAIL; tail -5 gpurun_out/prof_c5.log; exit 1; }
python3 tools/timeline.py gpurun_out/prof_c5 > gpurun_out/timeline_c5.json && head -4 gpurun_out/timeline_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ds -o run --output-format csv -- python3 tools/default_session_rate.py 3 > gpurun_out/prof_ds.log 2>&1 || { echo DSFAIL; tail -5 gpurun_out/prof_ds.log; exit 1; }
python3 tools/timeline.py gpurun_out/prof_ds > gpurun_out/timeline_ds.json && head -4 gpurun_out/timeline_ds.json
timeout -k 10 300 python3 bench.py --config c4 --scaling strong --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step > gpurun_out/c4_strong_n1.json 2> gpurun_out/c4_strong_n1.err || { echo C4FAIL; tail -5 gpurun_out/c4_strong_n1.err; exit 1; }
tail -c 400 gpurun_out/c4_strong_n1.json; echo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --config c4 --scaling strong --backend gloo --steps 1 --warmup 1 --no-cpu-baseline --no-serial-step > gpurun_out/c4_strong_gloo2.json 2> gpurun_out/c4_strong_gloo2.err || { echo C4G2FAIL; tail -5 gpurun_out/c4_strong_gloo2.err; exit 1; }
tail -c 400 gpurun_out/c4_strong_gloo2.json; echo
echo profiles-done
