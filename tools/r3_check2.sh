#!/bin/bash
# Whole GPU suite, then a 2-rank gloo rehearsal of the default weak-scaling
# bench on one GPU and smoke().
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t_all.log | head; tail -3 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g2.json 2> gpurun_out/g2.err || { echo G2FAIL; tail -5 gpurun_out/g2.err; exit 1; }
tail -1 gpurun_out/g2.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('gloo2', round(d['value']), round(d['ms_per_step'],1), d['scaling'], d['config'].get('parallelism'))"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo check2-done
