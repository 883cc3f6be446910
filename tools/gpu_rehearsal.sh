set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 > gpurun_out/b_g2.json 2> gpurun_out/b_g2.err || { echo GLOOFAIL; tail gpurun_out/b_g2.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/b_g2.json').read().strip().splitlines()[-1]);print('gloo2', round(d['value']), d['config']['parallelism'], d['scaling'])"
