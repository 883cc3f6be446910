set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1; rc=$?
tail -3 gpurun_out/t_par.log; grep -E "^FAILED|^E " gpurun_out/t_par.log | head -20
[ $rc -eq 0 ] || exit 1
AB_STEPS=5 bash tools/ab.sh base= bvh2=--opt=traversal=bvh2,--opt=traversal_sh=bvh2 c5=--config=c5,--steps=1,--no-serial-step c5x=--config=c5,--steps=1,--no-serial-step,--opt=traversal=bvh2,--opt=traversal_sh=bvh2
for f in base bvh2; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',d['work'],d['kernel_busy_ms_per_step'])"; done
