set -o pipefail
# GPU tests, then a same-session A/B of the traversals (exact BVH2, BVH4, fast
# tree) on C3 and the gloo world-2 rehearsal of the N>1 bench path (two ranks
# on one GPU). Usage on the box: bash tools/gpu_trav_ab.sh
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?
tail -2 gpurun_out/t_all.log; grep -E "^FAILED|^E " gpurun_out/t_all.log | head -20
[ $rc -eq 0 ] || exit 1
F=--opt=traversal=ft,--opt=traversal_sh=ft
AB_STEPS=4 bash tools/ab.sh bvh2= bvh4=--opt=traversal=bvh4,--opt=traversal_sh=bvh4 l1=$F,--opt=ft_max_leaf=1,--opt=ft_ctrav=0 bvh2b= || exit 1
for f in bvh2 bvh4 l1 bvh2b; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));w=d['work'];print('$f',round(d['value']),'tests/ray %.2f far %.4f retr %.2e'%(w['prim_tests_per_ray'],w['exact_origin_per_ray'],w['exact_retrace_per_ray']),d['kernel_serial_ms_per_step'])"; done
MASTER_ADDR=127.0.0.1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > gpurun_out/gloo2.json 2> gpurun_out/gloo2.err; echo gloo rc=$?
tail -c 1500 gpurun_out/gloo2.json
