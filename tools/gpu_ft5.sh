set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ft" --timeout 200 --timeout-method thread > gpurun_out/t_par.log 2>&1; rc=$?
tail -2 gpurun_out/t_par.log; grep -E "^FAILED|^E " gpurun_out/t_par.log | head -20
[ $rc -eq 0 ] || exit 1
F=--opt=traversal=ft,--opt=traversal_sh=ft,--opt=ft_max_leaf=1,--opt=ft_ctrav=0
AB_STEPS=4 bash tools/ab.sh bvh2= l1=$F l1d4=$F,--opt=drain_bpc=4 l2=--opt=traversal=ft,--opt=traversal_sh=ft,--opt=ft_max_leaf=2,--opt=ft_ctrav=50 c5=--config=c5,--steps=1,--no-serial-step,$F c5x=--config=c5,--steps=1,--no-serial-step
for f in bvh2 l1 l1d4 l2 c5 c5x; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));w=d['work'];print('$f',round(d['value']),'tests/ray %.2f far %.4f retr %.2e'%(w['prim_tests_per_ray'],w['exact_origin_per_ray'],w['exact_retrace_per_ray']),d['kernel_serial_ms_per_step'],'lanes/body %.1f %.1f'%(w['lanes_per_expand_body'],w['lanes_per_leaf_body']))"; done
