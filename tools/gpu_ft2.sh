set -o pipefail
mkdir -p gpurun_out
F=--opt=traversal=ft,--opt=traversal_sh=ft
AB_STEPS=4 bash tools/ab.sh bvh2= l8=$F,--opt=ft_max_leaf=8 l1=$F,--opt=ft_max_leaf=1,--opt=ft_ctrav=0 l2=$F,--opt=ft_max_leaf=2,--opt=ft_ctrav=50 l1o=$F,--opt=ft_max_leaf=1,--opt=ft_ctrav=0,--opt=ft_omax=32,--opt=ft_margin=12 l1n=$F,--opt=ft_max_leaf=1,--opt=ft_ctrav=0,--opt=ft_spatial=0
for f in bvh2 l8 l1 l2 l1o l1n; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));w=d['work'];print('$f',round(d['value']),'tests/ray %.2f far %.4f retr %.2e'%(w['prim_tests_per_ray'],w['exact_origin_per_ray'],w['exact_retrace_per_ray']),d['kernel_busy_ms_per_step'], d['scene_load'].get('fast_tree'))"; done
