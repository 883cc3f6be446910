F=--opt=traversal=ft,--opt=traversal_sh=ft,--opt=ft_max_leaf=1,--opt=ft_ctrav=0
AB_STEPS=4 bash tools/ab.sh bvh2= l1=$F l1b4=$F,--opt=drain_bpc=4 l1b8=$F,--opt=drain_bpc=8 l1e=--opt=traversal=ft,--opt=ft_max_leaf=1,--opt=ft_ctrav=0,--opt=drain_bpc=8 c5=--config=c5 c5l1b8=$F,--opt=drain_bpc=8,--config=c5 || exit 1
for f in bvh2 l1 l1b4 l1b8 l1e c5 c5l1b8; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));w=d['work'];print('$f',round(d['value']),'far %.4f retr %.2e'%(w['exact_origin_per_ray'],w['exact_retrace_per_ray']),d['kernel_serial_ms_per_step'])"; done
