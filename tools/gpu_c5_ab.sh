# Same-session A/B: C3 with the octant-ordered shade output (variant ss), and
# C5 with its late bounces in k_finish (finish_after = 2..5).
AB_STEPS=4 bash tools/ab.sh base= ss=WPT_LIB_VARIANT=ss base2= ss2=WPT_LIB_VARIANT=ss || exit 1
AB_STEPS=2 bash tools/ab.sh c5=--config=c5 c5f2=--config=c5,--opt=finish_after=2 c5f3=--config=c5,--opt=finish_after=3 c5f4=--config=c5,--opt=finish_after=4 c5f5=--config=c5,--opt=finish_after=5 c5ss=WPT_LIB_VARIANT=ss,--config=c5 || exit 1
for f in base ss base2 ss2 c5 c5f2 c5f3 c5f4 c5f5 c5ss; do python -c "import json;d=json.load(open('gpurun_out/ab_$f.json'));print('$f',round(d['value']),d['kernel_serial_ms_per_step'],d.get('parity',{}).get('bit_exact_frac'), d.get('secondary'))"; done
