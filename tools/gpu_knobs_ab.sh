# Same-session C3 A/B of launch knobs and k_shade grid variants (sg25 / sg50).
AB_STEPS=4 bash tools/ab.sh base= sg25=WPT_LIB_VARIANT=sg25 sg50=WPT_LIB_VARIANT=sg50 g40=--opt=grid_pct=40 g60=--opt=grid_pct=60 rs8=--opt=refill_sh=8 rs24=--opt=refill_sh=24 r8=--opt=refill=8 r16=--opt=refill=16 base2= sg50b=WPT_LIB_VARIANT=sg50
