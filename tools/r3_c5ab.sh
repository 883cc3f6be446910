#!/bin/bash
# C5 A/B: leaf-ancestor corner walks (product) vs root walks (noanc); fused
# k_trace grid size and small-batch lane count.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pnee or photon or adaptive" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
run() {  # tag variant opts...
  local tag=$1 v=$2; shift 2
  local o=""; for x in "$@"; do o="$o --opt $x"; done
  WPT_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 1 --no-serial-step $o > gpurun_out/ab_$tag.json 2>gpurun_out/ab_$tag.err || { echo FAIL $tag; tail -3 gpurun_out/ab_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));w=d['work'];print('$tag',round(d['value']),round(d['ms_per_step'],1),d['kernel_busy_ms_per_step']['trace'],d['kernel_busy_ms_per_step']['shade'],round(w['ext_loop_live_frac'],3),round(w['sh_loop_live_frac'],3))"
}
run base ""
run noanc noanc
run tg50 "" trace_grid_pct=50
run tg50l3 "" trace_grid_pct=50 small_lanes=3
run tg50l4 "" trace_grid_pct=50 small_lanes=4
run tg75 "" trace_grid_pct=75
run base2 ""
run noanc2 noanc
echo c5ab-done
