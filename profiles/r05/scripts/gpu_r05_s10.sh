# Round 5, tenth GPU session: the launch knobs re-measured on the build with
# leaf batching (refill thresholds, traversal grid share; C5: refill and the
# fused grid share), one session, runtime options only (no variant build).
set -o pipefail
mkdir -p gpurun_out/r05/knobs
AB_STEPS=4 bash tools/ab.sh base= r8=--opt=refill=8 r16=--opt=refill=16 base2= rs12=--opt=refill_sh=12 rs24=--opt=refill_sh=24 g45=--opt=grid_pct=45 g55=--opt=grid_pct=55 base3= c5=--config=c5 c5r8=--config=c5,--opt=refill=8 c5r16=--config=c5,--opt=refill=16 c5g75=--config=c5,--opt=trace_grid_pct=75 || exit 1
cp gpurun_out/ab_base.json gpurun_out/ab_r8.json gpurun_out/ab_r16.json gpurun_out/ab_base2.json gpurun_out/ab_rs12.json gpurun_out/ab_rs24.json gpurun_out/ab_g45.json gpurun_out/ab_g55.json gpurun_out/ab_base3.json gpurun_out/ab_c5.json gpurun_out/ab_c5r8.json gpurun_out/ab_c5r16.json gpurun_out/ab_c5g75.json gpurun_out/r05/knobs/
