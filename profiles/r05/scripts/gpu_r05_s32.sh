# Round 5, thirty-second GPU session: C5 launch knobs re-measured on the final
# build (device error sum, leaf batching): small-batch lanes 3 / 1, fused
# grid share 75 / 90 %, refill 16; runtime options only.
set -o pipefail
mkdir -p gpurun_out/r05/knobs5
AB_STEPS=4 bash tools/ab.sh c5=--config=c5 l3=--config=c5,--opt=small_lanes=3 l1=--config=c5,--opt=small_lanes=1 g75=--config=c5,--opt=trace_grid_pct=75 g90=--config=c5,--opt=trace_grid_pct=90 c5b=--config=c5 r16=--config=c5,--opt=refill=16 || exit 1
for n in c5 l3 l1 g75 g90 c5b r16; do cp gpurun_out/ab_$n.json gpurun_out/r05/knobs5/; done
