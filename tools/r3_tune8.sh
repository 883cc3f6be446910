#!/bin/bash
# Launch options re-tuned at 8 waves: refill thresholds and grid share (C3),
# small-batch lanes and fused grid share (C5).
export TMPDIR=/tmp
set -o pipefail
AB_STEPS=8 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh base= r8=--opt=refill=8 r16=--opt=refill=16 rs12=--opt=refill_sh=12 rs24=--opt=refill_sh=24 g40=--opt=grid_pct=40 g60=--opt=grid_pct=60 base2= || exit 1
AB_STEPS=1 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c5=--config=c5 c5l3=--config=c5,--opt=small_lanes=3 c5g75=--config=c5,--opt=trace_grid_pct=75 c5l3g75=--config=c5,--opt=small_lanes=3,--opt=trace_grid_pct=75 c5r8=--config=c5,--opt=refill=8 || exit 1
echo tune-done
