#!/bin/bash
# Lanes x traversal grid share on the 8-wave build (C3, same session).
export TMPDIR=/tmp
set -o pipefail
AB_STEPS=8 AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh base= l3g67=--opt=lanes=3,--opt=grid_pct=67 l3g50=--opt=lanes=3,--opt=grid_pct=50 g45=--opt=grid_pct=45 g55=--opt=grid_pct=55 l2g100=--opt=lanes=2,--opt=grid_pct=100 base2= || exit 1
echo lanes-done
