#!/bin/bash
# PNEE octree through address-space-typed LDS pointers (ds_read; product) vs
# generic pointers (flat loads; the previous commit as variant "head"): C5.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pnee or photon or adaptive or init_defaults or finish or light_debug or museum or torus" > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head; exit 1; }
tail -1 gpurun_out/t.log
AB_STEPS=1 AB_ARGS="--no-serial-step --config c5" bash tools/ab.sh base= head=WPT_LIB_VARIANT=head base2= head2=WPT_LIB_VARIANT=head || exit 1
AB_STEPS=2 AB_ARGS="--no-serial-step --config museum" bash tools/ab.sh mus= mushead=WPT_LIB_VARIANT=head || exit 1
echo oct-done
