#!/bin/bash
# Round-3 probe: GPU suite, SQ/TA/TCP counters of the product vs the one-phase
# loop (libwpt_old), and the small-batch workloads (C5, init defaults) A/B.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/t.log | head -20; exit 1; }
tail -1 gpurun_out/t.log
bash tools/pmc_ab.sh r3 base old || exit 1
for v in "" old; do
  WPT_LIB_VARIANT=$v timeout -k 10 200 python tools/default_session_rate.py 3 > gpurun_out/ds_$v.json 2>gpurun_out/ds_$v.err || { echo DSFAIL $v; tail -3 gpurun_out/ds_$v.err; exit 1; }
  cat gpurun_out/ds_$v.json
  WPT_LIB_VARIANT=$v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 1 --warmup 1 --no-serial-step > gpurun_out/c5_$v.json 2>gpurun_out/c5_$v.err || { echo C5FAIL $v; tail -3 gpurun_out/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5_$v.json'));print('c5 [$v]',round(d['value']),round(d['ms_per_step'],1),d['kernel_busy_ms_per_step'])"
done
echo probe-done
