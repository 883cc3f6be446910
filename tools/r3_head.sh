#!/bin/bash
# Re-entry check of HEAD: whole GPU suite, the default bench line, smoke().
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/head
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/head/gpu_tests.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/head/gpu_tests.log | head; tail -3 gpurun_out/head/gpu_tests.log; exit 1; }
tail -1 gpurun_out/head/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/head/bench.json 2> gpurun_out/head/bench.err || { echo BENCHFAIL; tail -5 gpurun_out/head/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/head/bench.json'));print('c3',round(d['value']),round(d['ms_per_step'],2),d['parity']['rel_l2'],d['parity'].get('bit_exact_frac'));[print(k,v.get('Mray/s'),v.get('ms_per_step'),v.get('bit_exact')) for k,v in d.get('secondary',{}).items() if isinstance(v,dict)]"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo head-done
