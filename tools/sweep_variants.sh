# A/B of experiment builds (csrc/Makefile `variant`) against the default library
set -o pipefail
mkdir -p gpurun_out/sweep
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 1 > gpurun_out/sweep/$tag.log 2>&1 || return 1; python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1))"; }
run vbase WPT_LIB_VARIANT= && run vilp WPT_LIB_VARIANT=max_ilp && run vmc WPT_LIB_VARIANT=max_memory_clause && run vbase2 WPT_LIB_VARIANT= \
 && WPT_LIB_VARIANT=max_ilp timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "100k or fused" --timeout 120 --timeout-method thread > gpurun_out/sweep/parity_ilp.log 2>&1; echo parity_ilp=$?; tail -1 gpurun_out/sweep/parity_ilp.log
