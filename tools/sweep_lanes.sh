set -o pipefail
mkdir -p gpurun_out/sweep
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --steps 5 --warmup 1 > gpurun_out/sweep/$tag.log 2>&1 || return 1; python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1))"; }
run base WPT_LANES=3 && run l4 WPT_LANES=4 && run l2 WPT_LANES=2 && run l5 WPT_LANES=5 && run r8 WPT_REFILL_LANES=8 && run r24 WPT_REFILL_LANES=24 && run base2 WPT_LANES=3
