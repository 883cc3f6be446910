set -e
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
run() { echo "== $1"; shift; env "$@" timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(round(d['value'],1), d['kernel_share'], d['roofline']['avg_launch_ms']); print(d['work'])"; }
run bvh4 A=1
run bvh2 WPT_TRAVERSAL=bvh2
