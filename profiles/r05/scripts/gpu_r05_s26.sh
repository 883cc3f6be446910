# Round 5, twenty-sixth GPU session: C5 GPU timeline of the final build
# (kernel trace of one counted + one timed step; tools/timeline.py: GPU busy,
# idle gaps by size, per-kernel busy), summary only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05 /tmp/c5tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/c5tl/trace -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-serial-step --no-secondary > gpurun_out/r05/c5_timeline_bench.log 2>&1 || { echo TRACEFAIL; tail -5 gpurun_out/r05/c5_timeline_bench.log; exit 1; }
python3 tools/timeline.py /tmp/c5tl/trace > gpurun_out/r05/timeline_c5_final.json || exit 1
head -c 1500 gpurun_out/r05/timeline_c5_final.json
