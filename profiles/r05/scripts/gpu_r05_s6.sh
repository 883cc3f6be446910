# Round 5, sixth GPU session: the GPU suite on the product (work counters
# moved to wave-uniform registers), then leaf batching in step(): a lane at a
# leaf waits until 16 / 8 lanes of its wave are at one (WPT_LEAF_BATCH).
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/s6_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/s6_tests.log; exit 1; }
tail -2 gpurun_out/r05/s6_tests.log
for V in lb16 lb8; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
