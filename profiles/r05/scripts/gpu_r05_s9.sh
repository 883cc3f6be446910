# Round 5, ninth GPU session: the GPU suite on the product with leaf batching
# on (16 leaf lanes / 32 active, triangle scenes), then the shadow walks'
# thresholds (k_shadow, and every walk of the fused k_trace): 8 or 24 leaf
# lanes, or a minimum of 48 / 16 active lanes.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/s9_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/s9_tests.log; exit 1; }
tail -1 gpurun_out/r05/s9_tests.log
for V in sh8 sh24 shm48 shm16; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
