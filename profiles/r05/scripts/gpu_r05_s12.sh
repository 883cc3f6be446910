# Round 5, twelfth GPU session: the BVH4 walk with leaf children in one
# nearest-first order under leaf batching (WPT_TRAV4_BATCH=1, variant t4b):
# the parity file on the variant, then museum lines (BVH4 is its default
# traversal) alternating product / variant.
set -o pipefail
mkdir -p gpurun_out/r05/t4b
timeout -k 10 600 env WPT_LIB_VARIANT=t4b python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/t4b/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/t4b/tests.log; exit 1; }
tail -1 gpurun_out/r05/t4b/tests.log
bash tools/museum_ab.sh "" t4b "" t4b || exit 1
cp gpurun_out/m_.json gpurun_out/m_t4b.json gpurun_out/r05/t4b/
