# Round 5, nineteenth GPU session: the GPU suite on the product (lanes 1..8),
# then the museum's traversal kernels at 5 waves (variant any5): its parity
# file, museum lines alternating product / variant.
set -o pipefail
mkdir -p gpurun_out/r05/any5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/s19_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/s19_tests.log; exit 1; }
tail -1 gpurun_out/r05/s19_tests.log
timeout -k 10 600 env WPT_LIB_VARIANT=any5 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/any5/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/any5/tests.log; exit 1; }
tail -1 gpurun_out/r05/any5/tests.log
bash tools/museum_ab.sh "" any5 "" any5 || exit 1
cp gpurun_out/m_.json gpurun_out/m_any5.json gpurun_out/r05/any5/
