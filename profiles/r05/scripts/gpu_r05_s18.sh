# Round 5, eighteenth GPU session: the museum's traversal kernels (other shape
# kinds: BVH4 walk + out-of-line f64 torus test) at 5 waves per SIMD without
# scratch (variant any5) against the product's 6 (80 VGPRs forced, 80-112 B
# scratch); parity file on the variant, museum lines alternating.
set -o pipefail
mkdir -p gpurun_out/r05/any5
timeout -k 10 600 env WPT_LIB_VARIANT=any5 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/any5/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/any5/tests.log; exit 1; }
tail -1 gpurun_out/r05/any5/tests.log
bash tools/museum_ab.sh "" any5 "" any5 || exit 1
cp gpurun_out/m_.json gpurun_out/m_any5.json gpurun_out/r05/any5/
