# Chained compute calls: their GPU tests, the whole GPU suite (chaining is on
# by default), then a same-session C3 A/B of chain / stagger settings.
# Usage on the box: bash tools/gpu_chain_ab.sh TAG "variant" "variant" ...
set -o pipefail
TAG=${1:-chain}; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_chain_tests.log 2>&1 || { echo CHAINFAIL; grep -E "^FAILED|^E " gpurun_out/${TAG}_chain_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_chain_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_suite.log 2>&1 || { echo SUITEFAIL; grep -E "^FAILED|^E " gpurun_out/${TAG}_suite.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_suite.log
timeout -k 10 600 python tools/session_rate.py c3 --reps 2 "$@" > gpurun_out/${TAG}_ab_c3.jsonl 2> gpurun_out/${TAG}_ab_c3.err || { echo ABFAIL; tail -5 gpurun_out/${TAG}_ab_c3.err; exit 1; }
tail -1 gpurun_out/${TAG}_ab_c3.jsonl
