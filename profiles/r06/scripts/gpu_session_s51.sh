set -o pipefail
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_stock.py tests/test_gpu_parity.py > gpurun_out/s51_tests.log 2>&1 || { echo FAIL; tail -20 gpurun_out/s51_tests.log; exit 1; }
tail -1 gpurun_out/s51_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
