# Round 5, final GPU session: the committed tree as the driver runs it: the
# GPU suite and smoke().
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/final_suite.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/final_suite.log; exit 1; }
tail -1 gpurun_out/r05/final_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05/final_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r05/final_smoke.log; exit 1; }
tail -1 gpurun_out/r05/final_smoke.log
