# Round 5, thirtieth GPU session: the torus quartic's root set kept in
# registers (constant-index selects; torus_hit's 128 B of scratch gone). The
# GPU suite (museum parity against the oracle's separately written quartic),
# then museum lines alternating the product and variant qold (the round-4
# solver).
set -o pipefail
mkdir -p gpurun_out/r05/quartic
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/quartic/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r05/quartic/tests.log; exit 1; }
tail -1 gpurun_out/r05/quartic/tests.log
bash tools/museum_ab.sh "" qold "" qold || exit 1
cp gpurun_out/m_.json gpurun_out/m_qold.json gpurun_out/r05/quartic/
