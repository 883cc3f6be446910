# Round 5, sixteenth GPU session: block prologues of the late, small launches
# (C5's chain of rounds): shs = k_shade blocks without paths leave at once and
# the PNEE octree is staged with batched loads; shs2 = the same plus
# traversal blocks without work leaving before their prologue. Parity subset
# on both, then C5 twice and C3 once each, same session.
set -o pipefail
mkdir -p gpurun_out/r05/stage
for V in shs shs2; do
  timeout -k 10 300 env WPT_LIB_VARIANT=$V python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_probe.py -x -q -k "closest_hit or shadow_query or image_parity or c5_settings or probe" --timeout 250 --timeout-method thread > gpurun_out/r05/stage/t_$V.log 2>&1 || { echo TESTFAIL $V; grep -E "^FAILED|^E " gpurun_out/r05/stage/t_$V.log | head; exit 1; }
  echo $V $(tail -1 gpurun_out/r05/stage/t_$V.log)
done
AB_STEPS=4 bash tools/ab.sh c5=--config=c5 c5s=WPT_LIB_VARIANT=shs,--config=c5 c5s2=WPT_LIB_VARIANT=shs2,--config=c5 c5b=--config=c5 c5sb=WPT_LIB_VARIANT=shs,--config=c5 c5s2b=WPT_LIB_VARIANT=shs2,--config=c5 base=--no-secondary s=WPT_LIB_VARIANT=shs,--no-secondary s2=WPT_LIB_VARIANT=shs2,--no-secondary || exit 1
for n in c5 c5s c5s2 c5b c5sb c5s2b base s s2; do cp gpurun_out/ab_$n.json gpurun_out/r05/stage/; done
