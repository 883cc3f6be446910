# Round 5, seventeenth GPU session: leaf batching inside k_finish's per-lane
# walks (RR-only tails of the init-default session; variant flb): its tests,
# then the same-session A/B (the init-default session is in the secondary block).
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 env WPT_LIB_VARIANT=flb python -u -m pytest tests -m gpu -x -q -k "finish or init_defaults or rr" --timeout 250 --timeout-method thread > gpurun_out/r05/t_flb.log 2>&1 || { echo TESTFAIL; grep -E "^FAILED|^E " gpurun_out/r05/t_flb.log | head; exit 1; }
echo flb $(tail -1 gpurun_out/r05/t_flb.log)
V=flb bash tools/gpu_var_ab.sh || exit 1
mkdir -p gpurun_out/r05/ab_flb; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_flb/
