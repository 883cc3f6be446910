# Round 5, fourth GPU session: (1) the spawn rehearsal VERDICT r4 asks for --
# bench.py --gpus 2 starts its own two ranks (gloo, both on the box's one
# GPU); (2) work-feed chunk size: 16- and 4-entry chunks against the
# product's 64 (finer chunks balance per-wave cost on the adaptive C5 rounds).
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 > gpurun_out/r05/gloo2_spawn.json 2> gpurun_out/r05/gloo2_spawn.err || { echo SPAWNFAIL; tail -20 gpurun_out/r05/gloo2_spawn.err; exit 1; }
echo spawn ok
for V in f16 f4; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
