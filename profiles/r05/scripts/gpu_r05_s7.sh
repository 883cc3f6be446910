# Round 5, seventh GPU session: leaf batching only while the wave is full
# (at least WPT_LEAF_BATCH_MIN active lanes; session 6: batching in draining
# waves cost C5 6-13 %): 8 leaf lanes / 32 active, 16 / 32, 8 / 48.
set -o pipefail
mkdir -p gpurun_out/r05
for V in lb8m32 lb16m32 lb8m48; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
