# Round 5, twenty-eighth GPU session: expand batching on top of leaf
# batching: when the leaf body runs this iteration anyway, lanes at internal
# nodes wait unless 8 / 16 of them would expand (variants eb8 / eb16).
set -o pipefail
mkdir -p gpurun_out/r05
for V in eb8 eb16; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
