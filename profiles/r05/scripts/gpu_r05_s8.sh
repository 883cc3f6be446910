# Round 5, eighth GPU session: leaf batching around the session-7 winner
# (16 leaf lanes / 32 active: C3 +4.9 %, C5 +1.6 %): 24 / 32, 16 / 24,
# 16 / 40, 32 / 48. The product's base also carries the auto-traversal fix
# (scenes without a BVH keep the BVH2 kernels' linear scan: C2).
set -o pipefail
mkdir -p gpurun_out/r05
for V in lb24m32 lb16m24 lb16m40 lb32m48; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
