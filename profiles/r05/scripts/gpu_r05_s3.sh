# Round 5, third GPU session: larger traversal blocks holding a larger LDS
# treelet (the traversal kernels' TA/TD data path is ~75-85 % busy at full
# residency, profiles/r05/pmc_full_residency_c3.json; LDS reads bypass it):
# 1024-thread blocks with 104 treelet pairs, 512 with 48, vs the product
# (256 threads, 23 pairs), each with its parity subset.
set -o pipefail
mkdir -p gpurun_out/r05
for V in b1024 b512; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
