# Round 5, fifth GPU session: (1) coarser work-feed chunks (256, 128 entries)
# against the product's 64 (finer chunks lost, session 4); (2) C5 kernel
# stats + counters of the product (the counting k_trace against the
# production one: VERDICT r4 item 2).
set -o pipefail
mkdir -p gpurun_out/r05
for V in f256 f128; do V=$V bash tools/gpu_var_ab.sh || exit 1; mkdir -p gpurun_out/r05/ab_$V; cp gpurun_out/ab_base.json gpurun_out/ab_v.json gpurun_out/ab_base2.json gpurun_out/ab_v2.json gpurun_out/ab_c5.json gpurun_out/ab_c5v.json gpurun_out/r05/ab_$V/; done
bash tools/profile_c5_small.sh r05 || exit 1
echo c5-profile-done
