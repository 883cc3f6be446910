# Round 5, thirty-fourth GPU session: C2's kernels (other shape kinds, no BVH:
# the linear scan) at 5 waves without scratch (variant c2w5) vs 6 with 32 B of
# scratch; the museum's BVH4 kernels stay at 6 either way.
set -o pipefail
V=c2w5 bash tools/gpu_c2_var.sh || exit 1
