# Round 5: the traversals (exact BVH2, BVH4 fast path; the fast tree was
# measured here too, then removed) on the configs where fewer steps could pay
# (C5, museum), same session, plus C3.
# Usage on the box: bash tools/gpu_trav_scenes.sh
set -o pipefail
mkdir -p gpurun_out
B4=--opt=traversal=bvh4,--opt=traversal_sh=bvh4
B2=--opt=traversal=bvh2,--opt=traversal_sh=bvh2
AB_STEPS=${AB_STEPS:-3} AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c3=$B2 c5=--config=c5,$B2 c5b4=--config=c5,$B4 \
  mus=--config=museum,$B2 musb4=--config=museum,$B4 c3b4=$B4 c3b=$B2
