# Round 5: the traversals (exact BVH2, BVH4 fast path, fast tree) on the
# configs where fewer steps could pay (C5, museum), same session, plus C3.
# Usage on the box: bash tools/gpu_trav_scenes.sh
set -o pipefail
mkdir -p gpurun_out
B4=--opt=traversal=bvh4,--opt=traversal_sh=bvh4
FT=--opt=traversal=ft,--opt=traversal_sh=ft
AB_STEPS=${AB_STEPS:-3} AB_ARGS="--no-serial-step --no-secondary" bash tools/ab.sh c3= c5=--config=c5 c5b4=--config=c5,$B4 c5ft=--config=c5,$FT \
  mus=--config=museum musb4=--config=museum,$B4 c3b4=$B4 c3ft=$FT c3b=
