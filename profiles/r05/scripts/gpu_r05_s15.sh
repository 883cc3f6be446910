# Round 5, fifteenth GPU session: more lanes than the default 4 on more
# hardware queues (GPU_MAX_HW_QUEUES is HIP's own per-process setting, 4 on
# the box): 6 / 8 lanes at traversal grid shares 25-50 %, same session.
set -o pipefail
mkdir -p gpurun_out/r05/lanes
AB_STEPS=4 bash tools/ab.sh base= q8=GPU_MAX_HW_QUEUES=8 q8l8=GPU_MAX_HW_QUEUES=8,--opt=lanes=8 q8l8g25=GPU_MAX_HW_QUEUES=8,--opt=lanes=8,--opt=grid_pct=25 q8l8g35=GPU_MAX_HW_QUEUES=8,--opt=lanes=8,--opt=grid_pct=35 q6l6g35=GPU_MAX_HW_QUEUES=6,--opt=lanes=6,--opt=grid_pct=35 base2= q8l8g35b=GPU_MAX_HW_QUEUES=8,--opt=lanes=8,--opt=grid_pct=35 || exit 1
for n in base q8 q8l8 q8l8g25 q8l8g35 q6l6g35 base2 q8l8g35b; do cp gpurun_out/ab_$n.json gpurun_out/r05/lanes/; done
