#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats, then separate --pmc passes (one counter group per pass,
#   MI355X_MICROARCH.md §rocprofv3 PMC slots; FETCH_SIZE and WRITE_SIZE apart).
# Default workload = bench.py's default (C3 1080p, 64 spp, depth 8), one step.
# Usage: tools/profile.sh <tag> [bench args...]
set -e
TAG=${1:-r01}; shift || true
ARGS=${@:-"--steps 1 --warmup 0 --no-cpu-baseline --no-serial-step --no-secondary"}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
i=0
# SQ_THREAD_CYCLES_VALU and SQ_ACTIVE_INST_VALU in one pass: their quotient is the lane count (tools/pmc.py)
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
           "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1
done
python3 tools/pmc.py $OUT > $OUT/pmc_summary.json
echo "$ARGS" > $OUT/args.txt
echo profile-done
