#!/bin/bash
# PMC probe of the traversal kernels' memory pipeline (one counter group per
# pass; run on the GPU box from the repo root). Usage: tools/pmc_probe.sh <tag>
export TMPDIR=/tmp
TAG=${1:-probe}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $grp"
  case $rc in 124|134|137|139) echo "stopping after rc=$rc"; exit $rc;; esac
done <<'GROUPS'
TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT
TD_BUSY_avr TD_TC_STALL_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_WAVES
GROUPS
echo probe-done
