#!/bin/bash
# SQ counters of library variants on one C3 step (run on the GPU box from the
# repo root; one counter group per pass). Usage: tools/pmc_ab.sh <tag> <variant...>
# ("base" = the product library; PMC_ARGS / PMC_KERNELS override the bench
# arguments and the kernels tabulated). Summary: python tools/pmc_table.py gpurun_out/pmcab_<tag>_<v>
export TMPDIR=/tmp
TAG=${1:-ab}; shift
ARGS=${PMC_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --no-serial-step --no-secondary"}
KERNELS=${PMC_KERNELS:-"k_extend k_shadow k_shade"}
for v in "$@"; do
  lib=$v; [ "$v" == "base" ] && lib=""
  OUT=gpurun_out/pmcab_${TAG}_$v
  mkdir -p $OUT
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    WPT_LIB_VARIANT=$lib timeout -s KILL 150 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
    rc=$?
    echo "$v pass $i rc=$rc"
    case $rc in 0) ;; *) echo "stopping after rc=$rc"; tail -3 $OUT/p$i.log; exit $rc;; esac
  done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS
GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr TA_BUSY_max
TD_BUSY_avr TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
GROUPS
  python3 tools/pmc_table.py $OUT $KERNELS > $OUT/table.txt
  cat $OUT/table.txt
done
echo pmc-ab-done
