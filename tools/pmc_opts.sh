#!/bin/bash
# SQ/TCP counters of the C3 step for named option sets (one counter group per
# pass), run on the GPU box from the repo root. Usage:
#   tools/pmc_opts.sh TAG NAME="--opt a=b --opt c=d" ...   ("NAME=" = defaults)
# Summary per set: python tools/pmc_table.py gpurun_out/pmco_<TAG>_<NAME>
export TMPDIR=/tmp
TAG=$1; shift
KERNELS=${PMC_KERNELS:-"k_extend k_shadow"}
for spec in "$@"; do
  name=${spec%%=*}; opts=${spec#*=}
  OUT=gpurun_out/pmco_${TAG}_$name
  mkdir -p $OUT
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-serial-step --no-secondary $opts > $OUT/p$i.log 2>&1
    rc=$?
    echo "$name pass $i rc=$rc"
    case $rc in 0) ;; *) echo "stopping after rc=$rc"; tail -3 $OUT/p$i.log; exit $rc;; esac
  done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
GROUPS
  python3 tools/pmc_table.py $OUT $KERNELS > $OUT/table.txt
  cat $OUT/table.txt
done
echo pmc-opts-done
