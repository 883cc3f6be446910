# Usage: bash tools/profile_c5_small.sh [tag]
# C5 kernel stats and PMC summary on the GPU box, keeping only the small
# summaries (the per-dispatch CSVs of a C5 step exceed gpurun's 64 MiB).
export TMPDIR=/tmp
O=gpurun_out/prof_c5small${1:+_$1}
ARGS="--config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-serial-step --no-secondary"
mkdir -p $O /tmp/c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/c5prof/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/trace.log 2>&1 || exit 1
cp $(find /tmp/c5prof/trace -name "*kernel_stats.csv" | head -1) $O/c5_kernel_stats.csv
i=0
# SQ_THREAD_CYCLES_VALU and SQ_ACTIVE_INST_VALU in one pass: their quotient is the lane count (tools/pmc.py)
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
           "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d /tmp/c5prof/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $O/pmc$i.log 2>&1 || exit 1
done
python3 tools/pmc.py /tmp/c5prof > $O/c5_pmc_summary.json
ls -la $O
