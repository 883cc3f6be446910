set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_museum /tmp/musprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/musprof/trace -o run --output-format csv -- python3 tools/session_rate.py museum --reps 1 "" > gpurun_out/prof_museum/trace.log 2>&1 || exit 1
cp $(find /tmp/musprof/trace -name "*kernel_stats.csv" | head -1) gpurun_out/prof_museum/kernel_stats.csv
python3 tools/timeline.py /tmp/musprof/trace > gpurun_out/prof_museum/timeline.json
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS -d /tmp/musprof/pmc1 -o run --output-format csv -- python3 tools/session_rate.py museum --reps 1 "" > gpurun_out/prof_museum/pmc1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d /tmp/musprof/pmc2 -o run --output-format csv -- python3 tools/session_rate.py museum --reps 1 "" > gpurun_out/prof_museum/pmc2.log 2>&1 || exit 1
python3 tools/pmc.py /tmp/musprof > gpurun_out/prof_museum/pmc_summary.json
head -12 gpurun_out/prof_museum/kernel_stats.csv | cut -c1-160
