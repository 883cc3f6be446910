set -o pipefail
mkdir -p gpurun_out/s39
timeout -k 10 400 python3 tools/mem_cycle.py init --reps 12 --spp 2 > gpurun_out/s39/mem.jsonl 2> gpurun_out/s39/mem.err || { echo FAIL1; tail -5 gpurun_out/s39/mem.err; exit 1; }
cat gpurun_out/s39/mem.jsonl
