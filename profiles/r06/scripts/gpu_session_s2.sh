set -o pipefail
mkdir -p gpurun_out
bash tools/profile_init.sh log "log=1" && cp /tmp/initprof/trace/*/run_kernel_trace.csv gpurun_out/prof_init_log/ 2>/dev/null; find /tmp/initprof/trace -name "*kernel_trace.csv" -exec cp {} gpurun_out/prof_init_log/kernel_trace.csv \; ; ls -la gpurun_out/prof_init_log
