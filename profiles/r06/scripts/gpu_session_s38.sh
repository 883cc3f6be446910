set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s38 /tmp/s38
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/s38/trace -o run --output-format csv -- python3 tools/session_rate.py init --reps 4 "stock_every=3" > gpurun_out/s38/trace.log 2>&1 || { echo FAIL1; tail -5 gpurun_out/s38/trace.log; exit 1; }
tail -1 gpurun_out/s38/trace.log
python3 tools/find_stall.py /tmp/s38/trace > gpurun_out/s38/stall.txt || exit 1
cat gpurun_out/s38/stall.txt
f=$(find /tmp/s38/trace -name "*kernel_trace.csv" | head -1); gzip -c "$f" > gpurun_out/s38/kernel_trace.csv.gz
