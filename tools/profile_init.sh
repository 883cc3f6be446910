# Kernel trace of the init-default session (tools/session_rate.py init: one
# warm-up call, then 3 timed compute(W*H*16) calls) and its timeline summary.
# Usage on the box: bash tools/profile_init.sh TAG ["opt=v,..."]
export TMPDIR=/tmp
O=gpurun_out/prof_init_${1:-x}
mkdir -p $O /tmp/initprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/initprof/trace -o run --output-format csv -- python3 tools/session_rate.py init --reps 1 "${2:-}" > $O/trace.log 2>&1 || exit 1
cp $(find /tmp/initprof/trace -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
python3 tools/timeline.py /tmp/initprof/trace > $O/timeline.json || exit 1
python3 tools/init_phases.py /tmp/initprof/trace > $O/phases.json || exit 1
ls -la $O
