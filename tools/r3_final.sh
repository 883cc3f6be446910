#!/bin/bash
# Evidence run of the build: whole GPU suite, the default bench line, smoke(),
# then the C3 profile (kernel trace + PMC passes) summarised into profiles/r03.
export TMPDIR=/tmp
set -o pipefail
bash tools/r3_head.sh || exit 1
cp gpurun_out/head/bench.json gpurun_out/head/c3_bench_line.json
bash tools/r3_prof3.sh || exit 1
echo final-done
