# rocprofv3 stochastic PC sampling (beta) of one C3 production step, on the
# line-table build (WPT_LIB_VARIANT=dbg: make variant V=dbg
# VFLAGS=-gline-tables-only; the same code as the product). Usage on the box:
# bash tools/pc_sample.sh [interval]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05/pcs
mkdir -p $OUT
WPT_LIB_VARIANT=dbg timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
  --pc-sampling-unit cycles --pc-sampling-interval ${1:-1048576} -d $OUT -o pcs --output-format csv \
  -- python3 tools/one_step.py c3 1 > $OUT/run.log 2>&1
echo pcs rc=$?
ls -la $OUT | head
