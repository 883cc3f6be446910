#!/bin/bash
# SQ / TA / TCP counters of C5's kernels (k_trace, k_shade, k_extend, k_shadow): one C5 step.
export TMPDIR=/tmp
PMC_ARGS="--config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-serial-step" PMC_KERNELS="k_trace k_shade k_extend k_shadow" bash tools/pmc_ab.sh c5 base
