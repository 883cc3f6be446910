# Round 5, thirteenth GPU session: are C5's late, small launches faster with
# the BVH4 walk (half the dependent steps per ray)? Wave-timeline probes of
# C5 with separate extend / shadow launches (fused_below=0), exact BVH2 vs
# the BVH4 fast path, per bounce.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u tools/probe_tails.py c5 1500 fused_below=0 > gpurun_out/r05/probe_c5_sep_bvh2.json 2> gpurun_out/r05/probe_c5_sep_bvh2.err || exit 1
timeout -k 10 300 python -u tools/probe_tails.py c5 1500 fused_below=0,traversal=bvh4,traversal_sh=bvh4 > gpurun_out/r05/probe_c5_sep_bvh4.json 2> gpurun_out/r05/probe_c5_sep_bvh4.err || exit 1
echo s13-done
