"""The traversal kernels' residency, pinned at build level (CPU only).

DESIGN.md §5 "Occupancy" / "No SLP vectoriser": the production (triangle-only,
non-counting) traversal kernels k_extend, k_shadow (exact BVH2, the default on
triangle scenes) and the fused k_trace run at
8 waves per SIMD, which needs <= 64 VGPRs, <= 80 SGPRs and no scratch, and
k_shade on NEE scenes at 7 (<= 72 VGPRs). The test compiles wpt_render.hip for
gfx950 with the Makefile's own `asm` command line (so it follows the Makefile's
flags, -fno-slp-vectorize included) and reads the kernels' resource metadata.
"""
import os
import re
import shlex
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "wasm-pathtracer_amd", "csrc")

# mangled-name fragment -> (max VGPRs, max SGPRs); scratch must be 0
LIMITS = {
    "k_extendILb1ELb0ELi0E": (64, 80),   # k_extend<TRI_ONLY, !COUNT, exact BVH2> (triangle scenes' default)
    "k_shadowILb1ELb0ELi0E": (64, 80),   # k_shadow<TRI_ONLY, !COUNT, exact BVH2>
    "k_traceILb1ELb0EE": (64, 80),       # k_trace<TRI_ONLY, !COUNT> (exact BVH2)
    "k_shadeILb1ELb0ELi0E": (72, 106),   # k_shade<TRI_ONLY, NEE, no octree>
}


def _asm_command(out):
    if shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("make / hipcc not available")
    lines = subprocess.run(["make", "-s", "-n", "asm"], cwd=CSRC, capture_output=True, text=True,
                           check=True).stdout.splitlines()
    cmd = next(l for l in lines if "hipcc" in l and "wpt_render.hip" in l)
    args = shlex.split(cmd)
    args[args.index("-o") + 1] = out
    return [a for a in args if not a.startswith("-Rpass")]


def test_traversal_kernels_fit_eight_waves(tmp_path):
    out = str(tmp_path / "wpt_render.s")
    subprocess.run(_asm_command(out), cwd=CSRC, check=True, capture_output=True, timeout=600)
    text = open(out).read()
    seen = {}
    for blk in text.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        for frag in LIMITS:
            if frag in name:
                seen[frag] = (int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1)),
                              int(re.search(r"\.sgpr_count:\s+(\d+)", blk).group(1)),
                              int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk).group(1)))
    assert set(seen) == set(LIMITS), f"kernels not found: {set(LIMITS) - set(seen)}"
    for frag, (v, s, scratch) in seen.items():
        vmax, smax = LIMITS[frag]
        assert v <= vmax and s <= smax and scratch == 0, (frag, v, s, scratch)
