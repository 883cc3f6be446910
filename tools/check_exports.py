"""Fails (exit 1) if a built libwpt*.so lacks a function include/wpt.h
declares. Run by the csrc Makefile after linking the product and every
`make variant` build, so an A/B library can never silently predate an export
the Python binding (wasm-pathtracer_amd/_lib.py) uses.
Usage: python3 tools/check_exports.py LIB.so"""
import os
import re
import subprocess
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
want = set(re.findall(r"\b(wpt_[a-z_0-9]+)\s*\(", open(os.path.join(root, "include", "wpt.h")).read()))
out = subprocess.run(["nm", "-D", "--defined-only", sys.argv[1]], capture_output=True, text=True, check=True).stdout
have = {line.split()[-1] for line in out.splitlines() if line.strip()}
missing = sorted(want - have)
if missing:
    print(f"{sys.argv[1]}: missing exports declared in include/wpt.h: {missing}", file=sys.stderr)
    sys.exit(1)
