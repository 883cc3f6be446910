"""msincos (wpt_math.h), the hemisphere sample's sin and cos from one
reduction, is msin / mcos bit for bit on its domain [0, 9pi/4]: every 31st
float here (tools/sincos_check.cpp; with step 1, all 1.09e9 floats of the
range: 0 mismatches), and the last float of the range."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_msincos_matches_msin_mcos(tmp_path):
    exe = tmp_path / "sincos_check"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-I", os.path.join(ROOT, "wasm-pathtracer_amd", "csrc"),
                    "-o", str(exe), os.path.join(ROOT, "tools", "sincos_check.cpp")], check=True)
    r = subprocess.run([str(exe), "31"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout
