"""The BRIEF steering cos/sin of the kernel (multiagent_orb_slam2_amd/csrc/orbx_sincos.h) equals the
oracle's (float)cos((double)x) / (float)sin((double)x) (reference src/ORBextractor.cc:112-113 with the
build's pin) for EVERY float x in the kernel's input domain [0, 6.2832] (x = fastAtan2
degrees * (float)(pi/180), at most 360 * that).  oracle/sincos_check.c compiles the same header for the
host (explicit fma, no contraction: IEEE double ops round identically on gfx950) and compares all
~1.09e9 floats against libm."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(ROOT, "oracle", "sincos_check")


def _run(*args):
    if not os.path.exists(CHECK):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return subprocess.run([CHECK, *map(str, args)], capture_output=True, text=True, timeout=600)


def test_sincos_exhaustive_over_kernel_domain():
    r = _run(min(8, os.cpu_count() or 1))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout and "checked 1086918650" in r.stdout, r.stdout

