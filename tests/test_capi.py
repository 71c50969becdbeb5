"""C-ABI surface checks that need no GPU: liborbx.so loads, exports every function include/orbx.h
declares, reports errors through status codes (no exceptions, no crash) when no device is present."""
import ctypes as C
import os
import subprocess

import pytest

import multiagent_orb_slam2_amd as pkg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    lib = pkg.load_library()
    declared = pkg.declared_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing


def test_exported_symbols_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.orbx.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in pkg.declared_symbols():
        assert s in exported, s


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", pkg.orbx.LIB_PATH],
                         capture_output=True, text=True)
    text = out.stdout + out.stderr
    assert "gfx950" in text


def test_constants_and_version():
    lib = pkg.load_library()
    assert lib.orbx_th_high() == 100 and lib.orbx_th_low() == 50 and lib.orbx_histo_length() == 30
    assert lib.orbx_version().decode().startswith("orbx")


def test_no_device_reports_error_without_throwing():
    lib = pkg.load_library()
    if lib.orbx_device_count() > 0:
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    rc = lib.orbx_extractor_create(2000, C.c_float(1.2), 8, 20, 7, 0, C.byref(h))
    assert rc in (pkg.orbx.ORBX_ERR_HIP, pkg.orbx.ORBX_ERR_ARG)
    assert h.value is None
    assert len(lib.orbx_last_error()) > 0
    with pytest.raises(pkg.OrbxError):
        pkg.ORBextractor(2000, 1.2, 8, 20, 7)


def test_null_arguments_are_rejected():
    lib = pkg.load_library()
    assert lib.orbx_extractor_create(2000, C.c_float(1.2), 8, 20, 7, 0, None) == pkg.orbx.ORBX_ERR_ARG
    assert lib.orbx_extract(None, None, 0, 0, 0, None, None, 0, None) == pkg.orbx.ORBX_ERR_ARG
    assert lib.orbx_extractor_destroy(None) == 0
    assert lib.orbx_matcher_destroy(None) == 0


def test_header_compiles_as_c():
    src = os.path.join(ROOT, "include", "orbx.h")
    r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Werror", "-x", "c", src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_keypoint_layout_matches_cv_keypoint():
    assert pkg.KP_DTYPE.itemsize == 28
    assert list(pkg.KP_DTYPE.names) == ["x", "y", "size", "angle", "response", "octave", "class_id"]


def test_packet_layout_matches_python():
    """The native keyframe packet layout (orbx_packet_layout) equals multiagent.PacketLayout byte for byte."""
    from multiagent_orb_slam2_amd import multiagent as MA
    from multiagent_orb_slam2_amd.orbx import packet_layout
    for cap in (1, 64, 320, 1203, 2045, 4096):
        off, nbytes = packet_layout(cap)
        lay = MA.PacketLayout(cap)
        assert nbytes == lay.bytes and off == lay.offsets, cap
