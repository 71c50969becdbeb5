"""The native multi-thread driver (tests/native/concurrency.cpp, built by `make` as build/concurrency) on the GPU: the
C-ABI called from C++ std::threads as the reference's own threads call ORBextractor / ORBmatcher / KeyFrameDatabase
(src/Frame.cc:78-81, :101; KeyFrameDatabase.cc:42-316) -- two extractors and four matchers on six threads, three
agents building stereo Frames at once (orbx_stereo_frame and the two-call form in turn), fresh extractors' first calls
racing on six threads, and the KeyFrameDatabase's detect / add / erase threads replayed in order.  Every repetition must equal the first result bit for bit (the Python
tests check those first results against the oracle); exit status = number of mismatches."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "concurrency")


def test_native_threads_bit_stable(gpu):
    if not os.path.exists(EXE):
        pytest.fail("build/concurrency is missing: run make (or __graft_entry__.build()) first")
    p = subprocess.run([EXE, "4"], capture_output=True, text=True, timeout=150)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out
    assert "0 mismatches" in out and "stereo frames: 3 agents" in out and "first calls:" in out, out
