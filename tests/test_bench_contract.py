"""bench.py's driver contract: one JSON line with the contract fields, the roofline / cpu_baseline blocks built from
SURVEY §8(d)'s per-unit bytes.  The CPU test checks the argument defaults and the algorithmic bytes; the GPU test runs a
short in-process bench (no subprocess: the test process has initialised the GPU) and validates the line."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    return bench


def test_defaults_and_compulsory_bytes(monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = b.parse()
    assert (a.gpus, a.steps, a.warmup, a.config, a.batch) == (1, 20, 5, "kitti", 256)
    assert a.desc_stream == 1 and a.sets == 3          # the measured schedule
    cb = b.compulsory_bytes(b.CONFIGS["kitti"])
    assert cb["extraction"] == 375 * 1242 + 2000 * 60 == 585750
    assert cb["stereo_match"] == 2 * 2000 * 32 + 2000 * 8
    assert b.compulsory_bytes(b.CONFIGS["euroc"])["extraction"] == 480 * 752 + 1200 * 60


@pytest.mark.gpu
def test_bench_json_line(gpu, capsys, monkeypatch):
    b = _bench()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "2", "--warmup", "3", "--batch", "16", "--cpu-seconds", "0",
                                      "--host-api-frames", "0", "--no-c3", "--host-fed-steps", "2"])
    import torch
    prev = torch.cuda.current_stream()
    try:
        b.main()
    finally:
        torch.cuda.synchronize()
        torch.cuda.set_stream(prev)                  # main() makes its front-end stream current
    d = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 3 and d["higher_is_better"] is True
    assert d["unit"] == "frames/s" and d["scaling"] == "weak" and d["vs_baseline"] is None and d["dtype"] == "u8"
    assert d["value"] > 0 and abs(d["value"] - 16 * 1000.0 / d["ms_per_step"]) / d["value"] < 0.01
    r = d["roofline"]
    assert r["algorithmic_bytes_per_step"] == 585750 * 32 and r["units_per_step"] == 32
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-4
    # achieved = algorithmic bytes per step / the kernel's live time per step (its launches' event spans summed)
    assert abs(r["achieved"] - r["algorithmic_bytes_per_step"] / (r["kernel_ms_per_step"] * 1e-3) / 1e9) / r["achieved"] < 1e-3
    assert r["kernel"].startswith("k_fast_wave") and r["launches_per_step"] == 2
    assert d["host_fed"]["frames_per_s"] > 0 and d["host_fed"]["input_bytes_per_step"] == 32 * 375 * 1242
    cd = d["covisibility_discovery"]
    assert cd["absorbed_keyframes"] == 16 and cd["searchbybow_pairs"] >= 1
    assert d["config"]["frames_per_gpu_per_step"] == 16 and d["config"]["keyframes_per_gpu_per_step"] == 3
