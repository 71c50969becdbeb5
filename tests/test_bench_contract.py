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


# ---- `bench.py --gpus N`: the rank launcher (CPU: children that do not touch a GPU) ----

def test_rank_env_and_world_checks(monkeypatch):
    b = _bench()
    e = b.rank_env({"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 3, 8, 29511)
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == ("3", "3", "8", "8")
    assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
    assert e["PATH"] == "/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"      # the caller's env is kept
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert b.world_from_env(1) == (False, 1)
    assert b.world_from_env(4) == (True, 1)            # no launcher: bench.py starts the 4 ranks itself
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert b.world_from_env(4) == (False, 4)           # torchrun's ranks: run as one of them
    with pytest.raises(SystemExit):
        b.world_from_env(8)                            # torchrun of 4 ranks asked for 8 GPUs: an error, not a 1-rank line


def _launch(world, child_src, timeout=120):
    import subprocess
    drv = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
           f"sys.exit(bench.launch_ranks({world}, [sys.executable, '-c', {child_src!r}], grace_s=5.0))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, "-c", drv], capture_output=True, text=True, timeout=timeout, env=env)


def test_launcher_starts_n_ranks_gloo_world2():
    """Two ranks from the launcher rendezvous over gloo on 127.0.0.1 and all-gather their ranks; only rank 0's line is
    on stdout (the driver reads one JSON line), the other rank's stdout goes to stderr."""
    child = ("import json, os, torch, torch.distributed as dist\n"
             "dist.init_process_group('gloo')\n"
             "t = [torch.zeros(1, dtype=torch.int64) for _ in range(dist.get_world_size())]\n"
             "dist.all_gather(t, torch.tensor([int(os.environ['RANK']) * 10 + int(os.environ['LOCAL_RANK'])]))\n"
             "print(json.dumps({'rank': dist.get_rank(), 'world': dist.get_world_size(), 'got': [int(x) for x in t],"
             " 'launcher': os.environ['ORBX_LAUNCHER']}), flush=True)\n"
             "dist.destroy_process_group()\n")
    r = _launch(2, child)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d == {"rank": 0, "world": 2, "got": [0, 11], "launcher": "bench.py --gpus"}
    assert '"rank": 1' in r.stderr


def test_launcher_failure_stops_peers():
    """A rank that fails ends the job with its status; a peer that would wait forever (as one blocked in a collective
    whose peer died) is stopped."""
    import time
    child = ("import os, sys, time\n"
             "if os.environ['RANK'] == '1': sys.exit(3)\n"
             "time.sleep(600)\n")
    t0 = time.monotonic()
    r = _launch(2, child)
    assert r.returncode == 3
    assert time.monotonic() - t0 < 60
