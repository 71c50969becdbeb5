"""The N > 1 path as the driver runs it: `bench.py --gpus N` starting its own ranks, the keyframe all-gather over RCCL
(torch.distributed nccl and liborbx's native orbx_exchange communicator), and the whole step at world 2.

The RCCL cases need one GPU per rank and skip on a box with fewer (an 8-GPU node runs them); the gloo rehearsal runs
two ranks on one GPU -- the packets staged through host memory -- so the full N > 1 step (tracking, CreateNewMapPoints,
Fuse, the exchange, MapFusion's query-then-add and the cross-agent SearchByBoW gate) runs on every GPU box.
Every child runs under its own time limit; the test process only waits for them."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "2", "--batch", "16", "--cpu-seconds", "0", "--host-api-frames", "0", "--no-c3",
         "--no-cd", "--host-fed-steps", "0", "--alone-reps", "0"]


def _gpus():
    import torch
    return torch.cuda.device_count()


def _env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}


def _bench(args, timeout=300):
    r = subprocess.run(["timeout", "-k", "10", str(timeout), sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, env=_env(), cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_world2(d, backend):
    assert d["n_gpus"] == 2 and d["ranks"]["world_size"] == 2 and d["ranks"]["backend"] == backend
    assert d["ranks"]["launched_by"] == "bench.py --gpus"
    assert d["config"]["global_batch"] == 32 and d["config"]["parallelism"] == "agent-per-gpu x2"
    # rank r's frames are its chunk of the sequence (generic_split_seq.cc:543-589): rank 0 holds the first half
    assert d["config"]["sequence_chunk"] == [0, 2271]
    # default scenes: 15 distinct (a multiple of 5), keyframes at the sequence's frames = 0 mod 5 (rows 0, 5, 10 on rank 0)
    assert d["config"]["distinct_stereo_pairs_per_gpu"] == 15 and d["config"]["keyframe_rows"] == [0, 15, 5]
    x = d["exchange"]
    assert x["calls"] == 2 and x["bytes_per_allgather"] == 2 * 3 * x["packet_bytes"]
    assert all(s["data_ok"] for s in d["xgmi_allgather"]["sweep"])
    # keyframes of the other agent reach MapFusion's 20-match gate (MapFusion.cc:275-281)
    assert d["fusion_gate_passed_per_step"] > 0
    assert d["value"] > 0 and abs(d["value"] - 32 * 1000.0 / d["ms_per_step"]) / d["value"] < 0.01


def test_bench_world2_gloo_rehearsal_one_gpu(gpu):
    """`bench.py --gpus 2 --dist-backend gloo`: two ranks on this box's GPU(s), the full step at world 2."""
    d = _bench(["--gpus", "2", "--dist-backend", "gloo", "--xgmi-mb", "0.17"] + SMALL)
    _check_world2(d, "gloo")
    if _gpus() < 2:
        assert "rehearsal" in d and d["ranks"]["devices_used"] == 1


@pytest.mark.parametrize("exchange", ["torch", "native"])
def test_bench_world2_rccl(gpu, exchange):
    """`bench.py --gpus 2` over RCCL, one rank per GPU: torch.distributed's nccl all-gather, or liborbx's own RCCL
    communicator (orbx_exchange_allgather_device, the C++ MultiAgentServer path)."""
    if _gpus() < 2:
        pytest.skip("needs 2 GPUs (one rank per GPU over RCCL)")
    d = _bench(["--gpus", "2", "--exchange", exchange, "--xgmi-mb", "0.17,16"] + SMALL)
    _check_world2(d, "nccl")
    assert "rehearsal" not in d and d["ranks"]["devices_used"] == 2
    assert ("orbx_exchange" in d["exchange"]["collective"]) == (exchange == "native")


_RCCL_CHILD = r"""
import os, sys, time
sys.path.insert(0, sys.argv[1])
import torch
import multiagent_orb_slam2_amd as pkg
rank, world, uidf = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
torch.cuda.set_device(rank)
if rank == 0:
    with open(uidf + ".tmp", "wb") as f:
        f.write(pkg.KeyframeExchangeRCCL.unique_id())
    os.rename(uidf + ".tmp", uidf)
t_end = time.time() + 60
while not os.path.exists(uidf):
    assert time.time() < t_end, "no unique id from rank 0"
    time.sleep(0.05)
uid = open(uidf, "rb").read()
x = pkg.KeyframeExchangeRCCL(uid, world, rank, rank)
n, P = 3, 172096
send = torch.full((n, P), rank + 1, dtype=torch.uint8, device=f"cuda:{rank}")
send[:, 0] = 100 + rank
recv = torch.zeros((world * n, P), dtype=torch.uint8, device=f"cuda:{rank}")
torch.cuda.synchronize()
s = torch.cuda.Stream()
x.allgather(send, recv, stream=s)
s.synchronize()
for r in range(world):
    blk = recv[r * n:(r + 1) * n]
    assert int(blk[:, 0].min()) == int(blk[:, 0].max()) == 100 + r, r
    assert int(blk[:, 1:].min()) == int(blk[:, 1:].max()) == r + 1, r
x.close()
pkg.orbx.device_check(rank)
print("rank", rank, "ok")
"""


def test_native_rccl_exchange_world2(gpu, tmp_path):
    """orbx_exchange at world 2: the unique id from rank 0, one communicator per process, keyframe packets all-gathered
    rank-major (the MapFusion ingress, MapFusion.cc:83-88)."""
    if _gpus() < 2:
        pytest.skip("needs 2 GPUs (one rank per GPU over RCCL)")
    uidf = str(tmp_path / "uid")
    procs = [subprocess.Popen(["timeout", "-k", "10", "120", sys.executable, "-c", _RCCL_CHILD, ROOT, str(r), "2", uidf],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=_env()) for r in range(2)]
    outs = [p.communicate() for p in procs]
    for r, (p, (o, e)) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, (r, e[-2000:])
        assert f"rank {r} ok" in o
