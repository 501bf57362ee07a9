"""GPU: bench.py's single-GPU path end to end (one JSON line, the contract fields)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def test_bench_contract_line():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                          "--cpu-seconds", "0.5"], capture_output=True, text=True, timeout=600, check=True)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["value"] > 0 and line["n_gpus"] == 1 and line["scaling"] == "weak"
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(line["roofline"])
    assert line["roofline"]["bound"] == "valu"   # FP64 vector pipe: no MFMA on the path
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] >= 1 and cpu["value"] > 0
    assert cpu["single_core"]["cores"] == 1 and cpu["single_core"]["value"] > 0
    assert line["status_ok_frac"] == 1.0


def test_bench_config1_drop_in_latency():
    """Config 1: the drop-in controller's per-tick latency line (B = 1, horizon 16)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "config1", "--steps", "5",
                          "--warmup", "2", "--cpu-seconds", "0.5"], capture_output=True, text=True, timeout=600,
                         check=True)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["higher_is_better"] is False and line["unit"] == "ms" and line["value"] > 0
    assert line["config"]["horizon"] == 16 and line["cpu_baseline"]["value"] > 0


_NCCL_WORLD1 = r'''
import os, sys, socket
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "pympc-quadruped_amd")]
with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
import torch
import torch.distributed as dist
from mpcqp import LinearMpc
from mpcqp.dist import gather_u0
from mpcqp.synthetic import make_batch
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
B = 256
bt = make_batch(B, 10, seed=1000, gaits=("trot10",), robots=("a1",))
eng = LinearMpc(horizon=10, robot="a1", device=dev)
res = eng.solve(bt["x0"], bt["xref"], bt["contact"], bt["feet"], robot=bt["robot"], return_all=True)
u0 = res.u0.contiguous()
assert u0.is_cuda and u0.dtype == torch.float32 and tuple(u0.shape) == (B, 12)
out = torch.empty_like(u0)
# the exact collective gather_u0 issues for world > 1 (mpcqp/dist.py), on RCCL
dist.all_gather_into_tensor(out, u0)
torch.cuda.synchronize(dev)
assert torch.equal(out, u0)
assert torch.equal(gather_u0(u0, total=B), u0)
assert int((res.status != 0).sum()) == 0
dist.barrier()
dist.destroy_process_group()
print("nccl world-1 all-gather ok", float(u0.abs().max()))
'''


def test_rccl_world1_all_gather():
    """The RCCL path itself (backend "nccl" = RCCL on ROCm): a one-rank communicator on the
    GPU box, the engine's u0 [B, 12] f32 through dist.all_gather_into_tensor -- the call
    gather_u0 makes at mpcqp/dist.py for world > 1 (isaacgym_a1.py:161-164's gather)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "-c", _NCCL_WORLD1, ROOT], capture_output=True, text=True,
                         timeout=240, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "nccl world-1 all-gather ok" in out.stdout


def test_bench_two_ranks_real_engine():
    """bench.py's N > 1 path with the real engine: two ranks on the one GPU of the box
    (RCCL refuses two ranks on one device, so the gather runs over gloo here), each solving
    its own seeded shard -- every robot status 0 -- and rank 0's line carrying the N = 1
    line's key set, the CPU baseline included."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MPCQP_BENCH_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
                          "--warmup", "1", "--cpu-seconds", "0.5", "--no-callers", "--event-every", "1"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 2048
    assert line["status_ok_frac"] == 1.0 and line["cpu_baseline"]["value"] > 0
    assert line["gather_ms_avg"] > 0 and "gloo" in line["config"]["parallelism"]
