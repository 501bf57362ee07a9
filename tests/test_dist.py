"""CPU over gloo: the multi-GPU path (shard + end-of-step u0 gather) at world sizes
2 and 8 -- the 8-GPU node's rank count, at the bench configs' global totals."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "pympc-quadruped_amd")]
    from mpcqp.dist import gather_u0, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = shard(total, rank, world)
    # each rank "solves" its shard: u0 rows carry their global robot index
    u0 = torch.arange(start, start + count, dtype=torch.float32)[:, None].repeat(1, 12)
    full = gather_u0(u0, total=total)
    q.put((rank, full[:, 0].tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [8, 7])
def test_gather_u0_world2(total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r] == [float(i) for i in range(total)]


@pytest.mark.parametrize("total", [2048, 7])
def test_bench_spawns_its_own_ranks(total):
    """`python bench.py --gpus 2` with no WORLD_SIZE spawns the two ranks itself (the
    parent makes no HIP call); --rehearse-cpu runs the rank logic over gloo on CPU
    tensors -- shard, stand-in solve, u0 all-gather (uneven shards for 7 robots),
    max-over-ranks timing -- and rank 0 prints one line with n_gpus = 2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--rehearse-cpu",
                          "--steps", "3", "--total", str(total), "--no-cpu"],
                         capture_output=True, text=True, timeout=300, env=env, check=True)
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout   # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["rehearsal"] is True
    assert line["gathered_rows"] == total and line["gather_ok"] is True
    assert line["config"]["global_batch"] == total


@pytest.mark.parametrize("config,total", [("config4", 0), ("config5", 0), ("config4", 16381), ("config2", 8191)])
def test_bench_rehearsal_world8(config, total):
    """`bench.py --gpus 8 --rehearse-cpu`: eight gloo ranks, each building its shard of the
    config's real workload (CONFIGS[config]: batch per GPU, horizon, gaits, robots; config
    4: 8 x 2048 = 16 384 robots at N = 16, config 5: 8 x 8192 = 65 536 at N = 20) or of an
    uneven global total, then the u0 all-gather: every robot's row arrives in global order
    on rank 0 (the loop it replaces is isaacgym_a1.py:119-164)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from mpcqp.dist import shard
    bpg, N = bench.CONFIGS[config][0], bench.CONFIGS[config][1]
    world = 8
    want_total = total or world * bpg
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    # the CPU baseline leg runs once (config 2's 1 024-robot shard); the big shards skip it
    cpu = ["--cpu-seconds", "0.4"] if config == "config2" else ["--no-cpu"]
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--rehearse-cpu",
           "--config", config, "--steps", "2"] + (["--total", str(total)] if total else []) + cpu
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, check=True)
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["gathered_rows"] == want_total and line["gather_ok"] is True
    assert line["config"]["global_batch"] == want_total and line["horizon"] == N
    assert line["per_rank_batch"] == [shard(want_total, r, world)[1] for r in range(world)]
    # the same key set as the measured N = 1 line (tests/test_gpu_dist.py::test_bench_contract_line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    if config == "config2":
        c = line["cpu_baseline"]
        assert c["kind"] == "port" and c["value"] > 0 and c["single_core"]["cores"] == 1 and "rank 0" in c["note"]
