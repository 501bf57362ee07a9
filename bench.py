"""bench.py -- QP solves/sec of the MI355X batched MPC engine (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W
  (N > 1: one rank per GPU over RCCL -- launched by torch.distributed.run, or, when
  WORLD_SIZE is unset, by bench.py itself: the parent spawns the N ranks before any
  HIP call and exits with their status)
  python bench.py --config config1      # the drop-in controller's per-tick latency (B = 1)

Workload (BASELINE.json configs[1]): per GPU B = 1024 A1 robots, trotting
(trot10), horizon N = 10, synthetic seeded states; weak scaling
(B per GPU is fixed as N grows).  One step = one pass of the hot path over the
batch: formulate (model, exact discretisation, condensing, H/g, cone rows) and
solve every robot's QP, plus -- on N > 1 -- the end-of-step RCCL all-gather of
u0 (the only exchange the path has).  Inputs are resident in HBM before the
timed region.

Prints ONE JSON line on rank 0 (metric/value/unit/... + roofline + cpu_baseline).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd"))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (batch per GPU, horizon, gaits, robots, tilt)
    "config2": (1024, 10, ("trot10",), ("a1",), 0.0),
    "config3": (4096, 10, ("trot10", "pace10", "bound8"), ("a1",), 0.0),
    "config4": (2048, 16, ("trot10", "pace10", "bound8"), ("a1",), 0.0),
    "config5": (8192, 20, ("trot10", "pace10", "bound8"), ("a1", "aliengo"), 15.0),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="config2", choices=sorted(CONFIGS) + ["config1"])
    ap.add_argument("--warm-fleet", action="store_true",
                    help="a fleet solved tick after tick: the batches are a drift sequence (x0 + N(0, 2e-3) "
                         "per tick, visited 0 1 2 3 2 1 ...) and the engine remembers each robot's active set "
                         "(LinearMpc.set_warm_start); an extra line, never the headline")
    ap.add_argument("--standing-every", type=int, default=0,
                    help="diagnostics: make every k-th robot stand (the interior-point class)")
    ap.add_argument("--cross-leg-r", action="store_true",
                    help="weights: the reference Q and an R coupling every pair of legs (mpcqp_set_weights)")
    ap.add_argument("--gait", default="trot10",
                    help="config1: the drop-in's gait (trot10 = Gait.TROTTING10; standing = Gait.STANDING, "
                         "the interior-point class at horizon 16)")
    ap.add_argument("--total", type=int, default=0, help="--rehearse-cpu: global robots (uneven shards)")
    ap.add_argument("--rehearse-cpu", action="store_true",
                    help="no GPU: rehearse the rank / shard / gather logic over gloo with a stand-in "
                         "that zero-fills u0 (no solve, not a measurement)")
    ap.add_argument("--batch", type=int, default=0, help="override batch per GPU")
    ap.add_argument("--no-gather", action="store_true", help="skip the end-of-step u0 gather")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--max-iter", type=int, default=0, help="active-set iteration cap (diagnostics only)")
    ap.add_argument("--step-events", action="store_true",
                    help="diagnostics: one HIP event pair per step (perturbs back-to-back dispatch, "
                         "~5%% slower steps); default: one pair around the timed loop")
    ap.add_argument("--no-callers", action="store_true", help="skip the planner/torque kernel timing")
    ap.add_argument("--order", type=int, default=1, choices=(0, 1),
                    help="dispatch order (mpcqp_set_order): 1 = largest predicted solve time first, 0 = batch order")
    ap.add_argument("--no-hint-line", action="store_true",
                    help="skip the no_hint sub-line (the default caller path without a stance promise)")
    ap.add_argument("--event-every", type=int, default=8,
                    help="N > 1: bracket every k-th step's solve and gather with HIP events (sampled)")
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "latest", "pmc_traffic.json"))
    return ap.parse_args()


def cpu_baseline(bt, N, budget_s, threads=1):
    """The compiled CPU restatement of the reference's per-tick formulate + solve
    (oracle/cpu_mpc.cpp: float32 model and dense condensing as mpc.py:173-233 builds them,
    float64 Goldfarb-Idnani solve), OpenMP over the batch's robots with `threads`
    threads, cycling over the batch until `budget_s` is spent.  Returns robots / s, robots
    solved, wall seconds, and the formulation / solve thread-seconds per robot."""
    from oracle import cpu_port
    cpu_port.solve_batch({k: v[:8] for k, v in bt.items()}, N, threads=threads)   # warm the pool
    t0 = time.perf_counter()
    done, tf, ts = 0, 0.0, 0.0
    while True:
        _, _, f, s_ = cpu_port.solve_batch(bt, N, threads=threads)
        done += int(bt["x0"].shape[0])
        tf += f
        ts += s_
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return done / dt, done, dt, tf / done, ts / done


def cpu_baseline_line(bt, N, seconds, world):
    """The `cpu_baseline` object: the compiled port timed on this host's cores (rank 0 only,
    after the measured region -- with N > 1 the other ranks are idle by then), 16 threads
    (the box's CPU share per GPU) and 1 thread, half of `seconds` each."""
    procs = _host_cores()
    v1, done1, dt1, f1, s1 = cpu_baseline(bt, N, seconds / 2, threads=1)
    vm, donem, dtm, fm, sm_ = cpu_baseline(bt, N, seconds / 2, threads=procs)
    cpu = {"value": vm, "unit": "QP/s", "cores": procs, "kind": "port",
           "sample": f"{donem} robot solves (the config's first synthetic batch, cycled) in {dtm:.1f}s, "
                     f"OpenMP {procs} threads ({_cpu_model()}): compiled restatement of the reference's "
                     "formulation (float32 model, dense condensing, mpc.py:173-260) + float64 "
                     "Goldfarb-Idnani QP (oracle/cpu_mpc.cpp, g++ -O3)",
           "formulation_us_per_robot": fm * 1e6, "solve_us_per_robot": sm_ * 1e6,
           "single_core": {"value": v1, "cores": 1, "formulation_us": f1 * 1e6, "solve_us": s1 * 1e6,
                           "sample": f"{done1} robots in {dt1:.1f}s, 1 thread"}}
    if world > 1:
        cpu["note"] = (f"timed on rank 0's host after the {world}-rank measured region: one host's "
                       f"{procs} threads, not {world} hosts' -- the same baseline as the N = 1 line")
    return cpu


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _host_cores():
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    # the box's share: OMP_NUM_THREADS / MAX_JOBS are set to it (16 for one GPU)
    return max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", "16")), 16))


def time_callers(eng, h, B, N, dev, stream, reps=20):
    """The hot path's device callers on the same batch, outside the timed region
    (they are not part of `value`): one MPC-tick mpcqp_plan (Isaac Gym root-state
    input) and one mpcqp_stance_torques (f4), HIP events on the
    launch stream; achieved GB/s from mpcqp.roofline.plan_bytes / torque_bytes."""
    import numpy as np
    import torch
    from mpcqp._lib import PLAN_REFERENCE, PLAN_STRIDE
    from mpcqp.params import gait_record
    from mpcqp.roofline import PEAK_HBM_GBS, plan_bytes, torque_bytes
    rng = np.random.default_rng(17)
    f32 = dict(dtype=torch.float32, device=dev)
    rs = torch.as_tensor(rng.standard_normal((B, 13)).astype(np.float32)).to(dev)
    rs[:, 3:7] = torch.nn.functional.normalize(rs[:, 3:7], dim=1)
    vb = torch.as_tensor(np.tile([0.6, 0.0, 0.0], (B, 1))).to(dev)
    yr = torch.full((B,), 0.2, dtype=torch.float64, device=dev)
    gait = torch.as_tensor(np.tile(gait_record("trot10"), (B, 1))).to(dev)
    it = torch.zeros((B,), dtype=torch.int32, device=dev)
    hgt = torch.full((B,), 0.42, **f32)
    state = torch.zeros((B, PLAN_STRIDE), dtype=torch.float64, device=dev)
    x0 = torch.empty((B, 13), **f32)
    xref = torch.empty((B, N, 13), **f32)
    ct = torch.empty((B, N, 4), **f32)
    jac = torch.as_tensor(rng.standard_normal((B, 4, 3, 3)).astype(np.float32)).to(dev)
    stance = torch.as_tensor(h["contact"][:, 0, :].copy()).to(dev)
    u0 = torch.as_tensor(rng.standard_normal((B, 12)).astype(np.float32)).to(dev)
    tau = torch.zeros((B, 12), **f32)

    def plan():
        eng.plan(PLAN_REFERENCE, state, x0, vb, yr, root_states=rs, gait=gait, iteration=it,
                 height_des=hgt, xref=xref, contact=ct, stream=stream)

    def plan_tick():   # a control iteration between MPC ticks: pack + integrate only
        eng.plan(0, state, x0, vb, yr, root_states=rs, stream=stream)

    def torques():
        eng.stance_torques(jac, stance, u0, tau, stream=stream)

    out = {}
    for name, fn, nbytes in (("plan", plan, B * plan_bytes(N, True, True)),
                             ("plan_between_mpc_ticks", plan_tick, B * plan_bytes(N, False, True)),
                             ("stance_torques", torques,
                              B * torque_bytes(float(stance.mean().item())))):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize(dev)
        us = sum(a.elapsed_time(b) for a, b in ev) / reps * 1e3
        gbs = nbytes / (us * 1e-6) / 1e9
        out[name] = {"us_avg": us, "bytes": nbytes, "achieved_GBs": gbs, "frac_hbm": gbs / PEAK_HBM_GBS}
    return out


def spawn_ranks(n):
    """One child process per rank (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set), started
    before this process makes any HIP call; returns the worst exit status."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def rehearse_cpu(args, world, rank, dist):
    """The N > 1 rank logic on CPU tensors over gloo: every rank builds its shard of the
    workload (seed = base + rank), a stand-in zero-fills u0 (NO solve, NOT a measurement),
    the u0 all-gather runs, max-over-ranks timing, one JSON line from rank 0."""
    import numpy as np
    import torch
    from mpcqp.dist import gather_u0
    from mpcqp.synthetic import make_batch
    Bpg, N, gaits, robots, tilt = CONFIGS[args.config if args.config in CONFIGS else "config2"]
    if args.batch:
        Bpg = args.batch
    from mpcqp.dist import shard
    total = args.total if args.total else world * Bpg   # --total: uneven contiguous shards
    start, Bpg = shard(total, rank, world)
    h = make_batch(Bpg, N, seed=1000 + rank, gaits=gaits, robots=robots, tilt_deg=tilt)
    x0 = torch.as_tensor(h["x0"])
    u0 = torch.empty((Bpg, 12), dtype=torch.float32)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    rows, gather_ok = 0, True
    for _ in range(args.steps):
        # stand-in for the HIP solve: each row carries its global robot index
        u0.copy_(torch.arange(start, start + Bpg, dtype=torch.float32)[:, None].expand(Bpg, 12))
        allu = gather_u0(u0, total=total) if world > 1 else u0
        rows = int(allu.shape[0])
        gather_ok &= bool(torch.equal(allu[:, 0], torch.arange(total, dtype=torch.float32)))
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # every rank's shard size and its synthetic inputs' shapes, checked on rank 0
    shapes = torch.tensor([Bpg, h["xref"].shape[0], h["xref"].shape[1], h["contact"].shape[0]], dtype=torch.int64)
    allshapes = [torch.zeros_like(shapes) for _ in range(world)] if world > 1 else [shapes]
    if world > 1:
        dist.all_gather(allshapes, shapes)
    per_rank = [int(t[0]) for t in allshapes]
    assert all(int(t[1]) == int(t[0]) == int(t[3]) and int(t[2]) == N for t in allshapes), allshapes
    tmax = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    if rank == 0:
        el = float(tmax.item())
        cpu = None if args.no_cpu else cpu_baseline_line(h, N, args.cpu_seconds, world)
        print(json.dumps({"metric": "QP solves/sec (whole node), horizon=10 GRF QP, at 1/2/4/8 MI355X",
                          "value": world * Bpg * args.steps / el, "unit": "QP/s",
                          "n_gpus": world, "steps": args.steps, "warmup": 0,
                          "ms_per_step": el / max(args.steps, 1) * 1e3, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                          "data": "synthetic (seeded SURVEY §8(d) states; seed = base + rank)",
                          "roofline": None, "cpu_baseline": cpu, "rehearsal": True,
                          "note": "gloo rehearsal on CPU tensors: stand-in solve (zero fill), not a measurement",
                          "gathered_rows": rows, "gather_ok": gather_ok, "x0_rows": int(x0.shape[0]),
                          "per_rank_batch": per_rank, "horizon": N,
                          "config": {"workload": f"{args.config}: {total} robots over {world} ranks",
                                     "batch_per_gpu": Bpg, "horizon": N, "global_batch": total,
                                     "parallelism": f"robot-sharded x{world} + gloo all-gather of u0"}}))
    if world > 1:
        dist.destroy_process_group()


class _SyntheticRobotData:
    """The RobotData fields the drop-in controller reads (mpc.py:65-79, :83), for an
    Aliengo trotting forward (synthetic: no simulator in the loop)."""

    def __init__(self, t):
        import numpy as np
        yaw = 0.2 * np.sin(0.5 * t)
        self.pos_base = np.array([1.2 * t, 0.01 * np.sin(t), 0.38 + 0.01 * np.sin(7 * t)])
        self.lin_vel_base = np.array([1.2, 0.01 * np.cos(t), 0.07 * np.cos(7 * t)])
        self.ang_vel_base = np.array([0.05 * np.sin(3 * t), 0.03, 0.1 * np.cos(0.5 * t)])
        h = yaw / 2
        self.quat_base = np.array([np.cos(h), 0.0, 0.0, np.sin(h)])
        c, s = np.cos(yaw), np.sin(yaw)
        self.R_base = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])
        body = [(0.2399, 0.134), (0.2399, -0.134), (-0.2399, 0.134), (-0.2399, -0.134)]
        self.pos_base_feet = [self.R_base @ np.array([x, y, -0.38]) for x, y in body]


def bench_config1(args):
    """Config 1: the drop-in ModelPredictiveController (pympc-quadruped_amd/linear_mpc/mpc.py)
    in the control loop of scripts/mujoco_aliengo.py:184-207 at the reference defaults
    (Aliengo, LinearMpcConfig.horizon = 16, Gait.TROTTING10, 1 kHz control, an MPC solve
    every 20th iteration).  Reports the wall-clock latency of an MPC tick (state packing,
    device planner, formulate + solve, the D2H of the forces: what a 1 kHz loop waits for)
    and of the iterations between MPC ticks, next to the CPU restatement of the
    reference's per-tick formulation + solve on the same states (1 core)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "pympc-quadruped_amd", "linear_mpc"))
    import importlib
    mpc = importlib.import_module("mpc")
    from mpcqp.synthetic import gait_table
    from oracle import formulation as F

    class LinearMpcConfig:   # config/linear_mpc_configs.py:4-24 (values)
        dt_control = 0.001
        iteration_between_mpc = 20
        dt_mpc = 0.05
        horizon = 16
        gravity = 9.81
        friction_coef = 0.7
        Q = np.diag(F.Q_DIAG)
        R = np.diag(F.R_DIAG)

    al = F.ROBOTS["aliengo"]

    class AliengoConfig:     # config/robot_configs.py:44-60 (values)
        mass_base = al["mass"]
        base_height_des = al["height"]
        base_inertia_base = al["inertia"]
        fz_max = al["fz_max"]

    N = LinearMpcConfig.horizon
    n_iter = (args.warmup + args.steps) * LinearMpcConfig.iteration_between_mpc
    v_des = np.array([1.2, 0.0, 0.0])

    def run(warm):
        """The control loop; `warm` False: the engine's warm start (the previous tick's
        active set, interior-point class only) disabled, every tick solved cold."""
        ctl = mpc.ModelPredictiveController(LinearMpcConfig, AliengoConfig)
        mpc_ms, other_ms, states, iters = [], [], [], []
        for it in range(n_iter):
            rd = _SyntheticRobotData(it * 1e-3)
            table = gait_table(args.gait, (it // 20) % 10, N).reshape(-1)
            if it == 0 and not warm:
                ctl._get_engine().set_warm_start(0)
            t0 = time.perf_counter()
            ctl.update_robot_state(rd)
            u = ctl.update_mpc_if_needed(it, v_des, 0.0, table, solver="drake")
            dt = (time.perf_counter() - t0) * 1e3
            if it >= args.warmup * 20:
                if it % 20 == 0:
                    mpc_ms.append(dt)
                    iters.append(int(ctl._dev["iters"].item()))
                    if len(states) < 64:
                        states.append((ctl.current_state.copy(), ctl.ref_traj.copy(), table.copy(),
                                       [np.asarray(f) for f in rd.pos_base_feet]))
                else:
                    other_ms.append(dt)
        assert np.all(np.isfinite(u))
        return mpc_ms, other_ms, states, iters

    mpc_ms, other_ms, states, iters = run(True)
    cold_ms, _, _, cold_iters = run(False)
    cpu = None
    if not args.no_cpu:
        from mpcqp.params import pack_robot, ROBOT_PRESETS
        rec = pack_robot(ROBOT_PRESETS["aliengo"])
        bt = {"x0": np.stack([st[0] for st in states]), "xref": np.stack([st[1] for st in states]),
              "contact": np.stack([st[2] for st in states]),
              "feet": np.stack([np.asarray(st[3], np.float32).reshape(12) for st in states]),
              "robot": np.tile(rec, (len(states), 1))}
        rate, done, dt, f1, s1 = cpu_baseline(bt, N, args.cpu_seconds, threads=1)
        cpu = {"value": dt / done * 1e3, "unit": "ms/tick", "cores": 1, "kind": "port",
               "formulation_ms": f1 * 1e3, "solve_ms": s1 * 1e3,
               "sample": f"{done} MPC ticks of the same run's states, 1 thread ({_cpu_model()}): compiled "
                         "restatement of the reference's formulation + float64 Goldfarb-Idnani QP "
                         "(oracle/cpu_mpc.cpp)"}
    med = float(np.median(mpc_ms))
    print(json.dumps({
        "metric": f"drop-in MPC tick latency (B=1, Aliengo, horizon 16, {args.gait})",
        "value": med, "unit": "ms", "n_gpus": 1, "steps": len(mpc_ms), "warmup": args.warmup,
        "higher_is_better": False, "dtype": "f64", "data": "synthetic Aliengo trot states (no simulator)",
        "config": {"workload": "config1: ModelPredictiveController drop-in, scripts/mujoco_aliengo.py loop, "
                               f"LinearMpcConfig.horizon = 16, gait {args.gait}", "batch": 1, "horizon": N,
                   "gait": args.gait},
        "mpc_tick_ms": {"median": med, "p90": float(np.percentile(mpc_ms, 90)), "mean": float(np.mean(mpc_ms))},
        "warm_start": "the drop-in's default: each tick's interior-point solve (n > 128) starts from the "
                      "previous tick's verified active set (mpcqp_set_warm_start); the dense classes "
                      "always start cold",
        "iterations_median": float(np.median(iters)),
        "cold_mpc_tick_ms": {"median": float(np.median(cold_ms)), "p90": float(np.percentile(cold_ms, 90)),
                             "iterations_median": float(np.median(cold_iters))},
        "other_tick_ms": {"median": float(np.median(other_ms)), "p90": float(np.percentile(other_ms, 90))},
        "cpu_baseline": cpu,
    }))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.config == "config1":
        return bench_config1(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # one rank per GPU; ranks beyond the visible devices wrap around (only a rehearsal
    # of the N > 1 path on a smaller box does that).  MPCQP_BENCH_BACKEND=gloo is for
    # such rehearsals too: the measured path is "nccl" (RCCL over xGMI).
    if args.rehearse_cpu:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        return rehearse_cpu(args, world, rank, dist)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("MPCQP_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from mpcqp import LinearMpc
    from mpcqp.dist import gather_u0
    from mpcqp.synthetic import make_batch
    from mpcqp.roofline import PEAK_FP64_TFLOPS, algorithmic_flops, executed_flops

    Bpg, N, gaits, robots, tilt = CONFIGS[args.config]
    if args.batch:
        Bpg = args.batch
    # a few distinct seeded batches per rank, cycled over the steps (seed = base + rank)
    nbat = 4
    host = [make_batch(Bpg, N, seed=1000 * (k + 1) + rank, gaits=gaits, robots=robots, tilt_deg=tilt)
            for k in range(nbat)]
    if args.standing_every:
        for h in host:
            h["contact"][::args.standing_every] = 1.0
    if args.warm_fleet:   # consecutive ticks of one fleet: each batch the previous one drifted
        rng = np.random.default_rng(77 + rank)
        for k in range(1, nbat):
            h = {kk: v.copy() for kk, v in host[k - 1].items()}
            h["x0"][:, :12] += rng.normal(0.0, 2e-3, size=(Bpg, 12)).astype(np.float32)
            host[k] = h

    def bi(k):   # the batch of step k: cycled, or ping-pong along the drift sequence
        if not args.warm_fleet:
            return k % nbat
        j = k % (2 * nbat - 2)
        return j if j < nbat else 2 * nbat - 2 - j
    # the caller knows its contact schedules: promise the largest stance count so the
    # engine launches only the capacity classes the workload can reach
    max_stance = int(max((h["contact"] > 0).reshape(Bpg, -1).sum(1).max() for h in host))
    min_stance = int(min((h["contact"] > 0).reshape(Bpg, -1).sum(1).min() for h in host))
    eng = LinearMpc(horizon=N, robot=robots[0], device=dev, max_iter=args.max_iter,
                    max_stance=max_stance)
    # and the smallest: the first capacity class any robot needs takes the batch directly
    # (mpcqp_set_stance_range; an all-standing fleet goes straight to the interior-point class)
    eng.set_stance_range(min_stance, max_stance)
    eng.set_order(args.order)
    if args.cross_leg_r:   # the reference's diagonals scaled by a dense correlation matrix on R
        from mpcqp.params import Q_DIAG, R_DIAG
        A = np.random.default_rng(12).standard_normal((12, 12))
        Cr = A @ A.T / 12.0 + 0.5 * np.eye(12)
        dr = np.sqrt(np.diag(Cr))
        sq = np.sqrt(np.asarray(R_DIAG, np.float64))
        Rx = np.outer(sq, sq) * Cr / np.outer(dr, dr)
        eng.set_weights(np.diag(Q_DIAG), 0.5 * (Rx + Rx.T))
    if args.warm_fleet:
        eng.set_warm_start(Bpg)
    dev_b = []
    for h in host:
        dev_b.append({k: torch.as_tensor(v).to(dev).contiguous() for k, v in h.items()})
    u0 = torch.empty((Bpg, 12), dtype=torch.float32, device=dev)
    status = [torch.empty((Bpg,), dtype=torch.int32, device=dev) for _ in range(nbat)]
    iters = [torch.empty((Bpg,), dtype=torch.int32, device=dev) for _ in range(nbat)]
    stream = torch.cuda.current_stream(dev)
    gather_events = []

    def step(k, ev=None):
        d = dev_b[bi(k)]
        if ev is not None:
            ev[0].record(stream)
        eng.solve_raw(Bpg, d["x0"], d["xref"], d["contact"], d["feet"], d["robot"], u0,
                      None, status[bi(k)], iters[bi(k)], stream=stream)
        if ev is not None:
            ev[1].record(stream)
        if world > 1 and not args.no_gather:
            if ev is not None:   # the RCCL all-gather, timed on its own
                g = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                g[0].record(stream)
                gather_u0(u0)
                g[1].record(stream)
                gather_events.append(g)
            else:
                gather_u0(u0)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    t0 = time.perf_counter()
    # HIP events on the launch stream: one pair brackets the K back-to-back launches
    # (per-step markers were measured to slow each step by ~6 us); with a per-step
    # all-gather (N > 1) the solve is bracketed per step so the gather stays outside
    sparse = not args.step_events and (world == 1 or args.no_gather)
    if sparse:
        events[0][0].record(stream)
        for k in range(args.steps):
            step(k)
        events[0][1].record(stream)
    else:
        # per-step event pairs cost ~6 us a step: bracket a sample of the steps
        # (every --event-every-th; every step with --step-events)
        every = 1 if args.step_events else max(1, args.event_every)
        for k in range(args.steps):
            step(k, events[k] if k % every == 0 else None)
        events = [e for k, e in enumerate(events) if k % every == 0]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if sparse:   # per-launch duration incl. the dispatch gap: an upper bound
        kern_ms = [events[0][0].elapsed_time(events[0][1]) / args.steps]
    else:
        kern_ms = [a.elapsed_time(b) for a, b in events]
    tmax = torch.tensor([elapsed], dtype=torch.float64,
                        device=dev if world == 1 or dist.get_backend() == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    elapsed = float(tmax.item())

    # algorithmic work per launch: per-robot n_eff and executed iterations
    flops_launch = []
    exec_launch = []
    it_all = []
    n_ipm = 0
    for k in range(nbat):
        it = iters[k].cpu().numpy()
        ns = 3 * (host[k]["contact"] > 0).reshape(Bpg, -1).sum(1)
        # iters of an interior-point robot (n > 128) count Newton factorisations, not
        # active-set steps: such robots are priced at the formulation + one n^3/3
        # factorisation only (K = 0), a lower bound on their work
        ki = [0 if n > 128 else int(i) for n, i in zip(ns, it)]
        n_ipm += int((ns > 128).sum())
        flops_launch.append(sum(algorithmic_flops(N, int(n), k) for n, k in zip(ns, ki)))
        exec_launch.append(sum(executed_flops(N, int(n), k) for n, k in zip(ns, ki)))
        it_all.append(it)
    st = np.concatenate([x.cpu().numpy() for x in status])   # every batch's last solve
    steps_per_bat = [sum(1 for s in range(args.steps) if bi(s) == k) for k in range(nbat)]
    F_avg = sum(f * c for f, c in zip(flops_launch, steps_per_bat)) / args.steps
    E_avg = sum(f * c for f, c in zip(exec_launch, steps_per_bat)) / args.steps
    kavg_s = sum(kern_ms) / len(kern_ms) / 1e3
    achieved = F_avg / kavg_s / 1e12
    it_all = np.concatenate(it_all)

    qps = world * Bpg * args.steps / elapsed
    # HBM traffic cannot be counted inside this process (PMC needs a rocprofv3 pass of its
    # own): it is attached only from a profile of THIS build (library SHA-256 match) of
    # the same config and batch, with its provenance; otherwise null
    traffic, traffic_source, traffic_note = None, None, None
    try:
        from mpcqp import _lib as _mlib
        with open(args.pmc_file) as fh:
            pmc = json.load(fh)
        entry = pmc.get(args.config)
        sha = _mlib.lib_sha256()
        if not entry or entry.get("batch") != Bpg:
            traffic_note = f"no PMC profile of {args.config} at batch {Bpg} in {os.path.relpath(args.pmc_file, ROOT)}"
        elif entry.get("lib_sha256") != sha:
            traffic_note = (f"the PMC profile in {os.path.relpath(args.pmc_file, ROOT)} was taken on another build "
                            f"(lib {str(entry.get('lib_sha256'))[:12]} != {sha[:12]}): not attached")
        else:
            traffic = entry.get("hbm_bytes_per_launch")
            kern = entry.get("kernels", {}).get(entry.get("dominant_kernel"), {})
            traffic_source = {"file": os.path.relpath(args.pmc_file, ROOT), "profile_dir": entry.get("profile_dir"),
                              "lib_sha256": sha, "kernel": entry.get("dominant_kernel"),
                              "fetch_kib_raw": kern.get("fetch_kib_per_launch_raw"),
                              "write_kib": kern.get("write_kib_per_launch"),
                              "formula": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM; the x2 is the "
                                         "guide's 16-B/lane stream calibration, uncalibrated for this kernel's "
                                         "per-robot slices)",
                              "measured_by": "separate rocprofv3 --pmc passes (tools/profile.sh), not this run"}
    except Exception as exc:   # noqa: BLE001 -- provenance is best effort, never fatal
        traffic_note = f"traffic unavailable: {exc}"

    callers = None if args.no_callers else time_callers(eng, host[0], Bpg, N, dev, stream)
    # the default caller path (no stance promise: every capacity class launched, the idle
    # workgroups of the queued classes exit at once), timed the same way, outside `value`
    no_hint = None
    if not args.no_hint_line and not args.warm_fleet and world == 1:
        eng.set_stance_range(0, 0)
        for k in range(5):
            step(k)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        nh_steps = min(args.steps, 50)
        t1 = time.perf_counter()
        e0.record(stream)
        for k in range(nh_steps):
            step(k)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        nh_el = time.perf_counter() - t1
        no_hint = {"max_stance": 0, "steps": nh_steps, "value": Bpg * nh_steps / nh_el, "unit": "QP/s",
                   "ms_per_step": nh_el / nh_steps * 1e3, "kernel_ms_avg": e0.elapsed_time(e1) / nh_steps,
                   "vs_hinted": (Bpg * nh_steps / nh_el) / qps,
                   "note": "LinearMpc(max_stance=0): the caller promises nothing about its schedules"}
        eng.set_stance_range(min_stance, max_stance)
    # a serving-style workload: independent batches alternating two HIP streams, so one
    # launch's tail (its slowest robots, most CUs idle) overlaps the next launch's start.
    # Outside `value`, which keeps one batch at a time (a control loop's dependency).
    two_streams = None
    if not args.no_hint_line and not args.warm_fleet and world == 1:
        s2 = [stream, torch.cuda.Stream(dev)]
        u0s = [u0, torch.empty_like(u0)]
        sts = [torch.empty((Bpg,), dtype=torch.int32, device=dev) for _ in range(2)]
        its = [torch.empty((Bpg,), dtype=torch.int32, device=dev) for _ in range(2)]

        def step2(k):
            d = dev_b[k % nbat]
            eng.solve_raw(Bpg, d["x0"], d["xref"], d["contact"], d["feet"], d["robot"], u0s[k & 1], None,
                          sts[k & 1], its[k & 1], stream=s2[k & 1])
        for k in range(4):
            step2(k)
        torch.cuda.synchronize(dev)
        ts_steps = min(args.steps, 100)
        t1 = time.perf_counter()
        for k in range(ts_steps):
            step2(k)
        torch.cuda.synchronize(dev)
        ts_el = time.perf_counter() - t1
        two_streams = {"steps": ts_steps, "value": Bpg * ts_steps / ts_el, "unit": "QP/s",
                       "ms_per_step": ts_el / ts_steps * 1e3, "vs_value": (Bpg * ts_steps / ts_el) / qps,
                       "note": "independent batches of the same config alternating two HIP streams (a serving "
                               "workload: one launch's tail overlaps the next); `value` is one batch at a time"}
    gather_ms = (sum(a.elapsed_time(b) for a, b in gather_events) / len(gather_events)
                 if gather_events else None)

    gather_label = ""
    if world > 1 and not args.no_gather:
        be = dist.get_backend()
        gather_label = " + " + ("RCCL" if be == "nccl" else be) + " all-gather of u0"
    if rank == 0:
        cpu = None if args.no_cpu else cpu_baseline_line(host[0], N, args.cpu_seconds, world)
        line = {
            "metric": "QP solves/sec (whole node), horizon=10 GRF QP, at 1/2/4/8 MI355X",
            "value": qps,
            "unit": "QP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded SURVEY §8(d) states, gait tables, feet; seed = base + rank)",
            "config": {"workload": f"{args.config}: batch {Bpg}/GPU, horizon {N}, gaits {'+'.join(gaits)}, "
                                   f"robots {'+'.join(robots)}" + (f", cone tilt <= {tilt} deg" if tilt else ""),
                       "batch_per_gpu": Bpg, "horizon": N, "global_batch": world * Bpg,
                       "parallelism": f"robot-sharded x{world}" + gather_label},
            # the governing pipe is the FP64 vector ALU (VALU): no MFMA instruction is on
            # the path (gfx950's FP64 MFMA peak equals its FP64 VALU peak)
            "roofline": {"bound": "valu", "pipe": "fp64 VALU", "achieved": achieved, "peak": PEAK_FP64_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic,
                         "traffic_source": traffic_source,
                         "executed_frac": E_avg / kavg_s / 1e12 / PEAK_FP64_TFLOPS},
            "cpu_baseline": cpu,
            "kernel_ms_avg": kavg_s * 1e3,
            "executed_tflops": E_avg / kavg_s / 1e12,
            "iters_mean": float(it_all.mean()),
            "iters_max": int(it_all.max()),
            "status_ok_frac": float((st == 0).mean()),
            "stance_range": [min_stance, max_stance],
            "dispatch_order": "predicted cost, largest first" if args.order else "batch order",
            "callers": callers,
        }
        if traffic_note:
            line["roofline"]["traffic_note"] = traffic_note
        if n_ipm:
            # robots of the interior-point class would be priced at the reference's dense
            # formulation + one n^3/3 factorisation, work that class never executes (it solves
            # the uncondensed horizon by Riccati recursions): no roofline fraction for such a
            # line, the rate goes to a field of its own
            rf = line["roofline"]
            line["reference_work_rate"] = {
                "achieved": rf["achieved"], "unit": "TFLOP/s", "vs_fp64_peak": rf["frac"],
                "note": (f"{n_ipm} of {nbat * Bpg} robots have n > 128 (the interior-point class); the whole "
                         "batch is priced at the reference's condensed-dense work (SURVEY §8(d)), which that "
                         "class does not execute: a reference-work rate, not hardware utilisation")}
            rf["achieved"] = rf["frac"] = rf["executed_frac"] = None
            rf["note"] = "frac null: the line's interior-point robots execute none of the priced work (reference_work_rate)"
        if no_hint is not None:
            line["no_hint"] = no_hint
        if two_streams is not None:
            line["two_streams"] = two_streams
        if gather_ms is not None:
            line["gather_ms_avg"] = gather_ms
        if args.standing_every:
            line["config"]["workload"] += f", every {args.standing_every}th robot standing"
        if args.cross_leg_r:
            line["config"]["workload"] += ", R coupling every pair of legs (the interior-point class's 12 x 12 stage weights)"
        if args.warm_fleet:
            line["config"]["workload"] += (", warm fleet: consecutive ticks of one fleet (x0 drifting "
                                           "N(0, 2e-3) per tick), each robot's active set remembered")
            line["data"] += "; warm start (mpcqp_set_warm_start): not comparable with the cold lines"
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
