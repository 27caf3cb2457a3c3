#!/usr/bin/env python3
"""Benchmark: batched MPC QP solves/s on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[4], weak-scaled): every rank solves a shard of 131,072
mixed Road*/Env instances (RoadEnv / RoadOneCarEnv / RoadMultipleCarsEnv, N = 20, n = 40, fp64),
grouped by environment; at 8 GPUs that is the 1,048,576-instance configuration.  One timed step =
one pass of the hot path over the shard (inputs resident in HBM).  The shard split needs no
collective; the only communication is the barrier and the max-over-ranks of the wall time, both
over gloo on host memory.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config5|config4|config3|config2]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

``--backend cpu`` runs the same control flow on the library's CPU QP path (hosts without a GPU;
the distributed flow is tested this way under gloo).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

ENVS = ("RoadEnv", "RoadOneCarEnv", "RoadMultipleCarsEnv")
PER_GPU = 131072
FP64_PEAK_TFLOPS = 78.6      # MI355X FP64, vector FMA rate == matrix (MFMA) rate, vendor figure
HBM_PEAK_GBS = 8000.0
METRIC = "QP solves/sec (batched MPC steps), N=20 n=4 m=2, at 1/2/4/8 MI355X"

# workload -> (environments, horizon, default per-GPU batch, controller, description)
WORKLOADS = {
    "config5": (ENVS, 20, PER_GPU, "statefb", "config5_mixed_road_envs_N20_weak"),
    "config4": (("RoadMultipleCarsEnv",), 20, 65536, "outputfb", "config4_RoadMultipleCarsEnv_outputfb_N20"),
    "config3": (("RoadOneCarEnv",), 20, 65536, "statefb", "config3_RoadOneCarEnv_statefb_N20"),
    "config2": (("RoadEnv",), 10, 4096, "statefb", "config2_RoadEnv_statefb_N10"),
}
KNAME = {1: "ipm_dense", 2: "ipm_staged", 3: "ipm_dense_4wave", 7: "ipm_riccati"}
KDESC = {1: "ipm_dense (wavefront per QP, G/H in LDS, dense normal matrix)",
         2: "ipm_staged (wavefront per QP, stage-structured G/H products and Riccati-style M build)",
         3: "ipm_dense, 4 waves per workgroup",
         7: "ipm_riccati (16 lanes per QP, 4 QPs per wavefront, row state in registers, stage-form Riccati "
            "factorization and solves on v_mfma_f64_4x4x4 with one matrix entry per lane, per-group instance "
            "refill; all environments per launch; large batches as three launches: iterations with hand-off, "
            "lock-step polish with one correction round, single-kernel solve of the rejected rest)"}


def sample_shard(rank: int, B: int, goals, seed: int = 5):
    """Config-5 inputs: env_id ~ U{0..len(goals)-1}, x in [g_x - 25, g_x], y in [-3, 3],
    psi in [-pi/8, pi/8], v in [-1, 5]; grouped by environment (sorted).  One environment: the same
    state distribution around its goal."""
    rng = np.random.default_rng(seed * 1000 + rank)
    env = np.sort(rng.integers(0, len(goals), B))
    gx = np.array([g[0] for g in goals])[env]
    X = np.stack([gx - 25 * rng.random(B), rng.uniform(-3, 3, B), rng.uniform(-np.pi / 8, np.pi / 8, B),
                  rng.uniform(-1, 5, B)], axis=1)
    offsets = np.searchsorted(env, np.arange(len(goals) + 1))
    return X, env, offsets


def sample_outputfb(rank: int, B: int, goal):
    """Config-4 inputs: x_true as the config-5 states, x_hat_prev = x_true + N(0, 0.05^2) per
    component, u_prev = 0, y0 = C x_true (C picks x, y, v: mpc.py:387-389)."""
    rng = np.random.default_rng(4 * 1000 + rank)
    gx = goal[0]
    xt = np.stack([gx - 25 * rng.random(B), rng.uniform(-3, 3, B), rng.uniform(-np.pi / 8, np.pi / 8, B),
                   rng.uniform(-1, 5, B)], axis=1)
    xhat = xt + rng.normal(0.0, 0.05, (B, 4))
    return xt, xhat, np.zeros((B, 2)), xt[:, [0, 1, 3]].copy()


def build_controllers(envs, N, device):
    import contextlib
    from carmpc_amd.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE
    from carmpc_amd.environments import ENVIRONMENTS
    from carmpc_amd.mpc import MPCOutputFB, MPCStateFB
    ctrls = []
    with contextlib.redirect_stdout(sys.stderr):          # keep stdout to the one JSON line
        for name in envs:
            kw = dict(env=ENVIRONMENTS[name](), terminal_set_dir=os.path.join(REPO, "terminal_sets"), device=device)
            c = MPCStateFB(DT_CONTROL, N, LINEARIZE_STATE, LINEARIZE_INPUT, **kw)
            c.qp  # assemble now
            ctrls.append(c)
    return ctrls


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def oracle_sample(envs, N, X, offsets, sample: int, threads: int, xref=None):
    """The oracle's C restatement of the dense IPM (oracle/ipm.c) on a bounded, equal-per-environment
    sample of this shard: the CPU baseline and I_ref (the oracle's iteration counts, so the
    canonical flop count does not depend on the kernel being measured)."""
    from oracle import assembly as oa
    from oracle.cpu import CpuProblem
    per = max(1, sample // len(envs))
    res = {"threads": threads, "n": 0, "t_all": 0.0, "n1": 0, "t_one": 0.0, "iters": {}}
    for j, name in enumerate(envs):
        sel = np.arange(offsets[j], min(offsets[j + 1], offsets[j] + per))
        if len(sel) == 0:
            res["iters"][name] = 0.0
            continue
        cp = CpuProblem(oa.build(name, N, terminal_set_dir=os.path.join(REPO, "terminal_sets")))
        xr = None if xref is None else np.ascontiguousarray(np.broadcast_to(xref, (len(sel), 4)))
        cp.solve(X[sel[:64]], xr[:64] if xr is not None else None, threads=threads)      # warm
        t0 = time.perf_counter()
        _, st, it = cp.solve(X[sel], xr, threads=threads)
        res["t_all"] += time.perf_counter() - t0
        res["n"] += len(sel)
        res["iters"][name] = float(it.mean())
        one = sel[:max(64, len(sel) // 8)]
        t0 = time.perf_counter()
        cp.solve(X[one], xr[:len(one)] if xr is not None else None, threads=1)
        res["t_one"] += time.perf_counter() - t0
        res["n1"] += len(one)
    return res


def product_cpu_sample(ctrls, X, offsets, sample: int, threads: int, xref=None):
    """The library's own CPU QP path (carmpc_cpu_solve_batch, the stage-form IPM) on the same sample."""
    from carmpc_amd.qp import CpuQPProblem
    per = max(1, sample // len(ctrls))
    n, t_all = 0, 0.0
    for j, c in enumerate(ctrls):
        sel = np.arange(offsets[j], min(offsets[j + 1], offsets[j] + per))
        if len(sel) == 0:
            continue
        rows, rhs = c._stage_rows()
        qp = CpuQPProblem(N=c.N, A=c.A, B=c.B, Q=c.Q, R=c.R, P=c.P, goal=c.goal, state_A=rows, state_b=rhs,
                          term_A=c.term_set_A[:, -4:], term_b=c.term_set_b, u_lower=c.input_lower,
                          u_upper=c.input_upper)
        qp.solve(X[sel[:64]], xref, threads=threads)
        t0 = time.perf_counter()
        qp.solve(X[sel], xref, threads=threads)
        t_all += time.perf_counter() - t0
        n += len(sel)
    return n / t_all if t_all > 0 else 0.0


class GpuBackend:
    """The device path: torch tensors as buffers, the C ABI for every kernel launch."""
    name = "gpu"

    def __init__(self, args, local_rank):
        import torch
        self.torch = torch
        ndev = torch.cuda.device_count()
        self.gpus_visible = ndev
        if local_rank >= ndev > 0:      # more ranks than GPUs: only as an explicit rehearsal of the N>1 flow
            if not args.share_gpus:
                raise SystemExit(f"bench: local rank {local_rank} has no GPU of its own ({ndev} visible); a run whose "
                                 "ranks share GPUs measures no scaling (--share-gpus runs it as a rehearsal and "
                                 "marks the line)")
            print(f"bench: local rank {local_rank} shares GPU {local_rank % ndev} ({ndev} visible): "
                  "throughput of this run is not a scaling number", file=sys.stderr)
            local_rank %= ndev
        self.device = torch.device("cuda", local_rank)
        torch.cuda.set_device(self.device)
        self.stream = torch.cuda.current_stream()
        self.args = args

    def setup(self, ctrls, kind, X, offsets, extra):
        torch = self.torch
        from carmpc_amd.qp import SolverSettings
        self.settings = SolverSettings(kernel=self.args.kernel)
        self.probs = [c.qp for c in ctrls]
        self.offsets = offsets
        self.kind = kind
        B = X.shape[0]
        self.Xd = torch.as_tensor(X).to(self.device)
        self.u = torch.zeros((B, self.probs[0].n), dtype=torch.float64, device=self.device)
        self.st = torch.empty(B, dtype=torch.int32, device=self.device)
        self.it = torch.empty(B, dtype=torch.int32, device=self.device)
        if kind == "outputfb":
            xhat0, uprev, y, xref = extra
            self.xhat0 = torch.as_tensor(xhat0).to(self.device)
            self.xhat = torch.empty_like(self.xhat0)
            self.uprev = torch.as_tensor(uprev).to(self.device)
            self.y = torch.as_tensor(y).to(self.device)
            self.xref = torch.as_tensor(np.ascontiguousarray(np.broadcast_to(xref, (B, 4)))).to(self.device)
            from carmpc_amd.mpc import MPCOutputFB
            self.C, self.L = MPCOutputFB.C_OUT, MPCOutputFB.L_GAIN
        torch.cuda.synchronize()
        return [self.settings.kernel or p.kernel for p in self.probs]

    def step(self):
        from carmpc_amd.qp import solve_segments
        if self.kind == "outputfb":
            # MPCOutputFB.step (mpc.py:450-478): observer on the previous estimate, then the QP at it
            self.xhat.copy_(self.xhat0)
            self.probs[0].observe(self.y, self.xhat, self.uprev, self.C, self.L, stream=self.stream)
            self.probs[0].solve(self.xhat, self.xref, settings=self.settings, out=(self.u, self.st, self.it),
                                stream=self.stream)
        elif self.args.per_problem_launches or len(self.probs) == 1:
            for j, p in enumerate(self.probs):
                sl = slice(int(self.offsets[j]), int(self.offsets[j + 1]))
                p.solve(self.Xd[sl], settings=self.settings, out=(self.u[sl], self.st[sl], self.it[sl]), stream=self.stream)
        else:
            solve_segments(self.probs, self.offsets, self.Xd, settings=self.settings, stream=self.stream,
                           out=(self.u, self.st, self.it))

    def sync(self):
        self.torch.cuda.synchronize()

    def timed_steps(self, steps):
        """K steps with HIP events on the launch stream around each step's device work."""
        torch = self.torch
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for a, b in evs:
            a.record(self.stream)
            self.step()
            b.record(self.stream)
        return evs

    def device_ms(self, evs):
        return float(np.mean([a.elapsed_time(b) for a, b in evs]))

    def results(self):
        return self.st.cpu().numpy(), self.it.cpu().numpy()

    def e2e_qps(self, X):
        """PCIe-inclusive rates (carmpc_amd.qp.HostPipeline: x0 from pinned host memory, u / status / iterations
        back to it, copies on their own streams): a sequence of batches with three in flight (steady-state rate),
        one batch at a time (latency-bound), and the three steps one after another on ONE stream."""
        torch = self.torch
        if self.kind == "outputfb":
            return None
        from carmpc_amd.qp import HostPipeline
        hp = HostPipeline(self.probs, self.offsets, settings=self.settings, depth=3)
        Xt = torch.as_tensor(X)
        for k in range(3):
            hp.staging(k).copy_(Xt)
        hp.wait(hp.submit())
        torch.cuda.synchronize()
        nb = 9
        t0 = time.perf_counter()
        tickets = [hp.submit(), hp.submit(), hp.submit()]
        for _ in range(nb - 3):
            hp.wait(tickets.pop(0))
            tickets.append(hp.submit())
        while tickets:
            last = hp.wait(tickets.pop(0))
        stream_rate = nb * X.shape[0] / (time.perf_counter() - t0)
        self.e2e_check = (last[1].numpy().copy(), last[2].numpy().copy())
        t0 = time.perf_counter()
        for _ in range(3):
            hp.wait(hp.submit())
        self.e2e_single = 3 * X.shape[0] / (time.perf_counter() - t0)
        Xh, uh, sh = hp.staging(0), hp.sets[0]["uh"], hp.sets[0]["sth"]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            self.Xd.copy_(Xh, non_blocking=True)
            self.step()
            uh.copy_(self.u, non_blocking=True)
            sh.copy_(self.st, non_blocking=True)
        torch.cuda.synchronize()
        self.e2e_serial = 3 * X.shape[0] / (time.perf_counter() - t0)
        # the first input of every sequence back to the host (what the reference's step() returns), one batch at a time
        hp1 = HostPipeline(self.probs, self.offsets, settings=self.settings, depth=1, first_action=True)
        hp1.staging(0).copy_(Xt)
        u_first = hp1.wait(hp1.submit())[0]
        self.e2e_first_ok = bool(np.array_equal(u_first.numpy(), self.u[:, :u_first.shape[1]].cpu().numpy()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(6):
            hp1.wait(hp1.submit())
        self.e2e_first = 6 * X.shape[0] / (time.perf_counter() - t0)
        return stream_rate


class CpuBackend:
    """The library's CPU QP path (carmpc_cpu_solve_batch) under the same control flow."""
    name = "cpu"

    gpus_visible = None

    def __init__(self, args, local_rank):
        self.args = args
        self.device = "cpu"

    def setup(self, ctrls, kind, X, offsets, extra):
        from carmpc_amd.qp import SolverSettings
        self.settings = SolverSettings()
        self.probs = [c.qp for c in ctrls]
        self.ctrls, self.kind, self.X, self.offsets, self.extra = ctrls, kind, X, offsets, extra
        B = X.shape[0]
        self.u = np.zeros((B, self.probs[0].n))
        self.st = np.zeros(B, np.int32)
        self.it = np.zeros(B, np.int32)
        return [0 for _ in self.probs]

    def step(self):
        thr = self.args.cpu_threads
        if self.kind == "outputfb":
            xhat0, uprev, y, xref = self.extra
            c = self.ctrls[0]
            from carmpc_amd.mpc import MPCOutputFB
            C, L = MPCOutputFB.C_OUT, MPCOutputFB.L_GAIN
            xhat = xhat0 @ c.A.T + uprev @ c.B.T + (y - xhat0 @ C.T) @ L.T          # mpc.py:448, batched
            self.u, self.st, self.it = self.probs[0].solve(xhat, xref.reshape(1, 4), self.settings, threads=thr)
            return
        for j, p in enumerate(self.probs):
            sl = slice(int(self.offsets[j]), int(self.offsets[j + 1]))
            self.u[sl], self.st[sl], self.it[sl] = p.solve(self.X[sl], settings=self.settings, threads=thr)

    def sync(self):
        pass

    def timed_steps(self, steps):
        out = []
        for _ in range(steps):
            t0 = time.perf_counter()
            self.step()
            out.append(time.perf_counter() - t0)
        return out

    def device_ms(self, evs):
        return float(np.mean(evs)) * 1e3

    def results(self):
        return self.st, self.it

    def e2e_qps(self, X):
        return None


def run(args, backend_cls=None) -> dict | None:
    """The benchmark's control flow; returns the result line on rank 0 (None elsewhere).
    ``backend_cls`` is injectable so the distributed flow can run anywhere."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        # one rank per GPU: a line that says n_gpus = N must come from N ranks
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE is {world}: launch one rank per GPU "
                         f"(python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}), "
                         "or run bench.py --gpus N without a launcher and it starts the ranks itself")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        # one process per GPU; ranks never exchange problem data.  The barrier and the max of the
        # wall times go over gloo on host tensors.
        import torch.distributed as dist
        dist.init_process_group("gloo")
    if backend_cls is None:
        backend_cls = CpuBackend if args.backend == "cpu" else GpuBackend
    be = backend_cls(args, local)

    envs, N, default_B, kind, wname = WORKLOADS[args.workload]
    B = args.per_gpu or default_B
    ctrls = build_controllers(envs, N, be.device)
    goals = [c.goal for c in ctrls]
    extra = xref = None
    if kind == "outputfb":
        xt, xhat0, uprev, y = sample_outputfb(rank, B, goals[0])
        from carmpc_amd.mpc import MPCOutputFB
        xref = goals[0]           # optimal target selection: the unique steady state is the goal (mpc.py:413-437)
        extra = (xhat0, uprev, y, xref)
        # the QP is solved at the observer's estimate: the oracle sample uses the same states
        X = xhat0 @ ctrls[0].A.T + uprev @ ctrls[0].B.T + (y - xhat0 @ MPCOutputFB.C_OUT.T) @ MPCOutputFB.L_GAIN.T
        offsets = np.array([0, B])
    else:
        X, _env, offsets = sample_shard(rank, B, goals, seed={"config5": 5, "config3": 3, "config2": 2}[args.workload])
    kernels = be.setup(ctrls, kind, X, offsets, extra)

    for _ in range(args.warmup):
        be.step()
    be.sync()
    if dist is not None:
        dist.barrier()
    be.sync()
    t0 = time.perf_counter()
    evs = be.timed_steps(args.steps)
    be.sync()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    wall_max = wall
    if dist is not None:
        import torch
        t = torch.tensor([wall], dtype=torch.float64)          # host tensor: gloo
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall_max = float(t.item())
    kern_ms = be.device_ms(evs)
    e2e = None if args.no_e2e else be.e2e_qps(X)
    st_np, it_np = be.results()
    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return None

    value = B * world * args.steps / wall_max
    probs = be.probs
    used = sorted(set(kernels))
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "QP/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall_max / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded state distribution of the configuration)",
        "config": {"workload": wname, "per_gpu_batch": B, "global_batch": B * world, "envs": list(envs), "N": N,
                   "n": 2 * N, "p_qp_rows": [p.p for p in probs],
                   "kernel": ("carmpc_cpu_solve_batch (host stage-form IPM)" if be.name == "cpu"
                              else "; ".join(KDESC.get(k, str(k)) for k in used)),
                   "step": ("observer kernel + QP solve (MPCOutputFB.step)" if kind == "outputfb" else "QP solve"),
                   "backend": be.name, "parallelism": f"shard{world} (no data-path collective)"},
        "status_split": {s: int((st_np == k).sum()) for k, s in enumerate(("optimal", "primal_infeasible", "max_iter",
                                                                         "numerical"))},
        "iters_mean_optimal": float(it_np[st_np == 0].mean()) if (st_np == 0).any() else 0.0,
    }
    if e2e is not None:
        out["e2e_qps_pcie_inclusive"] = round(e2e * world, 1)
        out["e2e_is"] = ("a sequence of batches, x0 from pinned host memory, u / status / iterations back to it, three "
                         "batches in flight so that one batch's copies run under another's solve "
                         "(carmpc_amd.qp.HostPipeline); never `value`")
        if getattr(be, "e2e_single", None):
            out["e2e_qps_pcie_one_batch_at_a_time"] = round(be.e2e_single * world, 1)
        if getattr(be, "e2e_serial", None):
            out["e2e_qps_pcie_serial_one_stream"] = round(be.e2e_serial * world, 1)
        if getattr(be, "e2e_first", None):
            out["e2e_qps_pcie_first_action_only"] = round(be.e2e_first * world, 1)
            out["e2e_first_action_equals_resident"] = be.e2e_first_ok
        chk = getattr(be, "e2e_check", None)
        if chk is not None:       # the chunked path returns the same statuses and iteration counts
            out["e2e_equals_resident"] = bool(np.array_equal(chk[0], st_np) and np.array_equal(chk[1], it_np))
    gpus_visible = getattr(be, "gpus_visible", None)
    if gpus_visible is not None:
        out["gpus_visible"] = gpus_visible
        out["ranks_share_gpu"] = world > gpus_visible
        if out["ranks_share_gpu"]:
            out["note"] = "REHEARSAL: ranks shared GPUs (--share-gpus); value is not a scaling measurement"
    assert out["n_gpus"] == args.gpus

    # CPU baseline and I_ref: the oracle on a bounded sample of rank 0's shard
    seg = np.diff(offsets)
    if not args.no_cpu:
        thr = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        osr = oracle_sample(envs, N, X, offsets, args.cpu_sample, thr, xref)
        I_ref = osr["iters"]
        prod = product_cpu_sample(ctrls, X, offsets, args.cpu_sample, thr, None if xref is None else np.asarray(xref).reshape(1, 4))
        out["cpu_baseline"] = {
            "value": round(osr["n"] / osr["t_all"], 1), "unit": "QP/s", "cores": thr, "kind": "port",
            "sample": f"{osr['n']} instances of rank 0's shard (equal per environment), oracle/ipm.c (dense Mehrotra "
                      f"IPM, the algorithm of the canonical flop count), OpenMP x{thr}",
            "cpu_model": cpu_model(),
            "single_thread": {"value": round(osr["n1"] / osr["t_one"], 1), "cores": 1, "sample": f"{osr['n1']} instances"},
            "product_cpu_path": {"value": round(prod, 1), "cores": thr,
                                 "what": "carmpc_cpu_solve_batch (the library's stage-form IPM on the host), same sample"},
        }
        iref_src = "oracle/ipm.c on the cpu_baseline sample (rank 0)"
    else:
        I_ref = {envs[j]: float(it_np[offsets[j]:offsets[j + 1]].mean()) if seg[j] else 0.0 for j in range(len(envs))}
        iref_src = "--no-cpu: this run's own iteration counts (not a valid roofline numerator)"
    if be.name == "gpu":
        canon = [seg[j] * I_ref[envs[j]] * probs[j].canonical_flops_per_iter() for j in range(len(envs))]
        execd = [float(it_np[offsets[j]:offsets[j + 1]].sum()) * probs[j].executed_flops_per_iter(kernels[j])
                 for j in range(len(envs))]
        flops_step = float(sum(canon))
        achieved = flops_step / (kern_ms * 1e-3) / 1e12
        exec_tf = sum(execd) / (kern_ms * 1e-3) / 1e12
        issued_tf = sum(float(it_np[offsets[j]:offsets[j + 1]].sum()) * probs[j].issued_flops_per_iter(kernels[j])
                        for j in range(len(envs))) / (kern_ms * 1e-3) / 1e12
        per_qp = 32 + 4 + 8 * 2 * N + 4 + 4 + (24 + 32 + 16 + 32 if kind == "outputfb" else 0)
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as f:
                    ent = json.load(f).get(args.workload + ":" + "+".join(KNAME.get(k, str(k)) for k in used))
                if ent is not None and ent.get("per_gpu_batch") == B:
                    traffic = ent.get("hbm_bytes_per_step")
            except Exception:
                traffic = None
        out["roofline"] = {
            "bound": "mfma",
            "compute": "FP64: v_mfma_f64_4x4x4 (stage recursions) and vector FMA (row phases); both pipes peak at "
                       "78.6 TFLOP/s.  The measured limiter is instruction issue at two wavefronts per SIMD (about one "
                       "instruction per 4 cycles and SIMD), not either pipe's arithmetic rate",
            "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / FP64_PEAK_TFLOPS, 5),
            "frac_is": "canonical dense-IPM flops (p n^2 + n^3/3 + 6 n^2 + 12 p n per iteration) x the oracle's "
                       "iteration counts / kernel time / peak: a normalised rate, NOT hardware utilisation",
            "executed_frac": round(exec_tf / FP64_PEAK_TFLOPS, 5),
            "executed_TFLOPs": round(exec_tf, 4),
            "executed_is": "flops the stage-form kernel performs for each QP (every recursion counted once) x its own "
                           "iteration counts / kernel time / peak: the useful FP64 utilisation",
            "issued_frac": round(issued_tf / FP64_PEAK_TFLOPS, 5),
            "issued_is": "as executed_frac, with every matrix-core instruction counted as a full 4x4x4 product "
                         "(part of the operands are structural zeros or replicated columns): FP64 pipe occupancy",
            "traffic": traffic,
            "traffic_is": "HBM bytes per step from the FETCH_SIZE / WRITE_SIZE counters of the committed profile "
                          "(profiles/traffic.json); about 0.79 GB of it are the iterates the iteration launch saves "
                          "with every hand-off (written once; read back for the few per cent whose polish is rejected)",
            "algorithmic_bytes_per_step": B * per_qp,
            "algorithmic_hbm_GBps": round(B * per_qp / (kern_ms * 1e-3) / 1e9, 3),
            "hbm_frac": round(B * per_qp / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
            "kernel_ms_per_step": round(kern_ms, 4), "canonical_flops_per_step": flops_step,
            "executed_flops_per_step": float(sum(execd)),
            "timing": "HIP events on the launch stream around each step's device work, mean over the timed steps",
            "I_ref": I_ref, "I_ref_source": iref_src,
            "launches": [{"env": envs[j], "kernel": KNAME.get(kernels[j], str(kernels[j])), "instances": int(seg[j]),
                          "canonical_flops": canon[j]} for j in range(len(envs))],
        }
    else:
        out["roofline"] = None
        out["cpu_step_ms"] = round(kern_ms, 3)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="config5", choices=sorted(WORKLOADS))
    ap.add_argument("--per-gpu", type=int, default=0, help="instances per rank (default: the configuration's batch)")
    ap.add_argument("--backend", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--cpu-threads", type=int, default=0, help="--backend cpu: threads per rank (0 = all)")
    ap.add_argument("--cpu-sample", type=int, default=131072,
                    help="instances of rank 0's shard timed on the host (all cores; an eighth of them on one thread)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive runs (profiles of the timed steps alone)")
    ap.add_argument("--per-problem-launches", action="store_true",
                    help="one carmpc_solve_batch launch per environment instead of one carmpc_solve_segments call")
    ap.add_argument("--kernel", type=int, default=0, help="carmpc_settings.kernel (0 auto, 1 dense, 2 staged, 7 riccati)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--share-gpus", action="store_true",
                    help="allow more ranks than visible GPUs (rehearsal of the N>1 flow; the line is marked)")
    return ap.parse_args(argv)


def spawn_ranks(args, argv) -> int:
    """``bench.py --gpus N`` from a plain shell (no launcher, WORLD_SIZE unset): start N ranks of this
    script as fresh child processes, one per GPU, before this process has touched the GPU, and
    relay rank 0's line.  Returns the exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    line, _ = procs[0].communicate()
    codes = [p.wait() for p in procs]
    if any(codes):
        print(f"bench: rank exit codes {codes}", file=sys.stderr)
        return next(c for c in codes if c) or 1
    for ln in line.splitlines():      # (gloo prints its own connection notes on stdout: keep stdout to the result)
        print(ln, file=sys.stdout if ln.startswith("{") else sys.stderr, flush=True)
    return 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be at least 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, argv))
    out = run(args)
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
