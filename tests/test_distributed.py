"""N>1 path of bench.py on CPU: world_size-2 gloo over 127.0.0.1.

The path shards (independent QP instances): every rank draws its own shard of the
config-5 batch, solves it with no data-path collective, and the only exchange is the
MAX over ranks of the wall time.  Here the solve is the oracle (test infrastructure);
on the GPU box the same code path runs the HIP kernel."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, TERMINAL_SETS


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    import time
    import torch
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle import assembly as oa
    from oracle.cpu import CpuProblem
    goals = [oa.ENVIRONMENTS[n][2] for n in bench.ENVS]
    X, env, offsets = bench.sample_shard(rank, 240, goals)
    t0 = time.perf_counter()
    stats = []
    for j, name in enumerate(bench.ENVS):
        cp = CpuProblem(oa.build(name, 20, terminal_set_dir=TERMINAL_SETS))
        _, st, _ = cp.solve(X[offsets[j]:offsets[j + 1]], threads=1)
        stats.append(np.bincount(st, minlength=4))
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    tot = torch.tensor(np.sum(stats, axis=0), dtype=torch.int64)
    dist.all_reduce(tot)
    q.put((rank, X[:3].copy(), env.tolist(), offsets.tolist(), float(t.item()), tot.tolist()))
    dist.destroy_process_group()


def test_two_rank_sharding_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, x0, e0, o0, t0, s0), (r1, x1, e1, o1, t1, s1) = res
    assert not np.allclose(x0, x1)                      # independent shards
    assert e0 == sorted(e0) and e1 == sorted(e1)        # grouped by environment
    assert o0[-1] == 240 and o1[-1] == 240
    assert t0 == t1                                     # max-over-ranks timing agrees
    assert s0 == s1 and sum(s0) == 480 and s0[2] == 0   # every instance certified
