"""Sequential vs concurrent (one stream per environment segment) solve launches of the bench
workload: wall ms per step for both (tail overlap experiment)."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from carmpc_amd.qp import SolverSettings  # noqa: E402

dev = torch.device("cuda", 0)
ctrls = bench.build_problems(dev)
probs = [c.qp for c in ctrls]
X, env, offsets = bench.sample_shard(0, 131072, [c.goal for c in ctrls])
Xd = torch.as_tensor(X).to(dev)
B = len(X)
u = torch.zeros((B, 40), dtype=torch.float64, device=dev)
st = torch.empty(B, dtype=torch.int32, device=dev)
it = torch.empty(B, dtype=torch.int32, device=dev)
segs = [(probs[j], slice(int(offsets[j]), int(offsets[j + 1]))) for j in range(3)]
settings = SolverSettings()
main = torch.cuda.current_stream()
aux = [torch.cuda.Stream(device=dev) for _ in range(3)]


def seq():
    for p, sl in segs:
        p.solve(Xd[sl], settings=settings, out=(u[sl], st[sl], it[sl]), stream=main)


def conc():
    ev = torch.cuda.Event()
    ev.record(main)
    for (p, sl), s in zip(segs, aux):
        s.wait_event(ev)
        p.solve(Xd[sl], settings=settings, out=(u[sl], st[sl], it[sl]), stream=s)
    for s in aux:
        e = torch.cuda.Event()
        e.record(s)
        main.wait_event(e)


for name, fn in (("seq", seq), ("conc", conc), ("seq", seq), ("conc", conc)):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    print(name, "ms/step %.3f" % ((time.perf_counter() - t0) / 10 * 1e3), flush=True)
