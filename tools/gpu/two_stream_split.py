"""One call on the whole bench shard against two calls on its halves issued on two streams at once (each half holds
half of every environment's instances): do the launch tails of one half hide under the other half's work?"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import bench  # noqa: E402
from carmpc_amd.qp import solve_segments  # noqa: E402

ctrls = bench.build_controllers(bench.ENVS, 20, torch.device("cuda", 0))
probs = [c.qp for c in ctrls]
X, env, offsets = bench.sample_shard(0, bench.PER_GPU, [c.goal for c in ctrls])
B = X.shape[0]
# halves: even and odd rows of every segment
halves = []
for h in (0, 1):
    rows = np.concatenate([np.arange(offsets[j] + h, offsets[j + 1], 2) for j in range(3)])
    offs = np.concatenate([[0], np.cumsum([len(np.arange(offsets[j] + h, offsets[j + 1], 2)) for j in range(3)])])
    halves.append((torch.as_tensor(X[rows]).cuda(), offs))
Xd = torch.as_tensor(X).cuda()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
outs = [tuple(torch.empty(s, dtype=d, device="cuda") for s, d in (((len(h[0]), 40), torch.float64), ((len(h[0]),), torch.int32), ((len(h[0]),), torch.int32))) for h in halves]
out = (torch.empty((B, 40), dtype=torch.float64, device="cuda"), torch.empty(B, dtype=torch.int32, device="cuda"), torch.empty(B, dtype=torch.int32, device="cuda"))


def one():
    solve_segments(probs, offsets, Xd, out=out)


def two():
    for (Xh, offs), o, s in zip(halves, outs, (s1, s2)):
        solve_segments(probs, offs, Xh, out=o, stream=s)


for name, fn in (("one call", one), ("two streams", two), ("one call", one), ("two streams", two)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20
    print(name, round(dt * 1e3, 3), "ms", round(B / dt / 1e6, 2), "M QP/s", flush=True)
