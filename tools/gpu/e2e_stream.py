#!/usr/bin/env python3
"""PCIe-inclusive rates of carmpc_amd.qp.HostPipeline on the bench shard: one batch at a time vs two batches in flight."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from carmpc_amd.qp import HostPipeline  # noqa: E402

ctrls = bench.build_controllers(bench.ENVS, 20, torch.device("cuda", 0))
probs = [c.qp for c in ctrls]
X, env, offsets = bench.sample_shard(0, bench.PER_GPU, [c.goal for c in ctrls])
B = X.shape[0]
for depth in (1, 2, 3):
    hp = HostPipeline(probs, offsets, depth=depth)
    for k in range(depth):
        hp.staging(k).copy_(torch.as_tensor(X))
    hp.wait(hp.submit())
    torch.cuda.synchronize()
    nb = 12
    t0 = time.perf_counter()
    tickets = [hp.submit() for _ in range(depth)]
    for _ in range(nb - depth):
        hp.wait(tickets.pop(0))
        tickets.append(hp.submit())
    while tickets:
        hp.wait(tickets.pop(0))
    dt = (time.perf_counter() - t0) / nb
    print("SDMA", os.environ.get("HSA_ENABLE_SDMA"), "depth", depth, round(dt * 1e3, 3), "ms/batch", round(B / dt / 1e6, 2), "M QP/s", flush=True)
