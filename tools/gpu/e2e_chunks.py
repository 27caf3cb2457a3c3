#!/usr/bin/env python3
"""PCIe-inclusive rate of the host pipeline (carmpc_amd.qp.HostPipeline) on the bench shard for several chunk splits."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from carmpc_amd.qp import HostPipeline  # noqa: E402

ctrls = bench.build_controllers(bench.ENVS, 20, torch.device("cuda", 0))
probs = [c.qp for c in ctrls]
X, env, offsets = bench.sample_shard(0, bench.PER_GPU, [c.goal for c in ctrls])
B = X.shape[0]
res = {}
for chunks in ([B], [65536, 65536], [65536, 32768, 32768], [65536, 32768, 16384, 16384], [98304, 32768], [98304, 16384, 16384],
               [49152, 49152, 32768], [81920, 49152], [32768] * 4):
    hp = HostPipeline(probs, offsets, chunks)
    hp.Xh.copy_(torch.as_tensor(X))
    hp.solve(hp.Xh)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        hp.solve(hp.Xh)
    dt = (time.perf_counter() - t0) / 5
    res[str(chunks)] = round(B / dt / 1e6, 3)
    print(chunks, round(dt * 1e3, 3), "ms", res[str(chunks)], "M QP/s", flush=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "e2e_chunks.json"), "w"), indent=1)
