#!/usr/bin/env python3
"""Per-phase cycle breakdown of the staged IPM kernel on the bench workload.

Needs the profiling build (python -m carmpc_amd.build --timing -> build/timing/libcarmpc.so,
kernels compiled with -DCARMPC_PHASE_TIMING).  Runs one step of bench.py's config-5 shard
and prints the share of wave-cycles per phase (clock64 deltas of lane 0, summed over waves).
The instrumentation itself perturbs scheduling (s_memtime waits on outstanding LDS/SMEM
traffic), so read the split, not the absolute numbers."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CARMPC_LIB"] = os.path.join(REPO, "build", "timing", "libcarmpc.so")
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from carmpc_amd import _native  # noqa: E402
from carmpc_amd.qp import SolverSettings  # noqa: E402

PHASES = ["residuals", "farkas/decisions", "M build", "cholesky", "rhs (G'/H products)", "triangular solves",
          "G dx + direction update", "step / polish verify"]


def main():
    kernel = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda", 0)
    ctrls = bench.build_problems(dev)
    probs = [c.qp for c in ctrls]
    X, env, offsets = bench.sample_shard(0, bench.PER_GPU, [c.goal for c in ctrls])
    Xd = torch.as_tensor(X).to(dev)
    lib = _native.load()
    fn = lib.carmpc_debug_phase_cycles
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = {}
    for j, p in enumerate(probs):
        sl = slice(int(offsets[j]), int(offsets[j + 1]))
        buf = (ctypes.c_ulonglong * 8)()
        p.solve(Xd[sl], settings=SolverSettings(kernel=kernel))      # warm
        torch.cuda.synchronize()
        fn(buf, 1)
        u, st, it = p.solve(Xd[sl], settings=SolverSettings(kernel=kernel))
        torch.cuda.synchronize()
        fn(buf, 1)
        c = np.array(list(buf), dtype=np.float64)
        iters = float(it.sum().item())
        out[bench.ENVS[j]] = {"share": {PHASES[i]: round(c[i] / c.sum(), 4) for i in range(8)},
                              "cycles_per_iteration": {PHASES[i]: round(c[i] / iters, 1) for i in range(8)},
                              "total_cycles_per_iteration": round(c.sum() / iters, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
