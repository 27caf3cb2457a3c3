#!/usr/bin/env python3
"""Per-phase cycle breakdown of the grouped Riccati kernel (settings.kernel 7) on the bench
workload.  Needs the profiling build (python -m carmpc_amd.build --timing).  Instrumentation
perturbs scheduling: read the split, not the absolute numbers."""
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

PHASES = ["init", "residual rows", "adjoint pass", "decisions", "factor rows", "factorization pass",
          "backward passes", "forward passes", "rows k0 (predictor)", "rows k1 (corrector)", "rows k2 (step)",
          "polish rows / loop"]


def main():
    """Phase split per launch kind (translation unit) on the bench shard solved in one call (the three-launch form)."""
    dev = torch.device("cuda", 0)
    ctrls = bench.build_controllers(bench.ENVS, 20, dev)
    probs = [c.qp for c in ctrls]
    X, env, offsets = bench.sample_shard(0, bench.PER_GPU, [c.goal for c in ctrls])
    Xd = torch.as_tensor(X).to(dev)
    from carmpc_amd.qp import solve_segments
    lib = _native.load()
    out = {}
    units = {"m1": "iteration launch", "m2": "polish launch", "m0": "single kernel (retry launch)"}
    fns = {}
    for u in units:
        fn = getattr(lib, "carmpc_debug_ric_cycles_" + u)
        fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        fns[u] = fn
    buf = (ctypes.c_ulonglong * 12)()
    solve_segments(probs, offsets, Xd)
    torch.cuda.synchronize()
    for u in units:
        fns[u](buf, 1)
    solve_segments(probs, offsets, Xd)
    torch.cuda.synchronize()
    for u, what in units.items():
        fns[u](buf, 1)
        c = np.array(list(buf), dtype=np.float64)
        out[what] = {"share": {PHASES[i]: round(float(c[i] / max(c.sum(), 1.0)), 4) for i in range(12)},
                     "total_cycles_all_waves": float(c.sum())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
