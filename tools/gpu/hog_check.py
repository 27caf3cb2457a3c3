"""Pipeline against single-kernel solves while another stream keeps part of the CUs busy (build/probe/libpoison.so):
the solver's workgroups start late and unevenly, so instances meet other groups, waves and list positions than in a
quiet run.  Results must not depend on that.  Usage: python tools/gpu/hog_check.py [trials]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from conftest import TERMINAL_SETS  # noqa: E402
from carmpc_amd.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE  # noqa: E402
from carmpc_amd.environments import ENVIRONMENTS  # noqa: E402
from carmpc_amd.mpc import MPCStateFB  # noqa: E402
from carmpc_amd.qp import solve_segments  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "..", "build", "probe", "libpoison.so"))
lib.hog.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

# (workgroups, LDS bytes, spin rounds)
HOGS = [None, (128, 150 * 1024, 400), (256, 150 * 1024, 100), (2048, 2048, 3000), (512, 64 * 1024, 300), (64, 150 * 1024, 2000)]


def states(n, seed):
    rng = np.random.default_rng(seed)
    return np.column_stack([rng.uniform(0, 28, n), rng.uniform(-2.5, 2.5, n), rng.uniform(-0.3, 0.3, n), rng.uniform(0, 4, n)])


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    p20 = [MPCStateFB(dt=DT_CONTROL, N=20, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT, env=ENVIRONMENTS[e](),
                      terminal_set_dir=TERMINAL_SETS).qp for e in ("RoadEnv", "RoadOneCarEnv", "RoadMultipleCarsEnv")]
    p10 = MPCStateFB(dt=DT_CONTROL, N=10, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT, env=ENVIRONMENTS["RoadEnv"](),
                     terminal_set_dir=TERMINAL_SETS).qp
    cases = {"first_offset_positive": ([p20[1], p20[2]], np.array([5000, 33000, 61000])),
             "leading_other_horizon": ([p10, p20[0], p20[2]], np.array([0, 3000, 30000, 56000]))}
    side = torch.cuda.Stream()
    total_bad = 0
    for name, (probs, offsets) in cases.items():
        B = int(offsets[-1]) + 100
        X = torch.as_tensor(states(B, 21)).cuda()
        ref = []
        for j, p in enumerate(probs):
            ref.append(tuple(t.clone() for t in p.solve(X[int(offsets[j]):int(offsets[j + 1])])))
        torch.cuda.synchronize()
        for hog in HOGS:
            for trial in range(trials):
                for which in ("segments", "single"):
                    u = torch.full((B, 40), -7.0, dtype=torch.float64, device="cuda")
                    st = torch.full((B,), -7, dtype=torch.int32, device="cuda")
                    it = torch.full((B,), -7, dtype=torch.int32, device="cuda")
                    torch.cuda.synchronize()
                    t0 = torch.cuda.Event(enable_timing=True)
                    t1 = torch.cuda.Event(enable_timing=True)
                    if hog:
                        assert lib.hog(hog[0], hog[1], hog[2], ctypes.c_void_p(side.cuda_stream)) == 0
                    t0.record()
                    if which == "segments":
                        solve_segments(probs, offsets, X, out=(u, st, it))
                        got = [(u[int(offsets[j]):int(offsets[j + 1]), :p.n], st[int(offsets[j]):int(offsets[j + 1])],
                                it[int(offsets[j]):int(offsets[j + 1])]) for j, p in enumerate(probs)]
                    else:
                        got = [p.solve(X[int(offsets[j]):int(offsets[j + 1])]) for j, p in enumerate(probs)]
                    t1.record()
                    torch.cuda.synchronize()
                    for j, ((u1, s1, i1), (u0, s0, i0)) in enumerate(zip(got, ref)):
                        bad = ((s1 != s0) | (i1 != i0)).nonzero().flatten()
                        if bad.numel():
                            total_bad += int(bad.numel())
                            b8 = bad[:8]
                            print("MISMATCH", name, hog, trial, which, "seg", j, "count", int(bad.numel()), "idx", b8.tolist(),
                                  "status", s1[b8].tolist(), "ref", s0[b8].tolist(), "iters", i1[b8].tolist(), "ref", i0[b8].tolist(),
                                  flush=True)
                    print("done", name, hog, trial, which, "%.2f ms" % t0.elapsed_time(t1), flush=True)
    print("total mismatches", total_bad)


if __name__ == "__main__":
    main()
