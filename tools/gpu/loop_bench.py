"""Throughput of the device closed loop (carmpc_closed_loop_batch): B random start states of
RoadMultipleCarsEnv through the run_MPCStateFB.py runner; prints one JSON line with closed-loop
runs/s and MPC steps (QP solves inside the loop)/s."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from carmpc_amd.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE, N  # noqa: E402
from carmpc_amd.environments import RoadMultipleCarsEnv  # noqa: E402
from carmpc_amd.mpc import MPCStateFB  # noqa: E402
from carmpc_amd.closed_loop import run_closed_loop  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--reps", type=int, default=2)
args = ap.parse_args()
env = RoadMultipleCarsEnv()
REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
c = MPCStateFB(dt=DT_CONTROL, N=N, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT, env=env,
               terminal_set_dir=os.path.join(REPO, "terminal_sets"))
rng = np.random.default_rng(0)
B = args.batch
starts = np.column_stack([rng.uniform(0, 25, B), rng.uniform(-2.8, 2.8, B), rng.uniform(-0.3, 0.3, B),
                          rng.uniform(0, 5, B)])
run_closed_loop(c, starts[:1024])   # warm-up
best = None
for _ in range(args.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = run_closed_loop(c, starts)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    best = dt if best is None else min(best, dt)
steps = int(res["steps"].sum())
out = {"batch": B, "seconds": best, "runs_per_s": B / best, "mpc_steps": steps, "mpc_steps_per_s": steps / best,
       "outcomes": {str(k): int((res["outcome"] == k).sum()) for k in range(5)}}
print(json.dumps(out))
