"""Region-of-attraction grid search (the paper's closed-loop sweep) as one batched GPU run.

Every grid cell is a start position (x, y) with heading 0 and speed v; each car runs the
run_MPCStateFB.py runner loop (plant -> MPC step -> goal / time-out test) on the device.
Prints the outcome map: '#' reached the goal box, '.' left the region of attraction
(infeasible QP), 't' timed out."""
import argparse
import os
import time

import numpy as np

from lib.configuration import DT_CONTROL, LINEARIZE_INPUT, LINEARIZE_STATE, N
from lib.environments import RoadMultipleCarsEnv
from lib.mpc import MPCStateFB
from carmpc_amd.closed_loop import region_of_attraction

ap = argparse.ArgumentParser()
ap.add_argument("--nx", type=int, default=72)
ap.add_argument("--ny", type=int, default=24)
ap.add_argument("--v", type=float, default=2.0)
args = ap.parse_args()

env = RoadMultipleCarsEnv()
controller = MPCStateFB(dt=DT_CONTROL, N=N, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                        terminal_constraint=True, input_constraint=True, state_constraint=True, env=env,
                        terminal_set_dir=os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "terminal_sets"))
controller.set_goal(env.goal)
xs, ys = np.linspace(0.0, 28.0, args.nx), np.linspace(-2.9, 2.9, args.ny)
t0 = time.perf_counter()
roa = region_of_attraction(controller, xs, ys, psi=0.0, v=args.v)
dt = time.perf_counter() - t0
sym = {0: "#", 1: ".", 2: "!", 3: "t", 4: "?"}
for row in roa["outcome"][::-1]:
    print("".join(sym[int(o)] for o in row))
print(f"{roa['outcome'].size} closed-loop runs, {int(roa['steps'].sum())} MPC steps in {dt:.3f} s "
      f"({(roa['outcome'] == 0).mean():.1%} reach the goal)")
