"""State-feedback MPC closed loop on the MI355X solver (the loop of the reference's
examples/run_MPCStateFB.py: plant step, then controller step every STEPS_UPDATE).

    cd examples && python run_MPCStateFB.py [--env RoadMultipleCarsEnv] [--start 5 -1.5 0.1 0]

Set CARMPC_NO_PLOT=1 (or pass --no-plot) to skip the matplotlib views."""
import argparse
import itertools
import os

import numpy as np

from lib.configuration import DT_CONTROL, DT_SIMULATION, LINEARIZE_INPUT, LINEARIZE_STATE, N, STEPS_UPDATE
from lib.environments import RoadEnv, RoadMultipleCarsEnv, RoadOneCarEnv
from lib.mpc import MPCStateFB
from lib.simulator import CarSimulator


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="RoadMultipleCarsEnv", choices=["RoadEnv", "RoadOneCarEnv", "RoadMultipleCarsEnv"])
    ap.add_argument("--start", type=float, nargs=4, default=[5, -1.5, 0.1, 0])
    ap.add_argument("--horizon", type=int, default=N)
    ap.add_argument("--no-plot", action="store_true", default=bool(os.environ.get("CARMPC_NO_PLOT")))
    args = ap.parse_args()
    env = {"RoadEnv": RoadEnv, "RoadOneCarEnv": RoadOneCarEnv, "RoadMultipleCarsEnv": RoadMultipleCarsEnv}[args.env]()
    ctrl = MPCStateFB(dt=DT_CONTROL, N=args.horizon, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                      terminal_constraint=True, input_constraint=True, state_constraint=True, env=env)
    ctrl.set_goal(env.goal)
    print(ctrl.P)
    plant = CarSimulator(dt=DT_SIMULATION)
    plant.reset(np.array(args.start))
    u = [0, 0]
    states, inputs = [], []
    for step in itertools.count():
        log = plant.step(u)
        states.append(log["car"])
        inputs.append(log["inputs"])
        if step % STEPS_UPDATE == 0:
            u = ctrl.step(plant.state)
            if not args.no_plot:
                from lib.visualize_state import plot_live
                plot_live(log, dt=0.01, time=plant.time, state_horizon=ctrl.x_horizon, env=env)
        if np.all(np.abs(plant.state - ctrl.goal) <= 1e-1) or step > 30 / DT_SIMULATION:
            break
    print(f"steps {len(states)} final {np.round(plant.state, 4)}")
    if not args.no_plot:
        from lib.visualize_state import plot_graphs, plot_history
        history = {"car": np.array(states), "inputs": np.array(inputs)}
        plot_history(history, dt=DT_SIMULATION, goal=ctrl.goal, env=env)
        plot_graphs(history, dt=DT_SIMULATION)


if __name__ == "__main__":
    main()
