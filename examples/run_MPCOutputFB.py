"""Output-feedback MPC closed loop on the MI355X solver (the loop of the reference's
examples/run_MPCOutputFB.py: plant measures y = C x, observer + target + QP every step).

    cd examples && python run_MPCOutputFB.py [--start 5 -1.5 0 0] [--no-plot]"""
import argparse
import itertools
import os

import numpy as np

from lib.configuration import DT_CONTROL, DT_SIMULATION, LINEARIZE_INPUT, LINEARIZE_STATE, N, STEPS_UPDATE
from lib.environments import RoadMultipleCarsEnv
from lib.mpc import MPCOutputFB
from lib.simulator import CarSimulator


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=float, nargs=4, default=[5, -1.5, 0, 0])
    ap.add_argument("--no-plot", action="store_true", default=bool(os.environ.get("CARMPC_NO_PLOT")))
    args = ap.parse_args()
    env = RoadMultipleCarsEnv()
    ctrl = MPCOutputFB(dt=DT_CONTROL, N=N, lin_state=LINEARIZE_STATE, lin_input=LINEARIZE_INPUT,
                       init_state=list(args.start), terminal_constraint=True, input_constraint=True,
                       state_constraint=True, env=env)
    ctrl.set_goal(env.goal)
    plant = CarSimulator(dt=DT_SIMULATION, C=ctrl.C)
    plant.reset(np.array(args.start))
    u = [0, 0]
    true_states, estimates, inputs = [], [], []
    for step in itertools.count():
        log = plant.step(u)
        inputs.append(log["inputs"])
        if step % STEPS_UPDATE == 0:
            u = ctrl.step(plant.output)
            if not args.no_plot:
                from lib.visualize_state import plot_live
                plot_live(log, dt=0.1, time=plant.time, estimate=ctrl.x_estimate, state_horizon=ctrl.x_horizon,
                          env=env)
        true_states.append(log["car"])
        estimates.append(ctrl.x_estimate)
        if step >= 15 / DT_SIMULATION:
            break
    print(f"steps {len(true_states)} final {np.round(plant.state, 4)} estimate {np.round(ctrl.x_estimate, 4)}")
    if not args.no_plot:
        from lib.visualize_state import plot_graphs, plot_history
        history = {"car": np.array(true_states), "inputs": np.array(inputs), "estimate": np.array(estimates)}
        plot_history(history, dt=DT_SIMULATION, goal=ctrl.goal, env=env)
        plot_graphs(history, dt=DT_SIMULATION)


if __name__ == "__main__":
    main()
