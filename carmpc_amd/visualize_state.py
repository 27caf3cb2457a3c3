"""matplotlib views of a run (API mirror of lib/visualize_state.py: plot_history, plot_live, plot_graphs).

Presentation only; set ``MPLBACKEND=Agg`` when headless.
"""
from __future__ import annotations

import numpy as np

from .simulator import CarTrailerDimension


def _car_patch(ax, x, y, psi, edge):
    import matplotlib.patches as patches
    import matplotlib.transforms as transforms
    d = CarTrailerDimension
    rect = patches.Rectangle((x - d.l12, y - d.car_width / 2), d.car_length, d.car_width, edgecolor=edge,
                             facecolor="none")
    rect.set_transform(transforms.Affine2D().rotate_around(x, y, psi) + ax.transData)
    ax.add_patch(rect)


def _finish(ax, env, lim, extra_handles=()):
    import matplotlib.pyplot as plt
    handles, _ = ax.get_legend_handles_labels()
    ax.legend(loc="upper center", handles=list(handles) + list(env.handles if env is not None else []),
              bbox_to_anchor=(0.5, -0.15), fancybox=True, shadow=True, ncol=4)
    plt.xlim(*lim[0])
    plt.ylim(*lim[1])
    ax.set_aspect("equal", "box")


def _lim(env):
    return [(-40, 40), (-40, 40)] if env is None or env.lim is None else env.lim


def plot_history(log_data: dict, dt: float = 0.01, goal=None, env=None) -> None:
    """Trajectory in the x-y plane with the car drawn at the first and last sample (visualize_state.py:11-63)."""
    import matplotlib.pyplot as plt
    car = np.asarray(log_data["car"])
    plt.figure()
    ax = plt.gca()
    if env is not None:
        env.plot()
    ends = car[[0, -1]] if len(car) > 1 else car
    for x, y, psi in ends[:, :3]:
        _car_patch(ax, x, y, psi, "b")
    if goal is not None:
        plt.scatter(goal[0], goal[1], marker="*", c="lime")
    plt.title("The position of the car")
    plt.scatter(ends[:, 0], ends[:, 1], label="car", c="b")
    plt.plot(car[:, 0], car[:, 1], label="true traject", c="b", linestyle="--")
    if "estimate" in log_data:
        est = np.asarray(log_data["estimate"])
        plt.plot(est[:, 0], est[:, 1], label="est. traject", c=(1, 0, 0, 0.5), linestyle="--")
    _finish(ax, env, _lim(env))
    plt.show()


def plot_live(log_data: dict, dt: float = 0.01, time=None, estimate=None, state_horizon=None, env=None) -> None:
    """Redraw the scene for the current step and pause dt seconds (visualize_state.py:66-130)."""
    import matplotlib.pyplot as plt
    plt.cla()
    ax = plt.gca()
    if env is not None:
        env.plot()
    x, y, psi = np.asarray(log_data["car"])[:3]
    _car_patch(ax, x, y, psi, "b")
    if estimate is not None:
        _car_patch(ax, x, y, estimate[2], (1, 0, 0, 0.5))
        plt.scatter(x, y, label="state est.", c=[(1, 0, 0, 0.5)])
    if state_horizon is not None:
        plt.scatter(state_horizon[:, 0], state_horizon[:, 1], marker="x", c="black", label="pred. horz.")
    plt.title("The position of the car" if time is None else f"The position of the car(t = {time: .1f} s)")
    plt.scatter(x, y, label="car", c="b")
    _finish(ax, env, _lim(env))
    plt.pause(dt)


def plot_graphs(log_data: dict, dt: float = 0.01) -> None:
    """Each state against time (visualize_state.py:133-156)."""
    import matplotlib.pyplot as plt
    car = np.asarray(log_data["car"])
    t = np.arange(len(car)) * dt
    fig, axs = plt.subplots(4, 1, figsize=(5, 12), constrained_layout=True)
    fig.suptitle("Car states")
    for i, (name, unit) in enumerate(zip(("x", "y", r"\psi", "v"), ("m", "m", "rad", "m/s"))):
        axs[i].step(t, car[:, i], label="true state")
        if "estimate" in log_data:
            axs[i].step(t, np.asarray(log_data["estimate"])[:, i], label="state estimate")
        axs[i].set_title(f"${name}$")
        axs[i].set_xlabel("Time [s]")
        axs[i].set_ylabel(f"${name}$ [{unit}]")
        axs[i].legend()
    plt.show()
