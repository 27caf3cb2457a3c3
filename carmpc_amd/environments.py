"""Scenario definitions (mirrors lib/environments.py).

Each environment contributes extra per-step state half-spaces ``A x_k <= b``
(stacked on x_1..x_N by the controller, lib/mpc.py:240-248), a goal state
(used as the reference and in the terminal-set file name, lib/mpc.py:97) and a
name.  Plotting is presentation only and imports matplotlib lazily.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from .simulator import CarTrailerDimension

_ROAD_EDGE = 3.0          # |y| <= 3 (environments.py:56-57)
_GREY = (0.6, 0.6, 0.6)
_YELLOW = (0.91, 0.8, 0.18)
_PURPLE = (0.78, 0.18, 0.91)


class BaseEnv:
    """Empty scenario: no extra rows, no goal (environments.py:10-49)."""

    def __init__(self):
        self.constraints_A: list = []
        self.constraints_b: list = []
        self.goal = None
        self.lim = None
        self.name = "BaseEnv"
        self.check_constraints()
        self._legend = [("goal", "star", "lime")]

    def set_goal(self, goal: Sequence[float]) -> None:
        self.goal = goal

    def set_lim(self, lim) -> None:
        """Plot ranges [(x_min, x_max), (y_min, y_max)]."""
        self.lim = lim

    def check_constraints(self) -> None:
        if len(self.constraints_A) != len(self.constraints_b):
            raise AssertionError(f"The constraints array (len(A) = {len(self.constraints_A)} and "
                                 f"len(B) = {len(self.constraints_b)})do not have the same length.")

    # ---- presentation -------------------------------------------------------
    def _add_rows(self, rows, rhs):
        self.constraints_A += [list(r) for r in rows]
        self.constraints_b += list(rhs)
        self.check_constraints()

    def plot(self) -> None:
        import matplotlib.pyplot as plt
        self.x_lim, self.y_lim = self.lim
        plt.scatter(self.goal[0], self.goal[1], marker="*", c="lime")

    @property
    def handles(self):
        """Legend handles for the plots (matplotlib objects, built on demand)."""
        import matplotlib.lines as mlines
        import matplotlib.patches as patches
        out = []
        for label, kind, color in self._legend:
            if kind == "star":
                out.append(mlines.Line2D([], [], color=color, marker="*", linestyle="None", markersize=10,
                                         label=label))
            else:
                out.append(patches.Patch(color=color, label=label))
        return out


class RoadEnv(BaseEnv):
    """Two-lane road, |y| <= 3, goal [30, 1.5, 0, 0] (environments.py:52-79)."""

    def __init__(self):
        super().__init__()
        self._add_rows([[0, 1, 0, 0], [0, -1, 0, 0]], [3, 3])
        self.y_lower, self.y_upper = -_ROAD_EDGE, _ROAD_EDGE
        self.lim = [(-10, 50), (-10, 10)]
        self.name = "RoadEnv"
        self.goal = [30, 1.5, 0, 0]
        self._legend.append(("Road boundaries", "patch", _GREY))

    def plot(self) -> None:
        import matplotlib.pyplot as plt
        super().plot()
        xs = list(self.x_lim)
        plt.fill_between(xs, self.y_upper, self.y_lim[1], color=_GREY)
        plt.fill_between(xs, self.y_lower, self.y_lim[0], color=_GREY)
        plt.plot(xs, [0, 0], color=(0, 0, 0), linestyle=(0, (5, 10)))


def _cars(ax, x0s, y_center, color):
    import matplotlib.patches as patches
    d = CarTrailerDimension
    for x in x0s:
        ax.add_patch(patches.Rectangle((x, y_center - d.car_width / 2), d.car_length, d.car_width,
                                       edgecolor="none", facecolor=color))


class RoadOneCarEnv(RoadEnv):
    """Parked car ahead in the right lane: x <= 30, goal [29.9, -1.5, 0, 0] (environments.py:81-116)."""

    def __init__(self):
        super().__init__()
        self._add_rows([[1, 0, 0, 0]], [30])
        self.name = "RoadOneCarEnv"
        self.goal = [29.9, -1.5, 0, 0]
        self._legend.append(("Obstacles", "patch", _YELLOW))

    def plot(self) -> None:
        import matplotlib.pyplot as plt
        super().plot()
        d = CarTrailerDimension
        plt.vlines(30, self.y_lim[0], self.y_lim[1], color=_YELLOW, linestyle="--")
        plt.fill_between([30, self.x_lim[1]], self.y_lim[0], self.y_lim[1], color=_YELLOW + (0.1,))
        _cars(plt.gca(), [30 + d.car_length - d.l12 + i * 1.25 * d.car_length for i in range(3)], -1.5, _YELLOW)


class RoadMultipleCarsEnv(RoadEnv):
    """Two slanted half-planes around queued cars, goal [30, 1.5, 0, 0] (environments.py:118-172)."""

    def __init__(self):
        super().__init__()
        self._add_rows([[-0.25, 1, 0, 0], [0.25, -1, 0, 0]], [-2, 6.25])
        self.name = "RoadMultipleCarsEnv"
        self.goal = [30, 1.5, 0, 0]
        self._legend += [("Obstacles", "patch", _YELLOW), ("Obstacles", "patch", _PURPLE)]

    def plot(self) -> None:
        import matplotlib.pyplot as plt
        super().plot()
        d = CarTrailerDimension
        x = np.linspace(*self.x_lim, 2)
        for (a, rhs), color, fill_to in zip(zip(self.constraints_A[-2:], self.constraints_b[-2:]),
                                            (_YELLOW, _PURPLE), (self.y_lim[1], self.y_lim[0])):
            y = (-a[0] * x + rhs) / a[1]
            plt.plot(x, y, color=color, linestyle="--")
            plt.fill_between(x, y, fill_to, color=color + (0.1,))
        _cars(plt.gca(), [-1 - i * 1.25 * d.car_length for i in range(3)], 1.5, _YELLOW)
        _cars(plt.gca(), [30 + i * 1.25 * d.car_length for i in range(4)], -1.5, _PURPLE)


ENVIRONMENTS = {cls().name: cls for cls in (RoadEnv, RoadOneCarEnv, RoadMultipleCarsEnv)}
