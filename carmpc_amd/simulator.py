"""Nonlinear kinematic-bicycle plant (mirrors lib/simulator.py).

``CarSimulator`` is the reference's scalar plant (the *caller* of the QP path,
kept so the example loops run unchanged).  ``BatchCarSimulator`` steps B
plants at once on the GPU with the ``carmpc_plant_step_batch`` kernel
so a whole closed loop stays on the device.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


class CarTrailerDimension:
    """Vehicle geometry [m] (simulator.py:5-13); l1 is the wheelbase used by the model."""
    l1 = 3.5
    l2 = 4
    l12 = 1
    car_length = 5
    car_width = 2
    trailer_length = 5.5
    trailer_width = 2
    triangle_length = 2


def bicycle_rhs(state: np.ndarray, control_input: Sequence[float], l1: float = CarTrailerDimension.l1) -> np.ndarray:
    """Continuous-time kinematic bicycle  d/dt [x, y, psi, v] = [v cos psi, v sin psi, v tan(delta)/l1, a]."""
    _, _, psi, v = state
    a, delta = control_input
    return np.array([v * np.cos(psi), v * np.sin(psi), v / l1 * np.tan(delta), a])


class CarSimulator:
    """Scalar plant with forward-Euler integration (simulator.py:16-118).

    state = [x, y, psi, v]; input = [acceleration, steering angle]; output y = C x (+ Cd d)."""

    def __init__(self, dt: float = 0.01, clip: bool = False, C: np.ndarray = None, Cd: np.ndarray = None) -> None:
        self.time = 0
        self.l1, self.l2, self.l12 = CarTrailerDimension.l1, CarTrailerDimension.l2, CarTrailerDimension.l12
        self.state = np.zeros(4)
        self.dt = dt
        self.clip = clip
        self.C = np.eye(4) if C is None else C
        if self.C.shape[1] != 4:
            raise AssertionError(f"The length of the second dimension (currently {self.C.shape[1]}) of C should "
                                 "be equal to the state length (4).")
        self.output = self.C @ self.state
        self.Cd = Cd
        # limits used by check_input (simulator.py:25-29), with the reference's 0.05 margins
        self.x_lower, self.x_upper = -np.inf, np.inf
        self.y_lower, self.y_upper = -np.inf, np.inf
        self.psi_lower, self.psi_upper = -np.pi, np.pi
        self.v_lower, self.v_upper = -10, 10
        self.delta_lower, self.delta_upper = -np.pi / 4 - 0.05, np.pi / 4 + 0.05
        self.acc_lower, self.acc_upper = -2 - 0.05, 2 + 0.05

    def reset(self, state=np.zeros(5)) -> None:
        if np.array(state).shape != (4,):
            raise AssertionError(f"The state should have shape (4,), but has shape{np.array(state).shape}")
        self.state = state

    def dynamics_continuous(self, state: np.ndarray, control_input) -> np.ndarray:
        """One Euler step of the bicycle model (simulator.py:51-69): rhs * dt + state."""
        if np.array(control_input).shape != (2,):
            raise AssertionError(f"The input should have shape (2,), but has shape{np.array(control_input).shape}")
        return bicycle_rhs(state, control_input, self.l1) * self.dt + state

    def get_log(self, control_input) -> dict:
        a, delta_f = control_input
        return {"car": self.state, "inputs": np.array([a, delta_f])}

    def check_input(self, control_input):
        """Raise on inputs outside the (margined) actuator limits, or clip (simulator.py:83-97)."""
        a, delta_f = control_input
        if self.clip:
            return np.clip(control_input, [self.acc_lower, self.delta_lower], [self.acc_upper, self.delta_upper])
        # The reference compares Python lists, [a, -a] <= [acc_upper, -acc_lower]
        # (simulator.py:92-95): list order is lexicographic, so the lower limit is only looked at
        # when a == acc_upper, and inputs below it pass.  Kept as is: callers see the same
        # AssertionError for the same inputs.
        if not ([a, -a] <= [self.acc_upper, -self.acc_lower]):
            raise AssertionError(f"Acceleration should be between [{self.acc_lower, self.acc_upper}], but is {a}.")
        if not ([delta_f, -delta_f] <= [self.delta_upper, -self.delta_lower]):
            raise AssertionError(f"Steering angle should be between [{self.delta_lower:.3f}, "
                                 f"{self.delta_upper:.3f}], but is {delta_f}.")
        return control_input

    def step(self, control_input, d: float = None) -> dict:
        """Check the input, integrate one dt, update the output (simulator.py:99-118)."""
        self.check_input(control_input)
        self.state = self.dynamics_continuous(self.state, control_input)
        self.output = self.C @ self.state
        if self.Cd is not None and d is not None:
            self.output += self.Cd * d
        self.time += self.dt
        return self.get_log(control_input)


class BatchCarSimulator:
    """B independent plants on the GPU (device-resident state, HIP kernel step)."""

    def __init__(self, states, dt: float = 0.01, device=None):
        import torch
        from .qp import require_gpu
        self.device = require_gpu(device)
        self.state = torch.as_tensor(np.asarray(states, dtype=np.float64)).to(self.device).contiguous()
        self.dt = dt
        self.l1 = CarTrailerDimension.l1

    def step(self, u, stream=None):
        """Advance every plant by dt with inputs u (B x >=2); returns the input-limit flags."""
        from .qp import plant_step
        return plant_step(self.state, u, self.dt, self.l1, stream=stream)
