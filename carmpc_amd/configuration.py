"""Controller constants of the CarMPC reference (mirrors lib/configuration.py:1-21).

``from carmpc_amd.configuration import *`` (or ``from lib.configuration import *``
through the drop-in shim) exposes the same CAPS names the reference examples use.
"""
import numpy as _np

__all__ = ["DT_CONTROL", "DT_SIMULATION", "STEPS_UPDATE", "LINEARIZE_STATE", "LINEARIZE_INPUT", "N",
           "STAGE_COST_Q", "STAGE_COST_R"]

#: MPC sample time [s]; inputs are held (ZOH) between updates.      (configuration.py:4)
DT_CONTROL = 0.2
#: integration step of the nonlinear plant [s].                      (configuration.py:7)
DT_SIMULATION = DT_CONTROL
#: plant steps per controller update.                                (configuration.py:9)
STEPS_UPDATE = int(DT_CONTROL / DT_SIMULATION)
#: linearisation point: state [x, y, psi, v] and input [a, delta].   (configuration.py:12-13)
LINEARIZE_STATE = [0, 0, 0, 3]
LINEARIZE_INPUT = [0, 0]
#: prediction horizon (steps).                                       (configuration.py:16)
N = 20
#: stage weights of the MPC / LQR cost.                              (configuration.py:19,21)
STAGE_COST_Q = _np.diag([5, 5, 10, 10])
STAGE_COST_R = _np.diag([10, 100])
