"""carmpc_amd -- MI355X-native batched linear-MPC QP solver for the CarMPC controllers.

Drop-in for the per-step QP of ``lib/mpc.py`` (MPCStateFB / MPCOutputFB): the
controller API lives in ``carmpc_amd.mpc`` (also importable as ``lib.mpc``
through the shim package at the repository root); the batched GPU solver is
``carmpc_amd.qp.QPProblem``; the HIP kernels and the C ABI (include/carmpc.h)
are in ``carmpc_amd/csrc`` and build into ``carmpc_amd/libcarmpc.so``.
"""
__version__ = "0.1.0"

from ._native import CarMPCNativeError, LIB_PATH  # noqa: F401
