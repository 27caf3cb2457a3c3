"""Drop-in shim: ``lib.mpc`` -> ``carmpc_amd.mpc`` (reference: lib/mpc.py)."""
from lib import _bootstrap  # noqa: F401  (puts the repository root on sys.path)
from carmpc_amd.mpc import *  # noqa: F401,F403
from carmpc_amd.mpc import (MPC, MPCOutputFB, MPCOutputFBWithDisturbance, MPCStateFB,  # noqa: F401
                            OutsideTheRegionOfAttractionError, SolverError)
