"""Drop-in shim: ``lib.simulator`` -> ``carmpc_amd.simulator`` (reference: lib/simulator.py)."""
from lib import _bootstrap  # noqa: F401  (puts the repository root on sys.path)
from carmpc_amd.simulator import *  # noqa: F401,F403
