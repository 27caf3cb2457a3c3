"""Drop-in shim: ``lib.visualize_state`` -> ``carmpc_amd.visualize_state`` (reference: lib/visualize_state.py)."""
from lib import _bootstrap  # noqa: F401  (puts the repository root on sys.path)
from carmpc_amd.visualize_state import *  # noqa: F401,F403
