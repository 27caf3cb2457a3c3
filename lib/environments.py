"""Drop-in shim: ``lib.environments`` -> ``carmpc_amd.environments`` (reference: lib/environments.py)."""
from lib import _bootstrap  # noqa: F401  (puts the repository root on sys.path)
from carmpc_amd.environments import *  # noqa: F401,F403
