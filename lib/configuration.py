"""Drop-in shim: ``lib.configuration`` -> ``carmpc_amd.configuration`` (reference: lib/configuration.py)."""
from lib import _bootstrap  # noqa: F401  (puts the repository root on sys.path)
from carmpc_amd.configuration import *  # noqa: F401,F403
