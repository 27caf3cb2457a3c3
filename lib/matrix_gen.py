"""Drop-in shim: ``lib.matrix_gen`` -> ``carmpc_amd.matrix_gen`` (reference: lib/matrix_gen.py)."""
from lib import _bootstrap  # noqa: F401  (puts the repository root on sys.path)
from carmpc_amd.matrix_gen import *  # noqa: F401,F403
