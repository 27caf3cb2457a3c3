"""Scripts in examples/ import ``lib`` relative to their own directory (as the
reference's examples do); point that package at the repository-root ``lib``."""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))), "lib")]
