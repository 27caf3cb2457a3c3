"""Terminal-set synthesis restatement (oracle/terminal_set.py, lib/terminal_set.py:23-213) pinned
against the reference's own outputs: the terminal_sets/*.npy files it ships.

RoadEnv_0_0_0_0.npy is not reproducible by the reference's current code: its rows carry
v >= 0 (today v >= -1, mpc.py:92-93) and a different closed-loop matrix, i.e. it was written by
an earlier configuration; it is checked only for its format."""
import glob
import os

import numpy as np
import pytest

from conftest import TERMINAL_SETS

STALE = {"RoadEnv_0_0_0_0.npy"}


def _cases():
    out = []
    for f in sorted(glob.glob(os.path.join(TERMINAL_SETS, "*.npy"))):
        parts = os.path.basename(f)[:-4].split("_")
        out.append((os.path.basename(f), parts[0], np.array([float(g) for g in parts[1:]])))
    return out


@pytest.mark.parametrize("fname,env,goal", [c for c in _cases() if c[0] not in STALE])
def test_oracle_reproduces_reference_terminal_sets(fname, env, goal):
    from oracle import terminal_set as ots
    ref = np.load(os.path.join(TERMINAL_SETS, fname))
    got = ots.calc_terminal_set(env, goal)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-9)


def test_stale_file_format():
    ref = np.load(os.path.join(TERMINAL_SETS, "RoadEnv_0_0_0_0.npy"))
    assert ref.shape[1] == 5
    # rows are not unit-norm either: written before the polytope normalisation/reduction step
    assert np.abs(np.linalg.norm(ref[:, :4], axis=1) - 1.0).max() > 0.1
    assert ref[3, 4] == 0.0 and np.array_equal(ref[3, :4], [0, 0, 0, -1])   # v >= 0: not today's v >= -1


def test_filename_rule():
    from carmpc_amd.environments import RoadMultipleCarsEnv, RoadOneCarEnv
    from carmpc_amd.terminal_set import filename_for
    assert filename_for(RoadMultipleCarsEnv()) == "RoadMultipleCarsEnv_30_1.5_0_0.npy"
    assert filename_for(RoadOneCarEnv()) == "RoadOneCarEnv_29.9_-1.5_0_0.npy"


def test_polytope_ops():
    from carmpc_amd.terminal_set import Polytope
    p = Polytope([[2.0, 0, 0, 0], [0, -3.0, 0, 0]], [4.0, 3.0])
    np.testing.assert_allclose(np.linalg.norm(p.A, axis=1), 1.0)
    np.testing.assert_allclose(p.b, [2.0, 1.0])
    q = p.translation([1.0, 1.0, 0, 0])
    np.testing.assert_allclose(q.b, [3.0, 0.0])       # {x : A (x - d) <= b}
    assert len(p.intersect(q)) == 4
