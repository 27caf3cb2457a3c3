"""The C ABI used from a plain C program (examples/c_host/carmpc_solve.c, no Python on the
solve path): same statuses as the oracle and u within 1e-6 of the certified optimum."""
import os
import subprocess

import numpy as np
import pytest

from conftest import TERMINAL_SETS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("env", ["RoadEnv", "RoadMultipleCarsEnv"])
def test_c_host_solves(gpu_available, tmp_path, env):
    import c_host
    from oracle import assembly as oa
    from oracle import qp as oq
    asm = oa.build(env, 20, terminal_set_dir=TERMINAL_SETS)
    exe = c_host.build(tmp_path)
    c_host.write_problem(tmp_path / "problem.bin", asm)
    rng = np.random.default_rng(5)
    B = 64
    x0 = np.column_stack([rng.uniform(0, 28, B), rng.uniform(-2.5, 2.5, B), rng.uniform(-0.3, 0.3, B),
                          rng.uniform(0, 4, B)])
    x0[:16] = asm.goal + rng.normal(scale=0.3, size=(16, 4))
    x0.tofile(tmp_path / "x0.bin")
    r = subprocess.run([exe, str(tmp_path / "problem.bin"), str(tmp_path / "x0.bin"), str(tmp_path / "u.bin"),
                        str(tmp_path / "st.bin")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "solved 64 instances" in r.stdout
    u = np.fromfile(tmp_path / "u.bin", dtype=np.float64).reshape(B, 40)
    st = np.fromfile(tmp_path / "st.bin", dtype=np.int32)
    feasible = 0
    for b in range(B):
        ref = oq.solve_instance(asm, x0[b])
        if ref["status"] == 0 and ref["certified"]:
            feasible += 1
            assert st[b] == 0 and np.abs(u[b] - ref["u_exact"]).max() <= 1e-6, b
        elif ref["status"] == 1:
            assert st[b] == 1, b
    assert feasible >= 8
