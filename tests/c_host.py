"""Helpers for the C-host tests: build examples/c_host/carmpc_solve.c with gcc against the
in-tree libcarmpc.so and write its binary inputs."""
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def build(out_dir) -> str:
    exe = os.path.join(str(out_dir), "carmpc_solve")
    src = os.path.join(REPO, "examples", "c_host", "carmpc_solve.c")
    lib = os.path.join(REPO, "carmpc_amd")
    cmd = ["gcc", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(REPO, "include"),
           "-I" + os.path.join(ROCM, "include"), src, "-o", exe, "-L" + lib, "-lcarmpc",
           "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-Wl,-rpath," + lib, "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def write_problem(path, asm):
    """problem.bin for an oracle.assembly.Assembly (format in carmpc_solve.c)."""
    rows = np.asarray(asm.state_rows_A, float).reshape(-1, 4)
    rhs = np.asarray(asm.state_rows_b, float)
    tA = asm.term_A[:, -4:]
    tb = np.asarray(asm.term_b, float)
    from oracle import assembly as oa
    with open(path, "wb") as f:
        f.write(np.array([asm.N, len(rhs), len(tb)], dtype=np.int32).tobytes())
        for a in (asm.A, asm.B, oa.STAGE_COST_Q, oa.STAGE_COST_R, asm.P, rows, rhs, tA, tb, asm.input_lower,
                  asm.input_upper, asm.goal):
            f.write(np.ascontiguousarray(a, dtype=np.float64).tobytes())
