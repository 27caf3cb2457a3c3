"""Build libcarmpc.so in-tree for gfx950 (hipcc).  ``python -m carmpc_amd.build``."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(REPO, "build", "obj")
LIB = os.path.join(HERE, "libcarmpc.so")
SOURCES = ["ipm_riccati_m0.hip", "ipm_riccati_m1.hip", "ipm_riccati_m2.hip", "ipm_riccati_het.hip",    # (slowest first)
           "capi.hip", "assembly.hip", "ipm_dense.hip", "ipm_staged.hip", "ipm_riccati.hip", "closed_loop.hip", "lp.hip",
           "hetero.hip", "noalloc.hip", "cpu_ipm.hip"]
ARCH = os.environ.get("CARMPC_ARCH", "gfx950")
# -packed-fp32-ops off: hipcc -O3 forms v_pk_*_f32 from ordinary float code by itself and some of
# their forms have given wrong results on these GPUs; the flag only concerns the device pass (the
# host pass warns that it does not know the feature, which is harmless).
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
         "-I" + os.path.join(REPO, "include")]
# Per-file code generation: the Riccati kernel runs one wave per SIMD and is latency-bound in
# its stage recursions; the iterative ILP scheduler gains ~3 % there (tools/gpu/sched_sweep.sh:
# 6.71M -> 6.91M QP/s; max-ilp, max-memory-clause, iterative-minreg/maxocc were slower).
# --amdgpu-mfma-vgpr-form keeps the matrix-core results in ordinary registers: they feed vector
# FMAs at once, and the default (accumulation-register results) cost ~19 register moves per stage
# of the factorization pass (10.07M -> 10.35M QP/s).
# The kernel is instantiated in one translation unit per launch kind (ipm_riccati_m0 / m1 / m2 / het.hip), so
# that each can have its own flags and the four compile side by side.
_RIC = ["-mllvm", "--amdgpu-sched-strategy=iterative-ilp", "-mllvm", "--amdgpu-mfma-vgpr-form"]
# The polish launch's unit keeps the default scheduler: with the iterative-ILP strategy the register allocator of
# this hipcc (ROCm 7.2.0, clang 22) crashes on its 32-lanes-per-QP instantiation at N = 10.
FILE_FLAGS = {"ipm_riccati_m0.hip": _RIC, "ipm_riccati_m1.hip": _RIC, "ipm_riccati_m2.hip": _RIC[2:], "ipm_riccati_het.hip": _RIC}


def _hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _stale(obj, src, cmd):
    """Rebuild when the object is missing, older than its sources, or was built by another command line."""
    if not os.path.exists(obj) or not os.path.exists(obj + ".cmd"):
        return True
    with open(obj + ".cmd") as f:
        if f.read() != " ".join(cmd):
            return True
    deps = [src, os.path.join(REPO, "include", "carmpc.h"), os.path.join(CSRC, "carmpc_internal.h"), os.path.join(CSRC, "lanes.h")]
    if os.path.basename(src).startswith("ipm_riccati"):
        deps += [os.path.join(CSRC, "ipm_riccati_kernel.h"), os.path.join(CSRC, "ipm_riccati_solve.inc")]
    return any(os.path.getmtime(d) > os.path.getmtime(obj) for d in deps)


def build(verbose: bool = True, jobs: int = 8, variant: str = "") -> str:
    """Compile csrc/*.hip for gfx950 and link the shared library.  variant="timing"
    builds the phase-timing profiling library build/timing/libcarmpc.so instead."""
    obj_dir = OBJ if not variant else os.path.join(REPO, "build", variant, "obj")
    lib_path = LIB if not variant else os.path.join(REPO, "build", variant, "libcarmpc.so")
    extra = {"": [], "timing": ["-DCARMPC_PHASE_TIMING"]}[variant]
    os.makedirs(obj_dir, exist_ok=True)
    hipcc = _hipcc()

    def compile_one(src):
        s = os.path.join(CSRC, src)
        o = os.path.join(obj_dir, src.replace(".hip", ".o"))
        cmd = [hipcc, *FLAGS, *FILE_FLAGS.get(src, []), *extra, "-c", s, "-o", o]
        if _stale(o, s, cmd):
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            with open(o + ".cmd", "w") as f:
                f.write(" ".join(cmd))
        return o

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    if not os.path.exists(lib_path) or any(os.path.getmtime(o) > os.path.getmtime(lib_path) for o in objs):
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", lib_path]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return lib_path


if __name__ == "__main__":
    build(verbose="-q" not in sys.argv, variant="timing" if "--timing" in sys.argv else "")
