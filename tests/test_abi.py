"""The C ABI library: loads without a GPU and exports every symbol include/carmpc.h declares."""
import os
import re

from conftest import REPO


def _declared():
    with open(os.path.join(REPO, "include", "carmpc.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(carmpc_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported():
    from carmpc_amd import _native
    lib = _native.load()
    names = _declared()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(_native.EXPORTS) == names


def test_exports_are_c_linkage():
    out = os.popen(f"nm -D --defined-only {os.path.join(REPO, 'carmpc_amd', 'libcarmpc.so')}").read()
    for n in _declared():
        assert re.search(rf"\sT\s{n}$", out, re.M), n


def test_host_only_entry_points():
    from carmpc_amd import _native
    lib = _native.load()
    assert _native.version().startswith("carmpc-mi355x")
    # canonical dense-IPM count: p n^2 + n^3/3 + 6 n^2 + 12 p n
    assert abs(lib.carmpc_canonical_flops_per_iter(40, 202) - 451093.333) < 1e-2
    assert abs(lib.carmpc_canonical_flops_per_iter(20, 85) - 59466.667) < 1e-2
    # argument validation happens before any device call
    import ctypes
    rc = lib.carmpc_problem_create(None, ctypes.byref(ctypes.c_void_p()))
    assert rc == -1 and b"null" in lib.carmpc_last_error()


def test_build_entry_declares_gfx950():
    from carmpc_amd import build
    assert "--offload-arch=gfx950" in build.FLAGS
    import subprocess
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readobj", "--elf-output-style=GNU", "--notes",
                          os.path.join(REPO, "carmpc_amd", "libcarmpc.so")], capture_output=True, text=True)
    blob = open(os.path.join(REPO, "carmpc_amd", "libcarmpc.so"), "rb").read()
    assert b"gfx950" in blob


def test_c_host_compiles(tmp_path):
    """The header is plain C: a C host (examples/c_host) builds with gcc -Wall -Werror and links
    the in-tree library."""
    import c_host
    exe = c_host.build(tmp_path)
    assert os.path.exists(exe)
