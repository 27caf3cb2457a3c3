#!/usr/bin/env python3
"""Resource metadata of the kernels in a compiled object (no GPU needed): VGPR / AGPR / SGPR
counts, LDS bytes, scratch bytes, spills, from the code object's notes.
usage: kernel_meta.py [build/obj/ipm_riccati.o] [substring filter of the demangled name]"""
import os
import re
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin/"


def kernels(obj):
    tmp = tempfile.mkdtemp()
    fb, co = os.path.join(tmp, "fatbin"), os.path.join(tmp, "dev.co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
    subprocess.run([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([LLVM + "llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    body = notes[notes.index("---") + 3:notes.rindex("...")]
    return yaml.safe_load(body)["amdhsa.kernels"], co


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else "build/obj/ipm_riccati.o"
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    ks, _ = kernels(obj)
    names = subprocess.run(["c++filt"], input="\n".join(k[".name"] for k in ks), capture_output=True,
                           text=True).stdout.splitlines()
    for k, dem in zip(ks, names):
        dem = re.sub(r"\(carmpc::RicSegs.*", "", dem).replace("carmpc::(anonymous namespace)::", "").replace("void ", "")
        if flt not in dem:
            continue
        print(f"{dem:72s} vgpr {k['.vgpr_count']:>3} agpr {k['.agpr_count']:>3} sgpr {k['.sgpr_count']:>3} "
              f"lds {k['.group_segment_fixed_size']:>6} scratch {k['.private_segment_fixed_size']:>4} "
              f"spill v/s {k['.vgpr_spill_count']}/{k['.sgpr_spill_count']} wg {k['.max_flat_workgroup_size']}")


if __name__ == "__main__":
    main()
