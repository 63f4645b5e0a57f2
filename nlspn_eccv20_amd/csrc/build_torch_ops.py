#!/usr/bin/env python3
"""Build the torch operator layer (nlspn_torch.cpp -> nlspn_eccv20_amd/lib/libnlspn_torch.so).

Host-only C++ against the installed PyTorch-ROCm headers and libraries, linked to
libnlspn_hip.so (same directory, rpath $ORIGIN).  Rebuilt only when a source is newer
than the library.  Run by __graft_entry__.build() after the HIP library.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.normpath(os.path.join(HERE, "..", "lib"))
OUT = os.path.join(LIB_DIR, "libnlspn_torch.so")
SRC = os.path.join(HERE, "nlspn_torch.cpp")
DEPS = [SRC, os.path.join(HERE, "..", "..", "include", "nlspn_prop.h"), __file__]


def command():
    import torch
    from torch.utils import cpp_extension as ce
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    incs = ce.include_paths() + ["/opt/rocm/include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return (["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wall", "-Wno-unused-function"]
            + [f"-I{p}" for p in incs]
            + [SRC, "-o", OUT, f"-L{torch_lib}", f"-L{LIB_DIR}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-lnlspn_hip", "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{torch_lib}",
               "-L/opt/rocm/lib", "-lamdhip64"])


def build(force=False):
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in DEPS):
        return OUT
    if not os.path.exists(os.path.join(LIB_DIR, "libnlspn_hip.so")):
        raise RuntimeError("build libnlspn_hip.so first (make -C nlspn_eccv20_amd/csrc)")
    subprocess.run(command(), check=True)
    return OUT


if __name__ == "__main__":
    print(build(force="-f" in sys.argv))
