"""Build the PyTorch-ROCm operator library (torch.ops.po2q.*) in-tree.

po2_quantization_amd/csrc/po2q_torch.cpp is host C++ on top of the C ABI (libpo2q.so):
compiled with the host compiler against torch's headers and the HIP runtime headers,
linked to libpo2q.so / libc10_hip / libtorch_hip, placed next to libpo2q.so
(po2_quantization_amd/lib/libpo2q_torch.so, rpath $ORIGIN) so it travels with the tree.

    python -m po2_quantization_amd.build_ext
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "po2q_torch.cpp")
LIBDIR = os.path.join(HERE, "lib")
OUT = os.path.join(LIBDIR, "libpo2q_torch.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")


def build(force=False):
    import torch
    from torch.utils import cpp_extension

    if not os.path.exists(os.path.join(LIBDIR, "libpo2q.so")):
        raise RuntimeError("po2q: build libpo2q.so first (make -C po2_quantization_amd/csrc)")
    deps = [SRC, os.path.join(INCLUDE, "po2q.h")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-parameter",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           "-D_GLIBCXX_USE_CXX11_ABI=%d" % int(torch._C._GLIBCXX_USE_CXX11_ABI)]
    for inc in cpp_extension.include_paths() + ["/opt/rocm/include", INCLUDE]:
        cmd += ["-I", inc]
    cmd += [SRC, "-o", OUT + ".tmp", "-L", LIBDIR, "-lpo2q", "-L", torch_lib, "-lc10", "-lc10_hip", "-ltorch",
            "-ltorch_cpu", "-ltorch_hip", "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,$ORIGIN",
            "-Wl,--no-as-needed"]
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
