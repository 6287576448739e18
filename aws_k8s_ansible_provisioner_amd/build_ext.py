"""In-tree native build: gfx950 HIP kernels + torch op glue -> ``_C.so``;
host C++ runtime (block manager, scheduler core, tokenizer) -> ``_runtime.so``.

Drives ``hipcc --offload-arch=gfx950`` directly (no hipify, no torch JIT cache), so the
built objects live next to the sources and travel with the repo snapshot to a GPU box.
Incremental: an object is rebuilt only when its source or any header is newer.

    python -m aws_k8s_ansible_provisioner_amd.build_ext [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "csrc", "build")
ARCH = os.environ.get("AKAP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append([HIPCC, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics",
                              "-c", src, "-o", obj])
    ops_src = os.path.join(CSRC, "ops.cpp")
    ops_obj = os.path.join(BUILD, "ops.cpp.o")
    objs.append(ops_obj)
    if force or _newer(ops_obj, [ops_src] + headers):
        incs = sum([["-I", i] for i in inc], [])
        jobs_list.append([HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                          "-DTORCH_EXTENSION_NAME=_C", *incs, "-I", "/opt/rocm/include", "-x", "c++", "-c", ops_src,
                          "-o", ops_obj])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    out = os.path.join(PKG, "_C.so")
    if force or jobs_list or not os.path.exists(out):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out,
              f"-L{lib}", f"-Wl,-rpath,{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
              "-ltorch_hip", "-lamdhip64"])
    return out


def build_runtime(force: bool = False, out_dir: str = PKG, sanitize: bool = False) -> str:
    """sanitize: -fsanitize=address,undefined build (host code only) into out_dir, for
    tools/sanitize_runtime.sh (load it with AKAP_RUNTIME_DIR=out_dir + LD_PRELOAD libasan)."""
    import pybind11

    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(out_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out = os.path.join(out_dir, "_runtime" + ext)
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=undefined"] if sanitize else ["-O3"]
    if force or sanitize or _newer(out, srcs + hdrs):
        _run(["g++", *flags, "-std=c++17", "-shared", "-fPIC", "-Wall", "-fvisibility=hidden",
              "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"], *srcs,
              "-o", out])
    return out


def build(force: bool = False, jobs: int = 8) -> None:
    build_runtime(force)
    build_kernels(force, jobs)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 8))
    ap.add_argument("--runtime-only", action="store_true")
    ap.add_argument("--sanitize-runtime", metavar="DIR", default=None,
                    help="ASan+UBSan build of the host runtime into DIR")
    a = ap.parse_args()
    if a.sanitize_runtime:
        print(build_runtime(True, a.sanitize_runtime, sanitize=True))
        return
    if a.runtime_only:
        print(build_runtime(a.force))
        return
    build(a.force, a.j)
    print("built", os.path.join(PKG, "_C.so"))


if __name__ == "__main__":
    sys.exit(main())
