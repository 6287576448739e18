"""In-tree native build: gfx950 HIP kernels + torch op glue -> ``_C.so``;
host C++ runtime (block manager, scheduler core, tokenizer) -> ``_runtime.so``.

Drives ``hipcc --offload-arch=gfx950`` directly (no hipify, no torch JIT cache), so the
built objects live next to the sources and travel with the repo snapshot to a GPU box.

Content-addressed, not mtime-based: every object records the SHA-256 of what it was built
from (its source, every header, the compile command, the torch version it compiles against)
in ``<obj>.sha`` and is rebuilt exactly when that digest changes.  The digest of the whole
kernel tree is compiled INTO ``_C.so`` (``akap_build_hash()``, a generated C file linked in)
and into ``_runtime`` (``build_hash()``); ``ops.load_native`` recomputes it from the sources
beside the library and refuses a library built from different sources, so a tested ``_C.so``
provably came from the tree it was tested with.

    python -m aws_k8s_ansible_provisioner_amd.build_ext [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
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


def torch_version() -> str:
    import torch

    return torch.__version__


def _digest(files: list[str], extra: str = "") -> str:
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(os.path.relpath(f, PKG).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(extra.encode())
    return h.hexdigest()


def kernel_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) +
                  glob.glob(os.path.join(CSRC, "kernels", "*.h")) +
                  [os.path.join(CSRC, "ops.cpp")])


def runtime_sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")) +
                  glob.glob(os.path.join(CSRC, "runtime", "*.h")))


def kernel_tree_hash() -> str:
    """Digest of everything _C.so is built from (sources, headers, arch, torch version)."""
    return _digest(kernel_sources(), f"arch={ARCH};torch={torch_version()}")


def runtime_tree_hash() -> str:
    return _digest(runtime_sources(), f"python={sysconfig.get_config_var('EXT_SUFFIX')}")


class BuildLog:
    def __init__(self):
        self.lines: list[str] = []

    def __call__(self, msg: str) -> None:
        self.lines.append(msg)
        print(f"[build_ext] {msg}", flush=True)


def _stale(obj: str, digest: str) -> str:
    """'' when obj exists and was built from `digest`, else the reason it must be rebuilt."""
    if not os.path.exists(obj):
        return "no object"
    try:
        with open(obj + ".sha") as f:
            old = f.read().strip()
    except OSError:
        return "no recorded digest"
    return "" if old == digest else "inputs changed"


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)


def _compile(job) -> None:
    cmd, obj, digest = job
    _run(cmd)
    with open(obj + ".sha", "w") as f:
        f.write(digest + "\n")


def build_kernels(force: bool = False, jobs: int = 8, log=None) -> str:
    log = log or BuildLog()
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    tv = torch_version()
    common = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    jobs_list = []
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        cmd = [HIPCC, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics", "-c", src, "-o",
               obj]
        digest = _digest([src] + headers, " ".join(cmd[:-3]))
        why = "forced" if force else _stale(obj, digest)
        if why:
            log(f"compile {os.path.basename(src)} ({why})")
            jobs_list.append((cmd, obj, digest))
    ops_src = os.path.join(CSRC, "ops.cpp")
    ops_obj = os.path.join(BUILD, "ops.cpp.o")
    objs.append(ops_obj)
    incs = sum([["-I", i] for i in inc], [])
    cmd = [HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           "-DTORCH_EXTENSION_NAME=_C", *incs, "-I", "/opt/rocm/include", "-x", "c++", "-c",
           ops_src, "-o", ops_obj]
    digest = _digest([ops_src] + headers, " ".join(cmd[:-3]) + f";torch={tv}")
    why = "forced" if force else _stale(ops_obj, digest)
    if why:
        log(f"compile ops.cpp ({why})")
        jobs_list.append((cmd, ops_obj, digest))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_compile, jobs_list))
    out = os.path.join(PKG, "_C.so")
    tree = kernel_tree_hash()
    # the tree digest compiled into the library (read back by ops.load_native via ctypes)
    info_src = os.path.join(BUILD, "build_info.c")
    info_obj = info_src + ".o"
    with open(info_src, "w") as f:
        f.write(f'const char* akap_build_hash(void) {{ return "{tree}"; }}\n'
                f'const char* akap_build_torch(void) {{ return "{tv}"; }}\n')
    _run(["gcc", "-O1", "-fPIC", "-c", info_src, "-o", info_obj])
    link_digest = _digest(objs + [info_obj])
    why = "forced" if force else ("objects rebuilt" if jobs_list else _stale(out, link_digest))
    if why:
        log(f"link _C.so ({why}); tree {tree[:16]}, torch {tv}")
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, info_obj, "-o", out,
              f"-L{lib}", f"-Wl,-rpath,{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
              "-ltorch_hip", "-lamdhip64"])
        with open(out + ".sha", "w") as f:
            f.write(_digest(objs + [info_obj]) + "\n")
    else:
        log(f"reuse _C.so: built from this tree ({tree[:16]}, torch {tv})")
    return out


def build_runtime(force: bool = False, out_dir: str = PKG, sanitize: bool = False,
                  log=None) -> str:
    """sanitize: -fsanitize=address,undefined build (host code only) into out_dir, for
    tools/sanitize_runtime.sh (load it with AKAP_RUNTIME_DIR=out_dir + LD_PRELOAD libasan)."""
    import pybind11

    log = log or BuildLog()
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(out_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    ext = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out = os.path.join(out_dir, "_runtime" + ext)
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=undefined"] if sanitize else ["-O3"]
    tree = runtime_tree_hash()
    cmd = ["g++", *flags, "-std=c++17", "-shared", "-fPIC", "-Wall", "-fvisibility=hidden",
           f'-DAKAP_RT_HASH="{tree}"', "-I", pybind11.get_include(), "-I",
           sysconfig.get_paths()["include"], *srcs, "-o", out]
    digest = _digest(runtime_sources(), " ".join(cmd))
    why = "forced" if force else ("sanitizer build" if sanitize else _stale(out, digest))
    if why:
        log(f"build {os.path.basename(out)} ({why})")
        _run(cmd)
        with open(out + ".sha", "w") as f:
            f.write(digest + "\n")
    else:
        log(f"reuse {os.path.basename(out)}: built from this tree ({tree[:16]})")
    return out


def build_pmc_tool(force: bool = False, log=None) -> str:
    """The rocprofiler-sdk counter tool (csrc/tools/pmc_tool.cpp) -> libakap_pmc.so: host code
    only, loaded by the ROCm runtime through ROCP_TOOL_LIBRARIES (exporter/pmc_sampler.py)."""
    log = log or BuildLog()
    src = os.path.join(CSRC, "tools", "pmc_tool.cpp")
    out = os.path.join(PKG, "libakap_pmc.so")
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-shared", "-fPIC", "-fvisibility=hidden",
           "-I/opt/rocm/include", src, "-o", out, "-L/opt/rocm/lib", "-lrocprofiler-sdk",
           "-Wl,-rpath,/opt/rocm/lib"]
    digest = _digest([src], " ".join(cmd))
    why = "forced" if force else _stale(out, digest)
    if why:
        log(f"build libakap_pmc.so ({why})")
        _run(cmd)
        with open(out + ".sha", "w") as f:
            f.write(digest + "\n")
    else:
        log("reuse libakap_pmc.so: built from this tree")
    return out


def build(force: bool = False, jobs: int = 8) -> list[str]:
    """Build every native library; returns the log lines (what was compiled or reused, and
    why)."""
    log = BuildLog()
    build_runtime(force, log=log)
    build_pmc_tool(force, log=log)
    build_kernels(force, jobs, log=log)
    return log.lines


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
