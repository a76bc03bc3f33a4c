"""Native build of the MI355X engine (in-tree, no JIT cache).

* ``libalaya_hip.so``  -- the C-ABI library (include/alaya_hip.h): HIP kernels for gfx950 + host C++
  (graph builder, on-disk formats), compiled with hipcc --offload-arch=gfx950.
* ``_alayalitepy*.so`` -- pybind11 module mirroring the reference binding, linked to the library.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU-only build container too.
"""

from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sysconfig
import time

import pybind11

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ALAYA_OFFLOAD_ARCH", "gfx950")

LIB = os.path.join(HERE, "libalaya_hip.so")
EXT = os.path.join(HERE, "_alayalitepy" + sysconfig.get_config_var("EXT_SUFFIX"))

LIB_SOURCES = ["search_kernels.hip", "build_kernels.hip", "flat_kernels.hip", "capi.cpp", "hnsw_build.cpp", "graph_update.cpp"]
LIB_HEADERS = ["search_kernels.h", "search_device.h", "build_kernels.h", "flat_kernels.h", "hnsw_build.h", "host_distance.h", "graph_update.h"]
EXT_SOURCES = ["pybind_module.cpp"]


def source_hash() -> str:
    """sha256 (first 16 hex digits) over the library's sources and headers, in a fixed order -- the
    value compiled into libalaya_hip.so (alaya_build_info) and compared with the tree at run time, so
    a stale or foreign library is visible in every bench line and smoke run."""
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, f) for f in LIB_SOURCES + LIB_HEADERS] + [os.path.join(INCLUDE, "alaya_hip.h")]:
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _hipcc_version() -> str:
    try:
        out = subprocess.run([HIPCC, "--version"], capture_output=True, text=True, check=True).stdout
    except (OSError, subprocess.CalledProcessError):
        return "unknown"
    for line in out.splitlines():
        if "HIP version" in line or "clang version" in line:
            return line.strip()
    return out.splitlines()[0].strip() if out else "unknown"


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build(force: bool = False, verbose: bool = False) -> tuple[str, str]:
    lib_deps = [os.path.join(CSRC, f) for f in LIB_SOURCES + LIB_HEADERS] + [os.path.join(INCLUDE, "alaya_hip.h")]
    if force or _newer(LIB, lib_deps):
        src_hash = source_hash()
        hipcc = "".join(c if c.isalnum() or c in ".-+:()" else "_" for c in _hipcc_version())
        info = f"source={src_hash} arch={ARCH} hipcc={hipcc} built={time.strftime('%Y-%m-%dT%H:%M:%SZ', time.gmtime())}"
        objs, procs = [], []
        for src in LIB_SOURCES:  # compile translation units concurrently
            obj = os.path.join(CSRC, os.path.splitext(src)[0] + ".o")
            flags = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-pthread",
                     f"-I{INCLUDE}", "-c", os.path.join(CSRC, src), "-o", obj]
            if src == "capi.cpp":  # alaya_build_info()
                flags.insert(1, f'-DALAYA_BUILD_INFO="{info}"')
            if src.endswith(".hip"):
                flags[1:1] = ["-x", "hip", f"--offload-arch={ARCH}"]
                # diagnostic builds only (e.g. -DALAYA_FINE_STAMPS for tools/profile_phases.py)
                flags[1:1] = os.environ.get("ALAYA_EXTRA_HIPFLAGS", "").split()
            if verbose:
                print(" ".join(flags), flush=True)
            procs.append((subprocess.Popen(flags), flags))
            objs.append(obj)
        for proc, flags in procs:
            if proc.wait() != 0:
                raise subprocess.CalledProcessError(proc.returncode, flags)
        _run([HIPCC, "-shared", "-fPIC", "-pthread", "-o", LIB] + objs + ["-lamdhip64"], verbose)
        for o in objs:
            os.remove(o)
        with open(os.path.join(HERE, "BUILD_INFO.json"), "w") as fh:
            json.dump({"source_hash": src_hash, "arch": ARCH, "hipcc": hipcc, "info": info}, fh)
    ext_deps = [os.path.join(CSRC, f) for f in EXT_SOURCES + ["host_distance.h"]] + [LIB]
    if force or _newer(EXT, ext_deps):
        py_inc = sysconfig.get_paths()["include"]
        _run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", "-Wall", "-fvisibility=hidden",
              f"-I{pybind11.get_include()}", f"-I{py_inc}", f"-I{INCLUDE}",
              os.path.join(CSRC, "pybind_module.cpp"), "-o", EXT, f"-L{HERE}", "-lalaya_hip",
              "-Wl,-rpath,$ORIGIN"], verbose)
    return LIB, EXT


if __name__ == "__main__":
    build(force=True, verbose=True)
