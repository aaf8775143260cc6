"""Build the native libraries in-tree.

* ``lib/libspmm_hip.so``  — every HIP kernel in ``csrc/kernels/*.hip``,
  compiled for gfx950 only (``hipcc --offload-arch=gfx950``), C ABI launchers.
* ``lib/libspmm_host.so`` — the C++/OpenMP host runtime in ``csrc/host``:
  reference-format and Matrix-Market I/O, the CPU backend.
* ``bin/a4`` — the native drop-in executable (``csrc/runtime``: HIP engine,
  RCCL / MPI communicators, chain driver), linked against both libraries,
  RCCL and MPICH (``/opt/conda``, override with ``SPMM_MPI_HOME``).  Skipped
  with a message when no ``mpi.h`` is found.

Replaces the reference's Makefile (nvcc ``-arch=sm_35`` + mpicxx, Makefile:1-26).
Run ``python -m spmm_amd._build`` or call :func:`build`.  Rebuilds only when a
source or header is newer than the library.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "lib")
HIP_LIB = os.path.join(LIB_DIR, "libspmm_hip.so")
HOST_LIB = os.path.join(LIB_DIR, "libspmm_host.so")
BIN_DIR = os.path.join(PKG_DIR, "bin")
A4_BIN = os.path.join(BIN_DIR, "a4")
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (need ROCm in /opt/rocm)")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("native build failed: " + " ".join(cmd[:4]) + " ...")


def build_hip(force: bool = False, verbose: bool = False, out: str = HIP_LIB, extra=()) -> str:
    """``out`` / ``extra``: a diagnostic variant (e.g. ``-DSPMM_BM_STAMPS``)
    built next to the real library; load it with ``SPMM_HIP_LIB=<path>``.

    Every kernel file is compiled to its own object in parallel (one device
    code object per translation unit), objects are reused while their source
    and the shared headers are older, then one link."""
    from concurrent.futures import ThreadPoolExecutor

    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "kernels", "*.hpp"))
    deps = srcs + hdrs
    if force or _stale(out, deps):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        tag = "" if out == HIP_LIB else "_" + os.path.splitext(os.path.basename(out))[0]
        obj_dir = os.path.join(LIB_DIR, "obj" + tag)
        os.makedirs(obj_dir, exist_ok=True)
        flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
                 "-munsafe-fp-atomics", *extra]
        flag_file = os.path.join(obj_dir, "flags")
        same_flags = os.path.exists(flag_file) and open(flag_file).read() == " ".join(flags)

        def obj(src):
            o = os.path.join(obj_dir, os.path.basename(src) + ".o")
            if force or not same_flags or _stale(o, [src] + hdrs):
                cmd = [_hipcc(), *flags, "-c", src, "-o", o + ".tmp"]
                if verbose:
                    print(" ".join(cmd))
                _run(cmd)
                os.replace(o + ".tmp", o)
            return o

        with ThreadPoolExecutor(max_workers=min(len(srcs), max(1, (os.cpu_count() or 4) - 1))) as ex:
            objs = list(ex.map(obj, srcs))
        with open(flag_file, "w") as f:
            f.write(" ".join(flags))
        tmp = out + ".tmp"
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
        os.replace(tmp, out)
    return out


def build_host(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    deps = srcs + glob.glob(os.path.join(CSRC, "host", "*.hpp"))
    if force or _stale(HOST_LIB, deps):
        os.makedirs(LIB_DIR, exist_ok=True)
        tmp = HOST_LIB + ".tmp"
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-fvisibility=hidden",
               "-o", tmp] + srcs
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
        os.replace(tmp, HOST_LIB)
    return HOST_LIB


def mpi_home() -> str:
    return os.environ.get("SPMM_MPI_HOME", "/opt/conda")


def build_a4(force: bool = False, verbose: bool = False):
    """Native ``a4`` executable; returns its path or None without MPI headers."""
    rt = os.path.join(CSRC, "runtime")
    srcs = sorted(glob.glob(os.path.join(rt, "*.cpp"))) + sorted(glob.glob(os.path.join(rt, "*.hip")))
    deps = srcs + glob.glob(os.path.join(rt, "*.hpp")) + [HIP_LIB, HOST_LIB]
    mpi = mpi_home()
    if not os.path.exists(os.path.join(mpi, "include", "mpi.h")):
        if verbose:
            print(f"a4: no mpi.h under {mpi}; native executable not built")
        return None
    if force or _stale(A4_BIN, deps):
        os.makedirs(BIN_DIR, exist_ok=True)
        tmp = A4_BIN + ".tmp"
        # system libstdc++ before conda's (older) in the run path
        rpath = ":".join(["$ORIGIN/../lib", "/usr/lib/x86_64-linux-gnu", "/opt/rocm/lib", os.path.join(mpi, "lib")])
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-I", rt, "-I", os.path.join(mpi, "include"),
               "-o", tmp] + srcs + [
               "-L", LIB_DIR, "-lspmm_host", "-lspmm_hip", "-L/opt/rocm/lib", "-lrccl", "-lrocprofiler-sdk-roctx",
               # libmpi by path: a -L into conda would also pick conda's old libstdc++ at link time
               "-Wl," + os.path.join(mpi, "lib", "libmpi.so"), "-lpthread", f"-Wl,-rpath,{rpath}"]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
        os.replace(tmp, A4_BIN)
    return A4_BIN


def build(force: bool = False, verbose: bool = False) -> None:
    build_host(force, verbose)
    build_hip(force, verbose)
    build_a4(force, verbose)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
