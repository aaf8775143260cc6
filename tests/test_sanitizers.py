"""Host-code sanitizers: the native a4 built with AddressSanitizer
+ UndefinedBehaviorSanitizer on its host code (hipcc ``-Xarch_host -fsanitize=``;
GPU code is not instrumented) and run with the CPU engine under mpiexec, so the
reader, writer, canonicalisation, CPU multiply, row-panel split tree and MPI
transport all execute instrumented.  The reference's latent bugs of this class
(erase during iteration :589/:633, unchecked staging overflow :193-211) are the
motivation.  The instrumented binary is cached under build/ (git-ignored)."""
import os
import subprocess

import pytest

import spmm_amd  # noqa: F401
from spmm_amd import _build
from spmm_amd.utils import gen, golden, refio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN_BIN = os.path.join(ROOT, "build", "a4_asan")
MPIEXEC = os.path.join(_build.mpi_home(), "bin", "mpiexec")


def _sources():
    rt = os.path.join(_build.CSRC, "runtime")
    host = os.path.join(_build.CSRC, "host")
    srcs = sorted(os.path.join(rt, f) for f in os.listdir(rt) if f.endswith((".cpp", ".hip")))
    srcs += sorted(os.path.join(host, f) for f in os.listdir(host) if f.endswith(".cpp"))
    deps = srcs + [os.path.join(d, f) for d in (rt, host) for f in os.listdir(d) if f.endswith(".hpp")]
    return srcs, deps


@pytest.fixture(scope="module")
def san_bin():
    mpi = _build.mpi_home()
    if not os.path.exists(os.path.join(mpi, "include", "mpi.h")) or not os.path.exists(MPIEXEC):
        pytest.skip("no MPICH")
    hip_lib = _build.build_hip()
    srcs, deps = _sources()
    if _build._stale(SAN_BIN, deps + [hip_lib]):
        os.makedirs(os.path.dirname(SAN_BIN), exist_ok=True)
        rpath = ":".join([_build.LIB_DIR, "/usr/lib/x86_64-linux-gnu", "/opt/rocm/lib", os.path.join(mpi, "lib")])
        cmd = [_build._hipcc(), f"--offload-arch={_build.ARCH}", "-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17",
               "-fopenmp", "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
               "-I", os.path.join(_build.CSRC, "runtime"), "-I", os.path.join(mpi, "include"),
               "-o", SAN_BIN + ".tmp"] + srcs + [
               "-L", _build.LIB_DIR, "-lspmm_hip", "-L/opt/rocm/lib", "-lrccl", "-lrocprofiler-sdk-roctx",
               "-Wl," + os.path.join(mpi, "lib", "libmpi.so"), "-lpthread", f"-Wl,-rpath,{rpath}"]
        _build._run(cmd)
        os.replace(SAN_BIN + ".tmp", SAN_BIN)
    return SAN_BIN


@pytest.mark.parametrize("n,p", [(9, 3), (6, 1), (8, 4)])
def test_a4_host_code_asan_ubsan_clean(tmp_path, san_bin, n, p):
    mats = gen.random_chain(n, 6, 3, 0.5, "adversarial", seed=70 + n)
    folder = str(tmp_path / "in")
    refio.write_folder(folder, mats, 3)
    out = str(tmp_path / "matrix")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2")
    r = subprocess.run([MPIEXEC, "-n", str(p), san_bin, folder, "--device", "cpu", "--out", out, "--threads", "2"],
                       capture_output=True, text=True, timeout=300, env=env)
    report = r.stdout + r.stderr
    assert "AddressSanitizer" not in report and "runtime error" not in report, report[-4000:]
    assert r.returncode == 0, report[-4000:]
    want = golden.chain([golden.from_bsr(m) for m in mats], p=p)
    with open(out) as f:
        assert f.read() == golden.to_text(want)
