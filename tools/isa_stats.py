"""Per-kernel ISA statistics of one kernel file (device assembly for gfx950):
VGPRs / SGPRs / spills / LDS, and counts of s_waitcnt, barriers and buffer
memory instructions -- to check that a source change kept hipcc's schedule of
a hot kernel (e.g. the pipelined bitmap kernels' vmcnt waits) before spending
a GPU run on it.

    python tools/isa_stats.py csr_spgemm_bitmap.hip [kernel-name-regex] [-D...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "sparse-matrix-multiplication-using-openmp-mpi-and-cuda_amd", "csrc", "kernels")


def isa(src: str, defines) -> str:
    out = os.path.join(tempfile.mkdtemp(prefix="isa_"), "k.s")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
           "--cuda-device-only", "-S", *defines, src, "-o", out]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def main() -> None:
    args = [a for a in sys.argv[1:] if not a.startswith("-D")]
    defines = [a for a in sys.argv[1:] if a.startswith("-D")]
    src = args[0] if os.path.exists(args[0]) else os.path.join(KDIR, args[0])
    pat = re.compile(args[1] if len(args) > 1 else ".")
    text = isa(src, defines)
    # function bodies: "<name>: ; @<name>" at column 0 to its .Lfunc_endN label
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end\d+:", text, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if not pat.search(name):
            continue
        meta = {}
        for key in ("num_vgpr", "num_agpr", "numbered_sgpr", "private_seg_size"):
            mm = re.search(r"\.set " + re.escape(name) + r"\." + key + r", (\d+)", text)
            meta[key] = int(mm.group(1)) if mm else None
        mm = re.search(r"\.amdhsa_group_segment_fixed_size (\d+)", text[text.find(".amdhsa_kernel " + name):])
        meta["lds"] = int(mm.group(1)) if mm else None
        counts = {
            "insts": len(re.findall(r"^\s+[a-z_]", body, re.M)),
            "s_waitcnt": len(re.findall(r"\bs_waitcnt\b", body)),
            "vmcnt(0)": len(re.findall(r"vmcnt\(0\)", body)),
            "barrier": len(re.findall(r"\bs_barrier\b", body)),
            "buffer_load": len(re.findall(r"\bbuffer_load_", body)),
            "buffer_store": len(re.findall(r"\bbuffer_store_", body)),
            "global_load": len(re.findall(r"\bglobal_load_", body)),
            "scratch_ops": len(re.findall(r"\bscratch_(load|store)_", body)),
        }
        print(name[:110])
        print("   ", meta)
        print("   ", counts)


if __name__ == "__main__":
    main()
