#!/usr/bin/env python3
"""Register / scratch budget of every kernel in the built HIP library (build check).

Reads the gfx950 code objects embedded in pbrt-v2-spectral_amd/lib/libpbrtgpu.so (the
.hip_fatbin section: one clang offload bundle per translation unit), takes each kernel's
AMDGPU metadata (llvm-readelf --notes) and fails if a kernel exceeds the spill budget:

  * VGPR spills  <= MAX_VGPR_SPILL   (registers spilled to scratch)
  * scratch      <= MAX_SCRATCH      (private segment bytes per lane)

Why a budget: the first DirectLighting shade step, forced to 3 waves/SIMD, ran with 1,393
spilled VGPRs and 386 spilled SGPRs (2,164 B of scratch per lane) and gave run-to-run
different radiance, while the same source replayed on the CPU under MSan / ASan / UBSan
(tools/hostsan) reads nothing uninitialised or out of bounds and matches the oracle bit for bit
(DESIGN.md §4.4).  No product kernel is allowed back into that regime.

usage: kernel_budget.py [LIB] [--table]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAX_VGPR_SPILL = 160
MAX_SCRATCH = 1024
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    """gfx950 ELF code objects of every offload bundle in the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, lib, os.devnull],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    out = []
    for m in re.finditer(re.escape(MAGIC), data):
        base = m.start()
        p = base + len(MAGIC)
        (n,) = struct.unpack_from("<Q", data, p)
        p += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tlen].decode()
            p += tlen
            if "gfx950" in triple and size:
                out.append(data[base + off:base + off + size])
    return out


def kernels(elf_bytes):
    """[(name, vgpr, agpr, vgpr_spill, sgpr_spill, scratch)] from the code object's metadata note."""
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(elf_bytes)
        f.flush()
        txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], check=True,
                             capture_output=True, text=True).stdout
    res = []
    # one YAML mapping per kernel under amdhsa.kernels
    for block in re.split(r"\n\s+- \.", txt):
        name = re.search(r"\.name:\s+(\S+)", block) or re.search(r"^name:\s+(\S+)", block, re.M)
        if not name or ".vgpr_count" not in block:
            continue
        def num(key):
            m = re.search(r"\." + key + r":\s+(\d+)", block)
            return int(m.group(1)) if m else 0
        res.append((name.group(1), num("vgpr_count"), num("agpr_count"), num("vgpr_spill_count"),
                    num("sgpr_spill_count"), num("private_segment_fixed_size")))
    return res


def demangle(names):
    try:
        out = subprocess.run([os.path.join(LLVM, "llvm-cxxfilt")], input="\n".join(names), check=True,
                             capture_output=True, text=True).stdout.split("\n")
        return [re.sub(r"\(.*", "", o) for o in out[:len(names)]]
    except (OSError, subprocess.CalledProcessError):
        return names


def main(argv):
    lib = next((a for a in argv if not a.startswith("--")),
               os.path.join(ROOT, "pbrt-v2-spectral_amd", "lib", "libpbrtgpu.so"))
    rows = {}
    for co in code_objects(lib):
        for k in kernels(co):
            rows[k[0]] = k
    if not rows:
        print("kernel_budget: no gfx950 kernels found in", lib)
        return 1
    names = sorted(rows)
    pretty = dict(zip(names, demangle(names)))
    bad = []
    if "--table" in argv:
        print("%-60s %5s %5s %6s %6s %7s" % ("kernel", "vgpr", "agpr", "vspill", "sspill", "scratch"))
    for n in names:
        _, v, a, vs, ss, sc = rows[n]
        if "--table" in argv and "rocprim" not in n and "hipcub" not in n:
            print("%-60s %5d %5d %6d %6d %7d" % (pretty[n][:60], v, a, vs, ss, sc))
        if vs > MAX_VGPR_SPILL or sc > MAX_SCRATCH:
            bad.append("%s: %d VGPRs spilled, %d B scratch per lane" % (pretty[n], vs, sc))
    if bad:
        print("kernel_budget: over budget (VGPR spills <= %d, scratch <= %d B/lane):" % (MAX_VGPR_SPILL, MAX_SCRATCH))
        for b in bad:
            print("  " + b)
        return 1
    print("kernel_budget: %d kernels within budget (VGPR spills <= %d, scratch <= %d B/lane)"
          % (len(names), MAX_VGPR_SPILL, MAX_SCRATCH))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
