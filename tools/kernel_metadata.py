#!/usr/bin/env python3
"""Code-object metadata of the kernels in mythril_amd/libmq.so (VGPR / SGPR / AGPR counts, LDS,
spills), read from the embedded gfx950 code objects: the .hip_fatbin section is cut out of the
ELF, unbundled with clang-offload-bundler and its AMDGPU notes read with llvm-readelf.  rocprof's
kernel-trace `vgpr` field reports allocation granules (x4 here), not this count.
usage: tools/kernel_metadata.py OUT.json"""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")


def section(path, name):
    with open(path, "rb") as f:
        data = f.read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    hdr = lambda i: struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    stroff = hdr(shstrndx)[4]
    for i in range(shnum):
        h = hdr(i)
        nm = data[stroff + h[0]:data.index(b"\0", stroff + h[0])].decode()
        if nm == name:
            return data[h[4]:h[4] + h[5]]
    raise KeyError(name)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    lib = os.environ.get("MQ_LIB") or os.path.join(ROOT, "mythril_amd", "libmq.so")
    fat = section(lib, ".hip_fatbin")
    res = {}
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), fat)]
    with tempfile.TemporaryDirectory() as td:
        for bi, st in enumerate(starts):   # one bundle per translation unit
            end = starts[bi + 1] if bi + 1 < len(starts) else len(fat)
            fb = os.path.join(td, "fat.bin")
            with open(fb, "wb") as f:
                f.write(fat[st:end])
            targets = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--list", "--type=o", f"--input={fb}"],
                                     capture_output=True, text=True, check=True).stdout.split()
            for t in (t for t in targets if "gfx950" in t):
                co = os.path.join(td, "co.o")
                subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                                f"--targets={t}", f"--output={co}"], check=True)
                notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True, text=True).stdout
                for blk in notes.split("  - .agpr_count")[1:]:
                    blk = ".agpr_count" + blk
                    kv = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
                    if "name" in kv and not kv["name"].endswith(".kd"):
                        res[kv["name"]] = {k: (int(v) if v.isdigit() else v) for k, v in kv.items()
                                           if k in ("vgpr_count", "sgpr_count", "agpr_count", "vgpr_spill_count",
                                                    "sgpr_spill_count", "group_segment_fixed_size",
                                                    "private_segment_fixed_size", "max_flat_workgroup_size", "wavefront_size")}
    for k, v in res.items():
        v["waves_per_simd_by_vgpr"] = 512 // max(8, -(-v.get("vgpr_count", 1) // 8) * 8)
    doc = {"source": "code-object metadata (.hip_fatbin of mythril_amd/libmq.so, gfx950), tools/kernel_metadata.py",
           "kernels": res}
    text = json.dumps(doc, indent=1, sort_keys=True)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
