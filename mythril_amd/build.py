"""Build libmq.so (gfx950) in-tree with hipcc.  ``python -m mythril_amd.build``.

The kernels are compiled with ``-mllvm -simplifycfg-sink-common=false``: SimplifyCFG's
common-code sinking merges the per-stack-slot handler bodies into one store with a PHI'd
address, which turns the statically indexed register stack into a dynamically indexed array
and demotes it to scratch memory (observed: 260 B/lane of scratch, ~1800 scratch ops).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libmq.so")
OBJDIR = os.path.join(HERE, "csrc", "_obj")
SOURCES = ["mq_api.cpp", "host_keccak.cpp", "tape_compiler.cpp", "qs_kernels.hip", "keccak.hip", "qsa.hip", "fc.hip", "cw.hip"]
HEADERS = ["host_keccak.h", "gprog.h", "bvops.h", "qs_launch.h", "tape_compiler.h", "qsa_table.h", "qsa_gen.inc"]
ARCH = os.environ.get("MQ_OFFLOAD_ARCH", "gfx950")


def _rocm() -> str:
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc() -> str:
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc") or ""):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: libmq.so needs the ROCm toolchain")


def _flags(src: str):
    f = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unknown-pragmas", "-Wno-unused-variable"]
    if src.endswith(".hip"):
        f += ["-mllvm", "-simplifycfg-sink-common=false"]
    return f


def _stale(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(HERE, "..", "include", "mq.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _generated_current() -> bool:
    """qsa_gen.inc / qsa_table.h (generated, not tracked) carry the sha256 of gen_qsa.py."""
    import hashlib
    with open(os.path.join(CSRC, "gen_qsa.py"), "rb") as f:
        # (the diagnostic profile build, QSA_PROF=1, stamps differently: switching regenerates)
        stamp = hashlib.sha256(f.read() + (b"PROF" if os.environ.get("QSA_PROF") == "1" else b"")).hexdigest()[:16]
    for name in ("qsa_gen.inc", "qsa_table.h"):
        path = os.path.join(CSRC, name)
        if not os.path.exists(path):
            return False
        with open(path) as f:
            if f"(source {stamp})" not in f.readline():
                return False
    return True


def build_lowerwalk(force: bool = False) -> str:
    """The drop-in lowering's term walk (csrc/lowerwalk.cpp), a CPython extension built with the
    host compiler next to this file (lower.py imports it)."""
    import sysconfig
    src = os.path.join(CSRC, "lowerwalk.cpp")
    out = os.path.join(HERE, "_lowerwalk" + sysconfig.get_config_var("EXT_SUFFIX"))
    if force or not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        cmd = [os.environ.get("CXX", "g++"), "-O2", "-shared", "-fPIC", "-std=c++17", "-Wall", "-pthread",
               f"-I{sysconfig.get_paths()['include']}", src, "-o", out]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode:
            sys.stderr.write(res.stderr)
            raise RuntimeError("lowerwalk build failed")
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    # the host-only lowering walk first: it needs no ROCm toolchain, and lower.py uses it whether
    # or not the HIP build below succeeds
    build_lowerwalk(force)
    hipcc = _hipcc()
    if force or not _generated_current():
        subprocess.check_call([sys.executable, os.path.join(CSRC, "gen_qsa.py")])
    os.makedirs(OBJDIR, exist_ok=True)
    jobs = []
    objs = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJDIR, s + ".o")
        objs.append(obj)
        if force or _stale(obj, src):
            jobs.append([hipcc, *_flags(s), "-c", src, "-o", obj])
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for cmd, res in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
            if verbose or res.returncode:
                sys.stderr.write(res.stderr)
            if res.returncode:
                raise RuntimeError(f"compile failed: {' '.join(cmd)}")
    if force or jobs or not os.path.exists(OUT):
        # librccl: the in-library MIN all-reduce of a multi-device context (mq_ctx_create n_dev > 1)
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, *objs,
               f"-L{_rocm()}/lib", "-lrccl", f"-Wl,-rpath,{_rocm()}/lib", "-lpthread"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode:
            sys.stderr.write(res.stderr)
            raise RuntimeError("link failed")
    tool = os.path.join(HERE, "valu_peak")
    tsrc = os.path.join(CSRC, "valu_peak.hip")
    if force or not os.path.exists(tool) or os.path.getmtime(tool) < os.path.getmtime(tsrc):
        res = subprocess.run([hipcc, "-O3", f"--offload-arch={ARCH}", tsrc, "-o", tool], capture_output=True, text=True)
        if res.returncode:
            sys.stderr.write(res.stderr)
            raise RuntimeError("valu_peak build failed")
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
