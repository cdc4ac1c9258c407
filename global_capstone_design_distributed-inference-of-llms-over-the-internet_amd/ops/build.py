"""In-tree build of the gfx950 HIP kernels into one torch custom-op library.

No hipify, no torch JIT cache: every ``csrc/*.hip`` file is compiled by ``hipcc
--offload-arch=gfx950`` and linked with ``csrc/bindings.cpp`` (TORCH_LIBRARY
registrations) into ``ops/_mpamd_kernels.so`` next to this file, so the built
library travels with the repository snapshot to the GPU box.

Usage: ``python -m src.ops.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB_NAME = "_mpamd_kernels.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
ARCH = os.environ.get("MPAMD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# ablation builds: extra device-compile flags (e.g. "-DMP_RW_WAVES=8") go to their own object
# directory and library name (``--out``), never over the default library
EXTRA = os.environ.get("MPAMD_HIPCC_EXTRA", "").split()


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    return inc, lib


def _sources():
    hip = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    return [os.path.join(CSRC, f) for f in hip], os.path.join(CSRC, "bindings.cpp")


def _digest(paths, extra=""):
    h = hashlib.sha256(extra.encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(force: bool = False, jobs: int = 0, verbose: bool = False, out: str = None) -> str:
    """Compile (if stale) and return the path of the kernel library."""
    hips, binding = _sources()
    headers = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".h")]
    xtag = " ".join(EXTRA)
    if xtag and not out:
        raise SystemExit("MPAMD_HIPCC_EXTRA builds need --out (the default library stays the default build)")
    LIB_PATH = os.path.abspath(out) if out else globals()["LIB_PATH"]
    BUILD = globals()["BUILD"] + ("_" + hashlib.sha256(xtag.encode()).hexdigest()[:8] if xtag else "")
    tag = _digest(hips + [binding] + headers, extra=ARCH + HIPCC + xtag)
    stamp = os.path.join(BUILD, "stamp")
    if not force and os.path.exists(LIB_PATH) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == tag:
                return LIB_PATH
    os.makedirs(BUILD, exist_ok=True)
    inc, libdir = _torch_paths()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I" + CSRC] + EXTRA
    objs = []
    cmds = []
    hdr_tag = _digest(headers, extra=ARCH + HIPCC + xtag)

    def stale(src, obj):
        # per-object stamp: the source + every csrc header (a kernel edit rebuilds one object)
        t = _digest([src], extra=hdr_tag)
        st = obj + ".stamp"
        if force or not os.path.exists(obj) or not os.path.exists(st) or open(st).read().strip() != t:
            return t
        return None

    for src in hips:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        t = stale(src, obj)
        if t is not None:
            cmds.append(([HIPCC] + common + ["-c", src, "-o", obj], obj, t))
    bobj = os.path.join(BUILD, "bindings.o")
    objs.append(bobj)
    t = stale(binding, bobj)
    if t is not None:
        # host-only translation unit (torch headers): plain C++, no device pass
        cmds.append(([HIPCC, "-x", "c++", "-O2", "-fPIC", "-std=c++17", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                      "-I/opt/rocm/include"] + [f"-I{p}" for p in inc] + ["-c", binding, "-o", bobj], bobj, t))

    def run_one(job):
        cmd, obj, t = job
        out = _run(cmd)
        with open(obj + ".stamp", "w") as f:
            f.write(t)
        return out

    jobs = jobs or max(1, min(len(cmds), os.cpu_count() or 4, 8))
    with cf.ThreadPoolExecutor(jobs) as ex:
        for out in ex.map(run_one, cmds):
            if verbose and out.strip():
                print(out)
    tmp = LIB_PATH + ".tmp"
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs
         + ["-o", tmp, f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip",
            "-ltorch_hip"])
    os.replace(tmp, LIB_PATH)
    with open(stamp, "w") as f:
        f.write(tag)
    return LIB_PATH


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--out", default=None, help="library path of an ablation build (MPAMD_HIPCC_EXTRA)")
    a = ap.parse_args(argv)
    path = build(force=a.force, jobs=a.jobs, verbose=a.verbose, out=a.out)
    print(path)


if __name__ == "__main__":
    sys.exit(main())
