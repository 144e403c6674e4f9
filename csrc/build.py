#!/usr/bin/env python3
"""Build the native libraries in-tree (no JIT cache, no hipify).

* ``libfps_kernels.so`` — every ``csrc/kernels/*.hip`` compiled by
  ``hipcc --offload-arch=gfx950`` into one shared object exposing a C ABI
  (``fps_*`` launchers taking device pointers + a ``hipStream_t``).  Loaded
  with ctypes by ``flink_parameter_server_1_amd.ops`` *after* torch, so the
  HIP runtime torch already loaded (same SONAME ``libamdhip64.so.7``) serves it.
* ``libfps_host.so`` — ``csrc/host/*.cpp`` (C++17, g++): the host runtime
  pieces (synthetic data generators, ``id;value`` text codec, sharded
  hash store, ...).

Usage: ``python csrc/build.py [--force] [--only kernels|host]``.
Outputs land in ``flink_parameter_server_1_amd/_lib/``.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "flink_parameter_server_1_amd", "_lib")
ARCH = os.environ.get("FPS_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm not installed?)")


def _digest(paths, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()[:16]


def _up_to_date(target: str, digest: str) -> bool:
    stamp = target + ".stamp"
    return os.path.exists(target) and os.path.exists(stamp) and open(stamp).read().strip() == digest


def _write_stamp(target: str, digest: str):
    with open(target + ".stamp", "w") as f:
        f.write(digest + "\n")


#: per-source code-generation flags.  score_bf16.hip: MFMA accumulators in VGPRs (the
#: default form kept them in AGPRs, and every 32 x 32 block's filter first copied its 16
#: scores out with v_accvgpr_read: 16 of the ~30 vector instructions per 4 MFMAs)
PER_FILE_FLAGS = {"score_bf16.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def build_kernels(force: bool = False, verbose: bool = True, variant: str = None, defines=(), rev: str = None) -> str:
    """One object per source (compiled in parallel, each with its own digest stamp:
    a change rebuilds only its file), linked into one shared object.  ``variant`` +
    ``defines`` (``NAME=VALUE``): an A/B build of the library with extra macros, into
    ``_lib/ab/<variant>/libfps_kernels.so`` (select it with ``FPS_KERNELS_SO``);
    ``rev``: the variant's kernel sources as of that git revision (an A/B against
    earlier code)."""
    from concurrent.futures import ThreadPoolExecutor

    out = OUT if variant is None else os.path.join(OUT, "ab", variant)
    os.makedirs(out, exist_ok=True)
    objdir = os.path.join(out, "obj")
    os.makedirs(objdir, exist_ok=True)
    kdir = os.path.join(CSRC, "kernels")
    if rev is not None:
        if variant is None:
            raise ValueError("rev needs a variant (the main library is always built from the working tree)")
        kdir = os.path.join(out, "src")
        os.makedirs(kdir, exist_ok=True)
        root = os.path.dirname(CSRC)
        names = subprocess.run(["git", "-C", root, "ls-tree", "--name-only", rev, "csrc/kernels/"], check=True,
                               capture_output=True, text=True).stdout.split()
        for nm in names:
            body = subprocess.run(["git", "-C", root, "show", f"{rev}:{nm}"], check=True, capture_output=True).stdout
            with open(os.path.join(kdir, os.path.basename(nm)), "wb") as f:
                f.write(body)
    srcs = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(kdir, "*.h")))
    target = os.path.join(out, "libfps_kernels.so")
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-munsafe-fp-atomics", "-Wno-unused-result",
             "-I", kdir] + [f"-D{d}" for d in defines]

    def obj(src):
        extra = PER_FILE_FLAGS.get(os.path.basename(src), [])
        o = os.path.join(objdir, os.path.basename(src) + ".o")
        d = _digest([src] + hdrs, " ".join(flags + extra))
        if force or not _up_to_date(o, d):
            cmd = [_hipcc()] + flags + extra + ["-c", src, "-o", o + ".tmp"]
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
            os.replace(o + ".tmp", o)
            _write_stamp(o, d)
        return o

    workers = int(os.environ.get("MAX_JOBS", "8"))
    with ThreadPoolExecutor(max_workers=max(1, min(workers, 16))) as ex:
        objs = list(ex.map(obj, srcs))
    digest = _digest(objs, "link")
    if not force and _up_to_date(target, digest):
        return target
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", target + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(target + ".tmp", target)
    _write_stamp(target, digest)
    return target


def build_host(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    target = os.path.join(OUT, "libfps_host.so")
    if not srcs:
        return ""
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-march=x86-64-v2", "-I",
             os.path.join(CSRC, "host")]
    digest = _digest(srcs + hdrs, cxx + " ".join(flags))
    if not force and _up_to_date(target, digest):
        return target
    cmd = [cxx] + flags + srcs + ["-o", target + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(target + ".tmp", target)
    _write_stamp(target, digest)
    return target


def asan_selftest(workdir: str = "/tmp", verbose: bool = True) -> int:
    """Build the host runtime + ``csrc/tests/host_selftest.cpp`` with ASan/UBSan
    (host code only -- GPU sanitizers are not available) and run it; returns its
    exit code."""
    cxx = os.environ.get("CXX", "g++")
    exe = os.path.join(workdir, "fps_host_selftest_asan")
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp"))) + [os.path.join(CSRC, "tests", "host_selftest.cpp")]
    cmd = [cxx, "-O1", "-g", "-std=c++17", "-pthread", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", "-I", os.path.join(CSRC, "host")] + srcs + ["-o", exe]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    return subprocess.run([exe, workdir], env=env).returncode


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["kernels", "host"])
    ap.add_argument("--variant", default=None, help="A/B build name (with -D NAME=VALUE macros)")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--rev", default=None, help="--variant: kernel sources as of this git revision")
    ap.add_argument("--asan-selftest", action="store_true",
                    help="build + run the host runtime self-test under ASan/UBSan, then exit")
    a = ap.parse_args(argv)
    if a.asan_selftest:
        return asan_selftest()
    if a.variant:
        print(build_kernels(a.force, variant=a.variant, defines=a.defines, rev=a.rev))
        return 0
    if a.only in (None, "kernels"):
        print(build_kernels(a.force))
    if a.only in (None, "host"):
        print(build_host(a.force))


if __name__ == "__main__":
    sys.exit(main())
