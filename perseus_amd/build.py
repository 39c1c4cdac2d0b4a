"""Build libperseus_amd.so in-tree with hipcc for gfx950.

    python -m perseus_amd.build [--force]

Each csrc/*.hip (hipcc) and csrc/*.cpp (host-only: g++) is compiled to an object in
parallel (perseus_amd/lib/obj/, kept for
incremental rebuilds: only sources newer than their object, or including a newer
header, are recompiled), then linked into perseus_amd/lib/libperseus_amd.so
(git-ignored, shipped to the GPU box with the snapshot).
"""

from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libperseus_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-mllvm", "-disable-promote-alloca-to-lds", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-result"]


# measurement build: the timing-only kernel variants (wrong results by construction) compiled in
# (csrc/common.h PA_TIMING_VARIANTS); the release library refuses their ids
if os.environ.get("PERSEUS_AMD_TIMING_VARIANTS") == "1":
    FLAGS.append("-DPA_TIMING_VARIANTS=1")

OBJDIR = os.path.join(LIBDIR, "obj")  # incremental build state (git- and gpurun-ignored)
# per-source extra hipcc flags (file name -> list); part of the flags digest
EXTRA: dict = {}


CXX = os.environ.get("CXX_HOST", "g++")
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", f"-I{os.path.join(ROOT, 'include')}"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _includes(path, seen=None):
    """Local headers `path` includes, transitively."""
    seen = set() if seen is None else seen
    with open(path) as fh:
        for name in _INC.findall(fh.read()):
            h = os.path.normpath(os.path.join(os.path.dirname(path), name))
            if not os.path.exists(h):
                h = os.path.join(ROOT, "include", name)
            if os.path.exists(h) and h not in seen:
                seen.add(h)
                _includes(h, seen)
    return seen


STAMP = os.path.join(OBJDIR, "flags.stamp")
# the same digest beside the library (git-ignored, travels with it to the GPU box, where obj/ does
# not): a fresh tree with an up-to-date .so needs no rebuild
LIB_STAMP = LIB + ".flags"


def _flags_digest() -> str:
    """Compilers, flags and arch the objects are built with: a change invalidates every
    object (mtimes alone would link stale objects built with the old flags)."""
    import hashlib

    # the include path names this checkout's location: digest it relative to the tree, so the
    # library built here counts as up to date in a copy of the tree elsewhere (the GPU box)
    host = [f.replace(ROOT, "<root>") for f in HOST_FLAGS]
    return hashlib.sha256(repr((HIPCC, FLAGS, ARCH, CXX, host, sorted(EXTRA.items()))).encode()).hexdigest()


def _stamp_ok() -> bool:
    try:
        with open(STAMP) as fh:
            return fh.read().strip() == _flags_digest()
    except OSError:
        return False


def _obj(src: str) -> str:
    return os.path.join(OBJDIR, os.path.splitext(os.path.basename(src))[0] + ".o")


def _stale(src: str) -> bool:
    o = _obj(src)
    if not os.path.exists(o):
        return True
    t = os.path.getmtime(o)
    return any(os.path.getmtime(p) > t for p in [src, *_includes(src)])


def _lib_stamp_ok() -> bool:
    try:
        with open(LIB_STAMP) as fh:
            return fh.read().strip() == _flags_digest()
    except OSError:
        return False


def up_to_date() -> bool:
    if not os.path.exists(LIB) or not (_stamp_ok() or _lib_stamp_ok()):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in _deps())


def _compile(src: str) -> str:
    obj = _obj(src)
    if src.endswith(".cpp"):
        cmd = [CXX, *HOST_FLAGS, "-c", src, "-o", obj + ".tmp"]
    else:
        cmd = [HIPCC, *FLAGS, *EXTRA.get(os.path.basename(src), []), "-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd[0]} failed for {src}:\n{r.stdout}\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    if not force and up_to_date():
        return LIB
    srcs = sources()
    if not _stamp_ok():
        force = True
        if os.path.exists(STAMP):
            os.remove(STAMP)
    todo = [s for s in srcs if force or _stale(s)]
    # the fully unrolled conv kernels take minutes: start the slowest (largest) first
    todo.sort(key=lambda p: -os.path.getsize(p) - sum(os.path.getsize(h) for h in _includes(p)))
    with ThreadPoolExecutor(max_workers=min(8, max(1, len(todo)))) as ex:
        list(ex.map(_compile, todo))
    objs = [_obj(s) for s in srcs]
    tmp = LIB + ".tmp"
    # -z defs: an unresolved symbol (e.g. a kernel stub the host pass dropped) fails the link
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,-z,defs", "-o", tmp, *objs, "-lz"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    for st in (STAMP, LIB_STAMP):
        with open(st, "w") as fh:
            fh.write(_flags_digest() + "\n")
    if verbose:
        print(f"built {LIB} ({len(todo)} of {len(srcs)} objects recompiled)")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
