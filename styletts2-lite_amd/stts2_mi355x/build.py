"""Build libstts2.so (the C-ABI library of include/stts2.h) in-tree with hipcc for gfx950.

    python -m stts2_mi355x.build          (or __graft_entry__.build())

Sources: styletts2-lite_amd/csrc/*.hip, *.cpp.  Objects go to styletts2-lite_amd/build/,
the shared library next to this file so it travels to the GPU box with the snapshot.
Rebuilds only when a source or header is newer than the library.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(os.path.dirname(ROOT), "include")
OBJ = os.path.join(ROOT, "build")
LIB = os.path.join(PKG, "libstts2.so")
ARCH = os.environ.get("STTS_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-Wall",
         "-Wno-unused-function", f"-I{INCLUDE}"]


def _hipcc():
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found: the HIP library cannot be built")
    return h


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    hipcc = _hipcc()
    jobs, objs = [], []
    # (incremental: an object newer than its source and every header is reused)
    hdr_t = max([os.path.getmtime(h) for h in glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))]
                + [os.path.getmtime(__file__)])
    for src in sources():
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(src), hdr_t):
            continue
        cmd = [hipcc, *FLAGS, "-x", "hip", "-c", src, "-o", obj]
        jobs.append((src, obj, cmd))

    def run(job):
        src, obj, cmd = job
        r = subprocess.run(cmd, capture_output=True, text=True)
        return src, r

    n = min(max(len(jobs), 1), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=max(1, n)) as ex:
        for src, r in ex.map(run, jobs):
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
            if verbose and (r.stdout or r.stderr):
                print(r.stdout, r.stderr, file=sys.stderr)
    tmp = LIB + ".tmp"
    cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
