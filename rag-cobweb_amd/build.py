"""Build libcwq.so for gfx950 in-tree (hipcc cross-compiles without a GPU).

    python -c "import cobweb_pkg; cobweb_pkg.load().build.build_library()"

The sources are compiled in parallel (one hipcc per file) and linked.  The build id
(sha256 of the sources, the public header, the flags and the target) is compiled into
the library as `cwq_build_id()`: `build_library()` rebuilds whenever the id of the
library on disk differs from the sources' id, and `_lib.lib()` refuses to load a
library whose id does not match the sources next to it, so a stale binary can never
be the one that runs.
"""
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
HEADER = os.path.join(HERE, "..", "include", "cobweb_query.h")
SOURCES = ["cwq_kernels.hip", "cwq_api.hip", "cwq_fit.hip", "cwq_mfma.hip", "cwq_whiten.hip", "cwq_stream.hip", "cwq_fitdev.hip", "cwq_group.hip", "cwq_prune.hip"]
OUT = os.path.join(HERE, "libcwq.so")
ARCH = os.environ.get("CWQ_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC",
         # keep one fp32 op per element: SLP packing to v_pk_* needs SGPR-pair shuffles
         # in the scan kernel's inner loop
         "-fno-slp-vectorize"]


def source_id(extra=()):
    """Build id of the current sources (what cwq_build_id() of a fresh build returns)."""
    h = hashlib.sha256()
    deps = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    for f in deps:
        h.update(f.encode())
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(HEADER, "rb") as fh:
        h.update(fh.read())
    h.update(" ".join([ARCH, *FLAGS, *extra]).encode())
    return h.hexdigest()[:16]


def library_id(path=OUT):
    """The build id compiled into the library at `path` (None if missing or unstamped).
    Read from the file, not through dlopen: a process that already loaded an older
    library at this path would get that one back from the loader."""
    if not os.path.exists(path):
        return None
    import re
    with open(path, "rb") as fh:
        m = re.search(rb"CWQ_BUILD_ID=([0-9a-f]{16})\0", fh.read())
    return m.group(1).decode() if m else None


def build_library(force=False, verbose=False, jobs=None, build_dir=None):
    extra = os.environ.get("CWQ_HIPCC_FLAGS", "").split()   # A/B experiments only
    sid = source_id(extra)
    out = OUT
    if not force and library_id(out) == sid:
        return out
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    bdir = build_dir or os.path.join(HERE, "build")
    os.makedirs(bdir, exist_ok=True)
    common = [hipcc, f"--offload-arch={ARCH}", *FLAGS, *extra, f'-DCWQ_BUILD_ID="{sid}"']

    def compile_one(src):
        obj = os.path.join(bdir, src.replace(".hip", ".o"))
        cmd = [*common, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    n = jobs or min(len(SOURCES), max(1, (os.cpu_count() or 2) // 2), 8)
    with cf.ThreadPoolExecutor(n) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
