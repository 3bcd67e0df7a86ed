"""Build libcwq.so for gfx950 in-tree (hipcc cross-compiles without a GPU).

    python -c "import cobweb_pkg; cobweb_pkg.load().build.build_library()"
"""
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["cwq_kernels.hip", "cwq_api.hip", "cwq_fit.hip", "cwq_mfma.hip", "cwq_whiten.hip"]
OUT = os.path.join(HERE, "libcwq.so")
ARCH = os.environ.get("CWQ_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared",
         # keep one fp32 op per element: SLP packing to v_pk_* needs SGPR-pair shuffles
         # in the scan kernel's inner loop
         "-fno-slp-vectorize"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(HERE, "..", "include", "cobweb_query.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_library(force=False, verbose=False):
    if not force and not _stale():
        return OUT
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    extra = os.environ.get("CWQ_HIPCC_FLAGS", "").split()   # A/B experiments only
    cmd = [hipcc, f"--offload-arch={ARCH}", *FLAGS, *extra, *[os.path.join(CSRC, s) for s in SOURCES], "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
