"""Build an A/B variant of libcwq with extra compile flags (never the product library):

    python scripts/build_variant.py reg -DFG_REG=1      -> rag-cobweb_amd/libcwq_reg.so

Load it in scripts/ab_libs.py next to the product build (one process, interleaved rounds)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobweb_pkg  # noqa: E402

if __name__ == "__main__":
    tag, flags = sys.argv[1], sys.argv[2:]
    B = cobweb_pkg.load().build
    os.environ["CWQ_HIPCC_FLAGS"] = " ".join(flags)
    out = os.path.join(B.HERE, f"libcwq_{tag}.so")
    B.OUT_SAVED = B.OUT
    B.OUT = out
    bdir = os.path.join(B.HERE, f"build_{tag}")
    print(B.build_library(force=True, build_dir=bdir))
