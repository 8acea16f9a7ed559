"""Build the gfx950 HIP library in-tree: pgmpy_amd/lib/libpgmhip.so.

    python -m pgmpy_amd.build        (also run by __graft_entry__.build())

hipcc cross-compiles for gfx950 without a GPU, so this works in the build
container; the .so travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "pgmhip.hip")
SRC_DQ = os.path.join(HERE, "csrc", "pgmdq.cpp")  # direct AQL dispatch (host code, HSA runtime)
SRC_PM = os.path.join(HERE, "csrc", "pgmpm.cpp")  # plan-specialised batched-BP steps (host code, hipRTC)
SRC_HOST = os.path.join(HERE, "csrc", "pgmhost.cpp")  # DataFrame ingestion helpers (host threads only)
INC = os.path.join(ROOT, "include")
OUT = os.path.join(HERE, "lib", "libpgmhip.so")
ARCH = "gfx950"


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def build(force=False, verbose=True, out=OUT, defines=()):
    """defines: extra -D macros (tools only, e.g. PGM_ROWS_TIMELINE into lib/libpgmhip_timeline.so)."""
    deps = [SRC, SRC_DQ, SRC_PM, SRC_HOST, os.path.join(HERE, "csrc", "pgm_internal.h"), os.path.join(INC, "pgmhip.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-I", INC] + [f"-D{d}" for d in defines] + ["-o", tmp, SRC, SRC_DQ, SRC_PM, SRC_HOST, "-lhiprtc", "-lhsa-runtime64"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


TIMELINE_OUT = os.path.join(HERE, "lib", "libpgmhip_timeline.so")

if __name__ == "__main__":
    if "--timeline" in sys.argv:  # per-wave timestamps in the affine row kernel (tools/rows_timeline.py)
        print(build(force=True, out=TIMELINE_OUT, defines=("PGM_ROWS_TIMELINE",)))
    else:
        print(build(force="--force" in sys.argv))
