"""Build the gfx950 HIP library (libniidmix.so) in-tree.

    python -m niidmix.build            # from non-iid-topology-simulator_amd/

The library is compiled with hipcc for gfx950 only, -ffp-contract=off (the exact kernel needs
separate mul/add roundings; fast kernels use explicit fmaf).  The .so lands next to this file so it
travels with the repository snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                       # non-iid-topology-simulator_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(PKG_DIR, "libniidmix.so")
SOURCES = [os.path.join(CSRC, "niidmix.hip")]
HEADERS = [os.path.join(REPO, "include", "niidmix.h")]

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-mcode-object-version=5", "-Wall"]


def _hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the niidmix HIP library cannot be built")


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in SOURCES + HEADERS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return LIB
    cmd = [_hipcc()] + HIPCC_FLAGS + ["-I", os.path.join(REPO, "include"), "-o", LIB + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    _check_undefined(LIB + ".tmp")
    os.replace(LIB + ".tmp", LIB)
    return LIB


def _check_undefined(path):
    """Fail the build when a kernel's host stub is missing: hipcc can leave a template kernel's
    launch stub undefined (a construct the host pass rejects without a diagnostic), and the
    library then only fails at dlopen on the GPU box."""
    nm = shutil.which("nm")
    if nm is None:
        return
    out = subprocess.run([nm, "-D", "--undefined-only", path], capture_output=True, text=True,
                         check=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if "_GLOBAL__N_" in ln]
    if bad:
        os.remove(path)
        raise RuntimeError("libniidmix: undefined kernel symbols: " + ", ".join(bad[:4]))


if __name__ == "__main__":
    build(force="--force" in sys.argv)
