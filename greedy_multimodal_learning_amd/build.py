"""Build libgreedymml_hip.so in-tree with hipcc for gfx950.

`python -m greedy_multimodal_learning_amd.build` (or `__graft_entry__.build()`).
The library links the HIP runtime by SONAME (libamdhip64.so.7); loaded after
`import torch` it binds to the same runtime instance as PyTorch, so PyTorch's
streams and device pointers are valid inside it.
"""
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "libgreedymml_hip.so")
ARCH = os.environ.get("GREEDYMML_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def sources():
    return sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")))


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(PKG, "csrc", "*.h")) + \
        glob.glob(os.path.join(ROOT, "include", "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not needs_build():
        build_testkit()
        return LIB
    objs = []
    bdir = os.path.join(PKG, "csrc", "build")
    os.makedirs(bdir, exist_ok=True)
    cc = hipcc()
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
             "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "csrc")]
    procs = []
    for src in sources():
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        objs.append(obj)
        cmd = [cc] + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + out.decode(errors="replace"))
    tmp = LIB + ".tmp"
    cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout.decode(errors="replace"))
    os.replace(tmp, LIB)
    build_testkit(force=True, verbose=verbose)
    return LIB


TESTKIT_SRC = os.path.join(ROOT, "tests", "native", "testkit.hip")
TESTKIT = os.path.join(ROOT, "tests", "native", "libgm_testkit.so")


def build_testkit(force=False, verbose=False):
    """The test-only kernel library (CU-holding kernel of the residency tests), kept out of the
    product ABI: tests/native/libgm_testkit.so."""
    if not os.path.exists(TESTKIT_SRC):
        return None
    if not force and os.path.exists(TESTKIT) and os.path.getmtime(TESTKIT) >= os.path.getmtime(TESTKIT_SRC):
        return TESTKIT
    cmd = [hipcc(), "-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", TESTKIT_SRC, "-o", TESTKIT]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("testkit build failed:\n" + r.stdout.decode(errors="replace"))
    return TESTKIT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
