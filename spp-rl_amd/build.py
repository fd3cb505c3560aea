"""Build libspprl.so (gfx950) in-tree with hipcc.  Usage: python spp-rl_amd/build.py [--force]"""
import glob
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "spprl", "libspprl.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-I" + os.path.join(REPO, "include")]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*"))) + [os.path.join(REPO, "include", "spprl.h")]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in sources())


def build(force=False, verbose=True, prof=False, hopper_only=False):
    if prof:  # region-timing variant (never the default library)
        out = os.path.join(HERE, "spprl", "libspprl_prof.so")
        extra = ["-DSPP_ONLY_HOPPER"] if hopper_only else []
        cmd = [HIPCC] + FLAGS + ["-DSPP_PROF"] + extra + ["-o", out, os.path.join(CSRC, "api.hip")]
        subprocess.check_call(cmd)
        return out
    if not force and up_to_date():
        if verbose:
            print("libspprl.so up to date")
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT + ".tmp", os.path.join(CSRC, "api.hip")]
    t0 = time.time()
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    if verbose:
        print("built %s in %.0fs" % (OUT, time.time() - t0))
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, prof="--prof" in sys.argv, hopper_only="--hopper-only" in sys.argv)
