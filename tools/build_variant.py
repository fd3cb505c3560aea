"""Build an A/B variant of libspprl.so with extra compile definitions (never the default library).

    python tools/build_variant.py TAG [--only=ks_dw.hip,...] -DNAME=VALUE ...   ->  spp-rl_amd/spprl/libspprl_TAG.so

--only compiles just the named units with the definitions and links the default build's objects
for the rest.

Objects go to spp-rl_amd/build_TAG/.  Select the variant at run time with SPPRL_LIB=<path>.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "spp-rl_amd"))
import build as B  # noqa: E402


def main():
    tag = sys.argv[1]
    only = [a.split("=", 1)[1].split(",") for a in sys.argv[2:] if a.startswith("--only=")]
    only = only[0] if only else None
    defs = [a for a in sys.argv[2:] if not a.startswith("--only=")]
    objdir = os.path.join(B.HERE, "build_" + tag)
    os.makedirs(objdir, exist_ok=True)
    out = os.path.join(B.HERE, "spprl", "libspprl_%s.so" % tag)

    def comp(src):
        if only is not None and os.path.basename(src) not in only:
            return B._obj(src)
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        subprocess.check_call([B.HIPCC] + B.FLAGS + defs + ["-c", "-o", obj, src])
        print("  ", os.path.basename(src), flush=True)
        return obj

    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, B.units()))
    subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    print("built", out)


if __name__ == "__main__":
    main()
