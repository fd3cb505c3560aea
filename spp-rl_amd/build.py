"""Build libspprl.so (gfx950) in-tree with hipcc.  Usage: python spp-rl_amd/build.py [--force]

The library is one api.hip translation unit (C-ABI, non-template kernels) plus one
translation unit per phase-kernel config family (csrc/ks_*.hip); they compile in
parallel into build/ and link into spp-rl_amd/spprl/libspprl.so.
"""
import glob
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "spprl", "libspprl.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(REPO, "include")]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*"))) + [os.path.join(REPO, "include", "spprl.h")]


def units():
    return [os.path.join(CSRC, "api.hip")] + sorted(glob.glob(os.path.join(CSRC, "ks_*.hip")))


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in sources())


KSET_DEPS = ("kset.h", "sac.hip", "sac_team.h", "ddpg.hip", "sac_kernels.h", "mlp.h", "common.h")


def _obj(src):
    return os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))


def _stale(src):
    """api.hip depends on every csrc file; ks_*.hip only on the phase-kernel headers."""
    obj = _obj(src)
    if not os.path.exists(obj):
        return True
    if os.path.basename(src) == "ks_dw.hip":
        deps = [src] + [os.path.join(CSRC, d) for d in ("dw.hip", "internal.h", "common.h", "mlp.h")]
    elif os.path.basename(src).startswith("ks_"):
        deps = [src] + [os.path.join(CSRC, d) for d in KSET_DEPS]
    else:
        deps = [f for f in glob.glob(os.path.join(CSRC, "*")) if not os.path.basename(f).startswith("ks_")]
    deps.append(os.path.join(REPO, "include", "spprl.h"))
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)




def _resources(text):
    """{kernel: {vgpr, agpr, vgpr_spill, sgpr_spill, lds}} from -Rpass-analysis=kernel-resource-usage."""
    import re

    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|"
                      r"ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur is not None:
            key = {"VGPRs": "vgpr", "AGPRs": "agpr", "VGPRs Spill": "vgpr_spill", "SGPRs Spill": "sgpr_spill",
                   "LDS Size [bytes/block]": "lds", "ScratchSize [bytes/lane]": "scratch",
                   "Occupancy [waves/SIMD]": "occupancy"}[m.group(1)]
            cur[key] = int(m.group(2))
    return out


def _compile(src, verbose):
    obj = _obj(src)
    cmd = [HIPCC] + FLAGS + ["-Rpass-analysis=kernel-resource-usage", "-c", "-o", obj, src]
    t0 = time.time()
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed on %s:\n%s" % (src, r.stdout[-8000:]))
    os.utime(obj, (t0, t0))  # stamped with the compile's start: a source edited meanwhile stays newer
    import json

    with open(obj + ".res.json", "w") as f:
        json.dump(_resources(r.stdout), f, indent=0)
    if verbose:
        print("  %-22s %5.0fs" % (os.path.basename(src), time.time() - t0), flush=True)
    return obj


# Phase kernels whose VGPRs spill to scratch have produced wrong results (the round-1
# fragment prefetch, the DDPG Ant actor phase before its heads were parked).  Every kernel's register use is
# recorded (build/kernel_resources.json) and the build FAILS on any kernel that uses scratch memory, except
# the ones below: (name fragment, scratch bytes per lane at most), each covered by a phase-level GPU parity
# test at the bench sizes (DESIGN.md §8 lists them and the tests).  A new or grown scratch user is an error.
SCRATCH_ALLOWED = {
    # SAC_AcM HalfCheetah actor phase with acm_critic (4 VGPRs; tests: test_gpu_parity sac_hcheetah_paper fixture)
    "k_sac_actor_phaseINS_3CfgILi17ELi17ELi6ELb1ELb0EEE": 12,
    # DDPG_AcM Ant (111-dim obs) actor phase / policy act (3-4 VGPRs; test_gpu_ddpg test_ddpg_acm_ant_dims_match_oracle)
    "k_ddpg_actor_phaseINS_4DCfgILi111ELi111ELi8ELb1EEE": 16,
    "k_ddpg_policy_actINS_4DCfgILi111ELi111ELi8EL": 20,
    # the ACM regression kernels: 8 bytes of SGPR-spill staging, no VGPR spills
    "k_acm_regress": 8,
    "k_bacm_regress": 8,
    # rocprim's onesweep radix sort (ks_perm.hip, sppRandPerm): a 48-byte private array, no VGPR spills
    "radix_sort_onesweep": 48,
}


def report_spills(objs, verbose=True):
    """Write build/kernel_resources.json; return {kernel: scratch bytes} of the kernels that use scratch
    memory beyond SCRATCH_ALLOWED (the caller fails the build on any)."""
    import json

    allres = {}
    for o in objs:
        try:
            with open(o + ".res.json") as f:
                allres.update(json.load(f))
        except OSError:
            pass
    with open(os.path.join(OBJ, "kernel_resources.json"), "w") as f:
        json.dump(allres, f, indent=1, sort_keys=True)
    users = {k: v.get("scratch", 0) for k, v in allres.items() if v.get("scratch", 0) > 0}
    bad = {}
    for k, n in users.items():
        lim = max([b for frag, b in SCRATCH_ALLOWED.items() if frag in k], default=0)
        if n > lim:
            bad[k] = n
    if verbose and users:
        print("kernels using scratch memory (bytes/lane, VGPRs spilled; * = not allowed):")
        for k, n in sorted(users.items(), key=lambda kv: -kv[1]):
            print("  %s %4d  %3d  %s" % ("*" if k in bad else " ", n, allres[k].get("vgpr_spill", 0), k[:140]))
    return bad


def build(force=False, verbose=True, prof=False, hopper_only=False, jobs=None, nodense=False):
    if prof:  # region-timing variant (never the default library): single TU
        out = os.path.join(HERE, "spprl", "libspprl_prof.so")
        extra = (["-DSPP_ONLY_HOPPER"] if hopper_only else []) + (["-DSPP_PROF_NODENSE"] if nodense else []) + (
            ["-DSPP_ONLY_BF16"] if "--bf16-only" in sys.argv else []) + (
            ["-DSPP_PROF_DRAIN"] if "--drain" in sys.argv else []) + (
            ["-DSPP_WITH_HCHEETAH"] if "--hcheetah" in sys.argv else [])
        cmd = [HIPCC] + FLAGS + ["-shared", "-DSPP_PROF", "-DSPP_SINGLE_TU"] + extra + [
            "-o", out, os.path.join(CSRC, "api.hip"), os.path.join(CSRC, "ks_perm.hip")]
        subprocess.check_call(cmd)
        return out
    if not force and up_to_date():
        if verbose:
            print("libspprl.so up to date")
        build_c_host(verbose)
        return OUT
    os.makedirs(OBJ, exist_ok=True)
    t0 = time.time()  # the library is stamped with this time: a source edited during the build stays newer
    srcs = units()
    jobs = jobs or min(len(srcs), max(1, min(os.cpu_count() or 1, 8)))
    if verbose:
        print("hipcc %s  (%d units, %d jobs)" % (" ".join(FLAGS), len(srcs), jobs), flush=True)
    todo = [s for s in srcs if force or _stale(s)]
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda s: _compile(s, verbose), todo))
    objs = [_obj(s) for s in srcs]
    bad = report_spills(objs, verbose)
    if bad:
        raise RuntimeError("kernels use scratch memory (VGPR spills) beyond build.SCRATCH_ALLOWED: %s" % sorted(bad))
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs)
    os.replace(OUT + ".tmp", OUT)
    os.utime(OUT, (t0, t0))
    if verbose:
        print("built %s in %.0fs" % (OUT, time.time() - t0))
    build_c_host(verbose)
    return OUT


C_HOST = os.path.join(REPO, "examples", "c_host", "sac_acm_step")
INC = os.path.join(REPO, "include")


def build_c_host(verbose=True, strict=False):
    """The plain-C host of the C-ABI (examples/c_host/sac_acm_step.c: gcc, include/spprl.h, libspprl.so and the
    HIP runtime only), in-tree next to its source; tests/test_gpu_c_host.py runs it on the GPU box.  An example
    program, not the library: a failure (no gcc, ROCm elsewhere, a new compiler warning) is reported and the library
    build stands, unless strict (the test that runs the program asks for it)."""
    src = C_HOST + ".c"
    if not os.path.exists(src) or (os.path.exists(C_HOST) and os.path.getmtime(C_HOST) >= max(
            os.path.getmtime(src), os.path.getmtime(os.path.join(INC, "spprl.h")))):
        return C_HOST
    rocm_lib = os.path.join(os.path.dirname(os.path.dirname(os.path.realpath(HIPCC))), "lib")
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-I" + INC, src, "-L" + os.path.join(HERE, "spprl"),
           "-lspprl", "-L" + rocm_lib, "-lamdhip64", "-Wl,-rpath,$ORIGIN/../../spp-rl_amd/spprl", "-Wl,-rpath," + rocm_lib,
           "-o", C_HOST]
    try:
        subprocess.check_call(cmd)
    except (OSError, subprocess.CalledProcessError) as e:
        if strict:
            raise
        print("warning: the C-host example did not build (%s); the library is unaffected" % e, file=sys.stderr)
        return None
    if verbose:
        print("built %s" % C_HOST)
    return C_HOST


if __name__ == "__main__":
    build(force="--force" in sys.argv, prof="--prof" in sys.argv, hopper_only="--hopper-only" in sys.argv,
          nodense="--nodense" in sys.argv)
