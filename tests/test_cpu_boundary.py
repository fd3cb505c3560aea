"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/spprl.h declares, and the host package is wired to it (no
compute calls here: there is no GPU)."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "spp-rl_amd", "spprl", "libspprl.so")
HDR = os.path.join(REPO, "include", "spprl.h")


def declared():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:sppStatus|const char\*|int|int64_t)\s+(spp\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib_built():
    if not os.path.exists(LIB):
        pytest.skip("libspprl.so not built (run __graft_entry__.build())")
    return LIB


def test_header_declares_the_boundary():
    names = declared()
    for must in ("sppReplayCreate", "sppReplayAddObs", "sppReplayAddStep", "sppReplayGather", "sppReplayObsStats",
                 "sppAgentCreate", "sppAgentBindNet", "sppSacAcmUpdate", "sppSacAcmCriticGrads",
                 "sppSacAcmActorApply", "sppAcmRegressStep", "sppPolicyAct", "sppMTRandint", "sppGetLastError"):
        assert must in names


def test_library_exports_every_declared_symbol(lib_built):
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib_built]).decode()
    exported = set(re.findall(r"\sT\s(spp\w+)$", out, re.M))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_python_binding_covers_header(lib_built):
    from spprl import _lib

    assert sorted(_lib.EXPORTED) == declared()
    lib = _lib.load()  # loads without a GPU
    assert lib.sppGetVersion() == 1


def test_host_mt19937_matches_numpy(lib_built):
    """sppMTRandint is host code: bit-exact with np.random.RandomState(seed).randint."""
    import ctypes

    import numpy as np

    from spprl import _lib

    for seed, high in ((0, 100), (42, 1_000_000), (7, 3), (123, 1)):
        h = ctypes.c_void_p()
        _lib.call("sppMTCreate", ctypes.byref(h), seed)
        out = np.empty(500, np.int64)
        _lib.call("sppMTRandint", h, high, 500, out.ctypes.data_as(ctypes.c_void_p))
        _lib.call("sppMTDestroy", h)
        np.testing.assert_array_equal(out, np.random.RandomState(seed).randint(0, high, 500))


def test_errors_cross_as_status_codes(lib_built):
    import ctypes

    from spprl import _lib

    lib = _lib.load()
    st = lib.sppMTRandint(None, 10, 1, None)
    assert st == 1
    assert b"randint" in lib.sppGetLastError()


def test_product_never_imports_the_oracle():
    pkg = os.path.join(REPO, "spp-rl_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(root, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", txt, re.M), f
                assert "oracle/" not in txt.replace("oracle/_ref", ""), f


def test_bench_refuses_world_size_other_than_gpus():
    """bench.py under a launcher whose WORLD_SIZE differs from --gpus exits 2 before touching a GPU."""
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2, out.stderr[-2000:]
    assert "WORLD_SIZE=2" in out.stderr


def test_unknown_reference_kwargs_raise_and_no_effect_ones_are_listed():
    """Agent constructors reject keywords they neither take nor list in config.NO_EFFECT_KWARGS, as the
    reference's constructor chain does (MetaLearner, rl.py:17-26, takes no **kwargs); the check runs
    before the library is touched, so it needs no GPU."""
    import spprl
    from spprl import config

    for cls in (spprl.SAC_AcM, spprl.DDPG_AcM):
        with pytest.raises(TypeError, match="foo"):
            cls(unbiased_update=True, foo=1)
    with pytest.raises(TypeError, match="acm_epochs"):
        spprl.SAC(acm_epochs=3)
    with pytest.raises(TypeError, match="unbiased_update"):
        spprl.SAC(unbiased_update=True)
    with pytest.raises(TypeError, match="bar"):
        spprl.PPO_AcM(bar=2)
    assert {"use_gpu", "log_dir", "verbose", "render", "acm_val_buffer_size"} <= set(config.NO_EFFECT_KWARGS)
    assert "obs_norm_alpha" in config.ON_POLICY_NO_EFFECT_KWARGS
    config.check_kwargs("x", {"use_gpu": True, "tensorboard_comment": "c"})


def test_c_host_example_compiles_against_the_header():
    """examples/c_host/sac_acm_step.c is plain C11 against include/spprl.h (no C++, no torch types): a C host
    can bind the boundary directly (its GPU run: tests/test_gpu_c_host.py)."""
    import shutil

    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("gcc not on PATH")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([gcc, "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-I", os.path.join(repo, "include"),
                        os.path.join(repo, "examples", "c_host", "sac_acm_step.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_acm_ob_idx_validation_follows_what_the_reference_can_run():
    """acm_ob_idx (acm/acm.py:94-99): None and the identity mean the whole vector; a length-ob list (a permutation,
    repeats allowed) is the column map of acm_cat (acm.py:260-264); other lengths are refused at construction (the
    reference builds its AcM with ob + k inputs, acm.py:148, and feeds it 2k), as are out-of-range entries."""
    from spprl.config import acm_columns

    assert acm_columns(None, 5) is None
    assert acm_columns(range(5), 5) is None
    assert acm_columns([4, 3, 2, 1, 0], 5) == [4, 3, 2, 1, 0]
    assert acm_columns([0, 0, 1, 2, 3], 5) == [0, 0, 1, 2, 3]
    for bad in ([0, 1, 2], [0, 1, 2, 3, 5], [-1, 0, 1, 2, 3]):
        with pytest.raises(ValueError):
            acm_columns(bad, 5)


def test_acm_columns_are_checked_at_the_boundary(lib_built):
    """sppReplaySetAcmColumns refuses a map whose length is not ob (or an entry out of range) before touching the
    device, with the reason in sppGetLastError."""
    import ctypes

    from spprl import _lib

    lib = _lib.load()
    cols = (ctypes.c_int * 3)(0, 1, 2)
    assert lib.sppReplaySetAcmColumns(None, cols, 3) != 0
