"""GPU parity over several consecutive SAC_AcM updates, with the packed weight images checked.

The phase kernels never read the fp32 parameters: they read fragment-packed weight images that
k_pack_matrix rebuilds after every Adam step (bf16 agents: bf16 images, RNE of the fp32 master
weights).  A stale or mis-rounded image would stay inside the single-step loss tolerance, so here
each of 3 consecutive updates (sac_acm.py:89-162, fresh batch and eps every step) is followed by:
  - every image of every network unpacked (sppAgentUnpackImage) and compared BIT-EXACTLY with the
    fp32 parameters its kernels consumed in that update (fp32 agents) or with torch's RNE bf16
    rounding of them (bf16 agents);
  - the post-step parameters of every network compared with the float64 oracle run on the same
    batches (oracle/sac_acm.py): fp32 |d| <= 2 lr per step with < 0.2 % of weights beyond 1e-5 after
    step 1 (Adam's first step moves each weight by ~lr sign(g): a gradient sign flip at the fp32
    rounding level moves it by up to 2 lr); bf16 MLP (bf16 gradients, 8-bit mantissa) at B = 4,096 and
    at the bench batch 409,600: |d| <= 2 lr per step, mean |d| <= 0.05 lr per step and at most 1 % of
    the weights per step beyond lr (a sign flip; a wrong path flips about half of them);
  - losses: fp32 rtol 1e-4, bf16 rtol 3e-2.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

import spprl  # noqa: E402
from spprl import _lib  # noqa: E402
from oracle.sac_acm import OracleSacAcm  # noqa: E402
from test_gpu_bigbatch import SAC_NETS, random_batch, set_minmax, snapshot  # noqa: E402

DEV = torch.device("cuda:0")


def check_images(ag, bf16, before):
    """Every packed image equals the parameters its last consumer saw, bit for bit (bf16 agents: the
    RNE bf16 of them).  An update packs every image before its critic phase and re-packs the critic
    images after the critic Adam step (the actor phase reads the updated critics), so after an update
    the critic images hold the current critic parameters and the actor / target / ACM images hold
    the parameters from before the update (``before``)."""
    n_img = 0
    for name, net in SAC_NETS.items():
        p = ag.params[net] if name in ("critic_1", "critic_2") else before[name]
        cnt = np.zeros(1, np.int32)
        _lib.call("sppAgentImageCount", ag._h, net, cnt.ctypes.data)
        assert cnt[0] > 0, name
        want = p.to(torch.bfloat16).float() if bf16 else p
        for i in range(int(cnt[0])):
            out = torch.full_like(p, float("nan"))
            _lib.call("sppAgentUnpackImage", ag._h, net, i, _lib.ptr(out), _lib.stream_handle())
            torch.cuda.synchronize()
            cov = ~torch.isnan(out)
            assert int(cov.sum()) > 0, (name, i)
            bad = int((out[cov].view(torch.int32) != want[cov].view(torch.int32)).sum())
            assert bad == 0, "%s image %d: %d of %d entries differ from %s(params)" % (
                name, i, bad, int(cov.sum()), "RNE bf16" if bf16 else "fp32")
            n_img += 1
    return n_img


@pytest.mark.parametrize("env_name,ob,ac,B,bf16", [("Ant-v2", 111, 8, 4096, True),
                                                   ("Ant-v2", 111, 8, 409600, True),  # the sac_ant_bf16 bench batch
                                                   ("Hopper-v2", 11, 3, 65536, False)])
def test_three_updates_images_and_params_match_oracle(env_name, ob, ac, B, bf16):
    lr, steps = 1e-3, 3
    rng = np.random.RandomState(29 + ob)
    ag = spprl.SAC_AcM(env_name=env_name, acm_critic=True, custom_loss=0.2, norm_closs=False,
                       min_max_denormalize=True, denormalize_actor_out=True, gamma=0.99, max_batch=B,
                       buffer_size=128, device=DEV, seed=7, mlp_bf16=bf16)
    params = snapshot(ag, SAC_NETS)
    norm = set_minmax(ag, rng, ob)
    o = OracleSacAcm(ob, ob, ac, acm_critic=True, custom_loss=0.2, norm_closs=False, norm=norm, actor_lim=1.0,
                     acm_lim=np.ones(ac, np.float32), gamma=0.99, params=params, dtype=torch.float64)
    for step in range(1, steps + 1):
        batch = random_batch(rng, B, ob, ob, ac)
        e1, e2 = rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32)
        before = {k: ag.params[net].clone() for k, net in SAC_NETS.items()}
        ag.update(*batch, eps_next=e1, eps_cur=e2)
        torch.cuda.synchronize()
        ol = o.update(*batch, e1, e2)
        nimg = check_images(ag, bf16, before)
        gl = ag.loss
        tol = 3e-2 if bf16 else 1e-4
        for k in ("critic_1", "critic_2", "actor"):
            assert abs(gl[k] - ol[k]) <= tol * abs(ol[k]) + 1e-6, (step, k, gl[k], ol[k])
        stats = {}
        for k in ("actor", "critic_1", "critic_2", "critic_1_targ", "critic_2_targ"):
            got = ag.params[SAC_NETS[k]].cpu().numpy().astype(np.float64)
            d = np.abs(got - o.flat(k).astype(np.float64))
            stats[k] = (d.max() / lr, d.mean() / lr, float(np.mean(d > 1e-5)), float(np.mean(d > lr)))
            assert d.max() <= 2 * lr * step * 1.01, (step, k, d.max())
            if bf16:
                # |d| <= 2 lr per step is saturated by any one sign flip; these two can fail: a wrong operand
                # or gradient moves ~half the weights by 2 lr (mean ~lr, fraction beyond lr ~0.5)
                assert d.mean() <= 0.05 * lr * step, (step, k, d.mean())
                assert np.mean(d > lr) <= 0.01 * step, (step, k, np.mean(d > lr))
            elif step == 1:
                assert np.mean(d > 1e-5) < 2e-3, (k, np.mean(d > 1e-5))
        print("step %d: %d images exact; |d|/lr max, mean, frac>1e-5, frac>lr:" % (step, nimg),
              {k: tuple(round(x, 4) for x in v) for k, v in stats.items()})
        assert ag.current_alpha() == pytest.approx(o.alpha, rel=1e-4 if not bf16 else 1e-2)
