"""Debug: DDPG_AcM Ant-dims actor gradient vs the oracle, per parameter tensor."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "spp-rl_amd"), REPO, os.path.join(REPO, "tests")]
import spprl  # noqa: E402
from spprl import _lib, nets  # noqa: E402
from oracle import nets as onets  # noqa: E402
from oracle.ddpg_acm import OracleDdpgAcm  # noqa: E402

DEV = torch.device("cuda:0")
NAMES = {"actor": _lib.SPP_NET_ACTOR, "critic": _lib.SPP_NET_CRITIC1, "actor_targ": _lib.SPP_NET_ACTOR_TARG,
         "critic_targ": _lib.SPP_NET_CRITIC1_TARG, "acm": _lib.SPP_NET_ACM}
ob, ac = int(sys.argv[1]) if len(sys.argv) > 1 else 111, int(sys.argv[2]) if len(sys.argv) > 2 else 8
B = 96
for closs, acmc in ((1.0, True), (0.0, True), (1.0, False)):
    ag = spprl.DDPG_AcM(env_name="custom", env_spec=(ob, ac, 1.0, 1000), gamma=0.99, actor_lr=5e-4, critic_lr=5e-4,
                        acm_critic=acmc, custom_loss=closs, norm_closs=False, min_max_denormalize=True,
                        denormalize_actor_out=True, max_batch=B, buffer_size=64, device=DEV, seed=11)
    params = {k: {n: v.numpy() for n, v in ag.net_state(net).items()} for k, net in NAMES.items()}
    rng = np.random.RandomState(B)
    lo = -rng.uniform(0.5, 2, ob).astype(np.float32)
    hi = rng.uniform(0.5, 2, ob).astype(np.float32)
    rb = ag.replay_buffer
    rb.min_obs.copy_(torch.from_numpy(lo))
    rb.max_obs.copy_(torch.from_numpy(hi))
    rb._have_minmax = True
    norm = onets.Norm(True, torch.from_numpy(lo), torch.from_numpy(hi))
    o = OracleDdpgAcm(ob, ob, ac, norm=norm, actor_lim=np.ones(ob, np.float32), gamma=0.99, tau=0.005,
                      params=params, custom_loss=closs, acm_critic=acmc)
    batch = (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
             rng.uniform(-1, 1, (B, ob)).astype(np.float32), rng.randn(B).astype(np.float32),
             (rng.rand(B) < 0.1).astype(np.int8), rng.uniform(-1, 1, (B, ac)).astype(np.float32))
    ag.update(*batch)
    ol = o.update(*batch)
    torch.cuda.synchronize()
    print("custom_loss", closs, "acmc", acmc, "losses gpu", ag.loss, "oracle", {k: ol[k] for k in ("critic", "actor", "ddpg", "dist")})
    g = ag.grads[_lib.SPP_NET_ACTOR].cpu().numpy().astype(np.float64)
    r = np.asarray(o.last["grads"]["actor"], np.float64)
    off = 0
    for name, shape in nets.ddpg_actor_layout(ob, ob):
        n = int(np.prod(shape))
        a, b = g[off:off + n], r[off:off + n]
        print("  %-12s relerr %.3g  |ref| %.3g" % (name, np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30),
                                                   np.linalg.norm(b)))
        if name == "fc3.weight":
            d = np.abs((a - b).reshape(shape)).max(1)
            print("   fc3 rows with err > 1e-6 * max:", np.flatnonzero(d > 1e-3 * np.abs(b).max())[:40])
        off += n
