"""Vanilla SAC (BASELINE.json configs[0]): rltoolkit/algorithms/sac/sac.py on the MI355X library.

The update is SAC_AcM's device path with no ACM: the actor emits the env action
(ac dims, tanh-squashed and scaled by the env's action high), the twin critics take
cat(obs, action), there is no custom loss, and the actor output is not denormalised.
Kept from the reference:
  - constructor kwargs of SAC / DDPG / RL (sac.py:17-110, ddpg.py:18-130)
  - quirk Q1: ``tau`` and ``act_noise`` are not forwarded to DDPG (sac.py:17-24), so the
    config defaults (0.005, 0.1) apply; rollout actions are a ~ pi(s) + 0.1 N(0,1), clipped
  - quirk Q3: time-limit ends are not ``done`` (rl.py:185, ddpg.py:210-212)
  - quirk Q4: target entropy = -ac_dim (sac.py:104-106)
  - ``update(obs, next_obs, action, reward, done)`` (sac.py:218-280), ``loss`` keys,
    ``collect_params_dict`` keys (sac.py:287-309)
"""
from . import _lib
from .sac_acm import SAC_AcM


class SAC(SAC_AcM):
    ALGO = _lib.SPP_ALGO_SAC
    VANILLA = True

    def __init__(self, env_name="HalfCheetah-v2", **kw):
        # SAC -> DDPG -> RL -> MetaLearner (sac.py:17-25, ddpg.py:19-33, rl.py:17-26) take no AcMTrainer /
        # AcMOffPolicy / DDPG_AcM keyword: the reference raises TypeError on them, and so does this class
        acm_only = sorted(k for k in kw if k.startswith("acm_") or k in (
            "custom_loss", "norm_closs", "denormalize_actor_out", "unbiased_update", "acm_critic"))
        if acm_only:
            raise TypeError("SAC got unexpected keyword argument(s): %s (SPP / AcM options: use SAC_AcM)"
                            % ", ".join(acm_only))
        kw.pop("min_max_denormalize", None)  # MetaLearner's; without obs_norm it normalises nothing here
        super().__init__(env_name=env_name, acm_critic=False, custom_loss=0.0, min_max_denormalize=False,
                         denormalize_actor_out=False, **kw)

    def update(self, obs, next_obs, action, reward, done, eps_next=None, eps_cur=None):
        """SAC.update (sac.py:218-280): 5-tuple batch (ReplayBuffer.sample_batch, replay_buffer.py:233-261)."""
        super().update(obs, next_obs, action, reward, done, action, eps_next=eps_next, eps_cur=eps_cur)

    @property
    def loss(self):
        v = self._losses.detach().cpu().numpy()
        return {"actor": float(v[2]), "critic_1": float(v[0]), "critic_2": float(v[1])}

    def collect_params_dict(self):  # sac.py:287-296
        d = super().collect_params_dict()
        d.pop("acm", None)
        return d

    def apply_params_dict(self, d):  # sac.py:298-309
        d = dict(d)
        d.setdefault("acm", self.net_state(_lib.SPP_NET_ACM))
        super().apply_params_dict(d)

    def pre_train(self):
        raise AttributeError("vanilla SAC has no ACM pre-training (rltoolkit SAC defines none)")
