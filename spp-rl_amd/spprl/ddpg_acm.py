"""DDPG_AcM agent: rltoolkit's SPP-DDPG update path on the MI355X library.

Mirrors rltoolkit/acm/off_policy/ddpg_acm.py (reference @ v0) with the BasicAcM
the SPP-DDPG scripts inject (train/spp_ddpg_hcheetah.py):
  - ``update(obs, next_obs, action, reward, done, acm_action)``  (ddpg_acm.py:147-201):
    critic step, actor step, polyak of the critic AND actor targets (ddpg.py:273-284)
  - ``loss`` dict {critic, actor[, ddpg, dist]}, ``act`` (noise_action + process_action),
    ``batch_update_acm`` (AcMTrainer.batch_update, acm.py:246-258, BasicAcM incl. t / t1)
Parameters, Adam moments and the normaliser stay on the GPU.
"""
import ctypes

import numpy as np
import torch

from . import _lib, config, nets
from ._lib import call, ptr, stream_handle
from .replay import BufferAcMOffPolicy
from .trainer import OffPolicyLoop

_NETS = {"actor": _lib.SPP_NET_ACTOR, "critic": _lib.SPP_NET_CRITIC1, "actor_targ": _lib.SPP_NET_ACTOR_TARG,
         "critic_targ": _lib.SPP_NET_CRITIC1_TARG, "acm": _lib.SPP_NET_ACM}


class DDPG_AcM(OffPolicyLoop):
    def __init__(self, env_name="HalfCheetah-v2", gamma=config.GAMMA, actor_lr=config.DDPG_LR,
                 critic_lr=config.DDPG_LR, tau=config.TAU, act_noise=config.ACT_NOISE,
                 update_batch_size=config.UPDATE_BATCH_SIZE, buffer_size=config.BUFFER_SIZE, acm_lr=config.ACM_LR,
                 acm_critic=config.ACM_CRITIC, custom_loss=0.0, norm_closs=config.NORM_CLOSS,
                 min_max_denormalize=config.MIN_MAX_DENORMALIZE, denormalize_actor_out=config.DENORMALIZE_ACTOR_OUT,
                 obs_norm=config.OBS_NORM, max_batch=None, device="cuda", env_spec=None, seed=None,
                 unbiased_update=False, acm_ob_idx=None, **loop_kw):
        self._check_kwargs(loop_kw)
        _lib.load()
        ob, ac, ac_high, _ = env_spec or config.ENV_SPECS[env_name]
        self.env_spec = tuple(env_spec or config.ENV_SPECS[env_name])
        self.env_name, self.ob_dim, self.ac_dim = env_name, ob, ac
        self.device = torch.device(device)
        self.gamma, self.actor_lr, self.critic_lr, self.acm_lr, self.tau = gamma, actor_lr, critic_lr, acm_lr, tau
        self.act_noise = act_noise
        self.update_batch_size = update_batch_size
        self.acm_critic, self.custom_loss, self.norm_closs = bool(acm_critic), float(custom_loss), bool(norm_closs)
        self.unbiased_update = bool(unbiased_update)  # make_unbiased_update (ddpg_acm.py:59-79)
        self.min_max_denormalize, self.denormalize_actor_out = bool(min_max_denormalize), bool(denormalize_actor_out)
        self.actor_output_dim = aout = ob
        lim = 1.0 if self.min_max_denormalize else float(config.MAX_ABS_OBS_VALUE)  # acm.py:102-108
        self.actor_ac_lim = torch.full((aout,), lim)
        self.max_batch = int(max_batch or config.default_max_batch(update_batch_size, loop_kw))
        cin = ob + (ac if self.acm_critic else aout)
        self.layouts = {_lib.SPP_NET_ACTOR: nets.ddpg_actor_layout(ob, aout),
                        _lib.SPP_NET_ACTOR_TARG: nets.ddpg_actor_layout(ob, aout),
                        _lib.SPP_NET_CRITIC1: nets.critic_layout(cin), _lib.SPP_NET_CRITIC1_TARG: nets.critic_layout(cin),
                        _lib.SPP_NET_ACM: nets.basic_acm_layout(2 * ob, ac)}
        cfg = _lib.AgentConfig(_lib.SPP_ALGO_DDPG_ACM, ob, aout, ac, int(self.acm_critic),
                               int(self.min_max_denormalize), int(self.norm_closs), self.custom_loss, gamma, tau,
                               actor_lr, critic_lr, 0.0, acm_lr, 0.0, self.max_batch)
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        call("sppAgentCreate", ctypes.byref(h), ctypes.byref(cfg), dev)
        self._h = h
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        self.params, self.grads, self.exp_avg, self.exp_avg_sq = {}, {}, {}, {}
        for net, lay in self.layouts.items():
            n = ctypes.c_int64()
            call("sppAgentNetSize", self._h, net, ctypes.byref(n))
            assert n.value == nets.numel(lay), (net, n.value, nets.numel(lay))
            self.params[net] = nets.linear_init_(torch.empty(n.value, device=self.device), lay, gen)
        # gradient buckets (the data-parallel exchange units): [critic], [actor], [acm]
        for net in (_lib.SPP_NET_CRITIC1, _lib.SPP_NET_ACTOR, _lib.SPP_NET_ACM):
            n = self.params[net].numel()
            self.grads[net] = torch.zeros(n, device=self.device)
            self.exp_avg[net] = torch.zeros(n, device=self.device)
            self.exp_avg_sq[net] = torch.zeros(n, device=self.device)
        self.bucket_critic, self.bucket_actor = self.grads[_lib.SPP_NET_CRITIC1], self.grads[_lib.SPP_NET_ACTOR]
        self.bucket_acm = self.grads[_lib.SPP_NET_ACM]
        # ddpg.py:120-125: targets start as deep copies
        self.params[_lib.SPP_NET_CRITIC1_TARG].copy_(self.params[_lib.SPP_NET_CRITIC1])
        self.params[_lib.SPP_NET_ACTOR_TARG].copy_(self.params[_lib.SPP_NET_ACTOR])
        for net in self.layouts:
            call("sppAgentBindNet", self._h, net, ptr(self.params[net]), ptr(self.grads.get(net)),
                 ptr(self.exp_avg.get(net)), ptr(self.exp_avg_sq.get(net)))
        a_lim = self.actor_ac_lim.numpy().astype(np.float32)
        m_lim = np.full(ac, float(ac_high), np.float32)  # unused by BasicAcM (its scale is t1)
        call("sppAgentSetLimits", self._h, a_lim.ctypes.data_as(ctypes.c_void_p), m_lim.ctypes.data_as(ctypes.c_void_p))
        self.replay_buffer = BufferAcMOffPolicy(buffer_size, ob, aout, ac, device=self.device,
                                                min_max_denormalize=self.min_max_denormalize, obs_norm=obs_norm,
                                                n_envs=int(loop_kw.get("n_envs", 1)))
        rb = self.replay_buffer
        call("sppAgentBindNormalizer", self._h, ptr(rb.min_obs), ptr(rb.max_obs), ptr(rb.obs_mean), ptr(rb.obs_std))
        self.acm_ob_idx = list(range(ob)) if acm_ob_idx is None else [int(i) for i in acm_ob_idx]
        cols = config.acm_columns(acm_ob_idx, ob)  # AcMTrainer's acm_ob_idx (acm.py:94-99, 260-264)
        if cols is not None:
            rb.set_acm_columns(cols)
        self._losses = torch.zeros(_lib.NUM_LOSSES, device=self.device)
        self.acm_kind = "basic"  # BasicAcM: per-step regression path
        self._init_loop(update_batch_size=update_batch_size, **loop_kw)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sppAgentDestroy(h)
            self._h = None

    def net_state(self, net):
        return nets.state_dict(self.params[net], self.layouts[net])

    def load_net(self, net, state):
        nets.load_state(self.params[net], self.layouts[net], state)

    # ------------------------------------------------------------------ update
    def update(self, obs, next_obs, action, reward, done, acm_action):
        """DDPG_AcM.update (ddpg_acm.py:147-201)."""
        d = self.device
        t = lambda x, dt=torch.float32: torch.as_tensor(x, dtype=dt).to(d).contiguous()  # noqa: E731
        tens = [t(obs), t(next_obs), t(action) if action is not None else None, t(reward).reshape(-1),
                t(done, torch.int8).reshape(-1), t(acm_action)]
        b = _lib.Batch(tens[0].shape[0], *[ptr(x) for x in tens])
        call("sppDdpgAcmUpdate", self._h, ctypes.byref(b), ptr(self._losses), stream_handle())
        self._keep = tens

    def update_from_replay_dp(self, idx, allreduce=None, beside=None):
        """Device-sampled step split at its exchange points (allreduce averages a flat bucket); beside()
        enqueues independent work under the actor bucket's exchange."""
        st = stream_handle()
        self._stage(idx)
        call("sppDdpgAcmCriticGrads", self._h, None, ptr(self._losses), st)
        if allreduce is not None:
            allreduce(self.bucket_critic)
        call("sppDdpgAcmCriticApply", self._h, st)
        call("sppDdpgAcmActorGrads", self._h, ptr(self._losses), st)
        self._exchange(allreduce, self.bucket_actor, beside)
        call("sppDdpgAcmActorApply", self._h, st)

    def _fused_update(self, idx, counter, allreduce=None, beside=None):
        self.update_from_replay_dp(idx, allreduce, beside)

    @property
    def loss(self):
        v = self._losses.detach().cpu().numpy()
        out = {"critic": float(v[0]), "actor": float(v[1])}
        if self.custom_loss:
            out["ddpg"], out["dist"] = float(v[2]), float(v[3])
        return out

    # ------------------------------------------------------------------ ACM regression + acting
    def batch_update_acm(self, x, y):
        """AcMTrainer.batch_update (acm.py:246-258) on the BasicAcM (t, t1 trained too)."""
        x = torch.as_tensor(x, dtype=torch.float32).to(self.device).contiguous()
        y = torch.as_tensor(y, dtype=torch.float32).to(self.device).contiguous()
        loss = torch.zeros(1, device=self.device)
        call("sppAcmRegressStep", self._h, ptr(x), ptr(y), x.shape[0], ptr(loss), stream_handle())
        self._keep_acm = (x, y)
        return loss

    def act(self, obs, eps=None, noise=None, mode=1, act_noise=None):
        """noise_action + process_action (ddpg_acm.py:40-50, off_policy.py:89-106)."""
        obs = torch.as_tensor(obs, dtype=torch.float32).to(self.device).contiguous()
        E = obs.shape[0]
        tgt = torch.empty(E, self.actor_output_dim, device=self.device)
        env = torch.empty(E, self.ac_dim, device=self.device)
        call("sppPolicyAct", self._h, ptr(obs), E, ptr(eps), ptr(noise),
             self.act_noise if act_noise is None else act_noise, mode, int(self.denormalize_actor_out), ptr(tgt),
             ptr(env), stream_handle())
        self._keep_act = (obs, eps, noise)
        return tgt, env

    # ------------------------------------------------------------------ checkpoints (rl.py:263-301)
    def collect_params_dict(self):
        rb = self.replay_buffer
        return {"actor": self.net_state(_lib.SPP_NET_ACTOR), "critic": self.net_state(_lib.SPP_NET_CRITIC1),
                "obs_mean": rb.obs_mean.cpu(), "obs_std": rb.obs_std.cpu(),
                "min_obs": rb.min_obs.cpu() if rb._have_minmax else None,
                "max_obs": rb.max_obs.cpu() if rb._have_minmax else None,
                "acm": self.net_state(_lib.SPP_NET_ACM)}

    def apply_params_dict(self, d):
        for k in ("actor", "critic", "acm"):
            self.load_net(_NETS[k], d[k])
        rb = self.replay_buffer
        rb.obs_mean.copy_(torch.as_tensor(d["obs_mean"]))
        rb.obs_std.copy_(torch.as_tensor(d["obs_std"]))
        if d.get("min_obs") is not None and d.get("max_obs") is not None:
            rb.min_obs.copy_(torch.as_tensor(d["min_obs"]))
            rb.max_obs.copy_(torch.as_tensor(d["max_obs"]))
            rb._have_minmax = True
