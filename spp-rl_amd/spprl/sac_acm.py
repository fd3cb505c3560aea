"""SAC_AcM agent: rltoolkit's SPP-SAC update path on the MI355X library.

Mirrors rltoolkit/acm/off_policy/sac_acm.py (reference @ v0) and the pieces of
its MRO that shape the update (SAC sac.py:16-110, DDPG ddpg.py:18-130,
AcMTrainer acm.py:15-183, AcMOffPolicy off_policy.py:8-47):
  - constructor kwargs and defaults (quirks kept: Q1 tau/act_noise are the
    config values whatever is passed; Q4 target entropy = -env ac_dim)
  - ``update(obs, next_obs, action, reward, done, acm_action)``  (sac_acm.py:89-162)
  - ``loss`` dict, ``alpha``, ``collect_params_dict`` / ``apply_params_dict`` /
    ``save`` / ``load`` (rl.py:263-301, sac.py:287-309, ddpg_acm.py:87-94)
Parameters, Adam moments, log_alpha and the normaliser stay on the GPU; the
update never synchronises the host (losses are read lazily).
"""
import ctypes
import math
import pickle

import numpy as np
import torch

from . import _lib, config, nets
from ._lib import call, ptr, stream_handle
from .replay import BufferAcMOffPolicy, ReplayBuffer
from .trainer import OffPolicyLoop


class SAC_AcM(OffPolicyLoop):
    ALGO = _lib.SPP_ALGO_SAC_ACM
    VANILLA = False

    def __init__(self, env_name="Hopper-v2", gamma=config.GAMMA, actor_lr=config.DDPG_LR,
                 critic_lr=config.DDPG_LR, alpha_lr=config.ALPHA_LR, alpha=config.ALPHA, tau=config.TAU,
                 act_noise=0.0, update_batch_size=config.UPDATE_BATCH_SIZE, buffer_size=config.BUFFER_SIZE,
                 acm_lr=config.ACM_LR, acm_critic=config.ACM_CRITIC, custom_loss=0.0, norm_closs=config.NORM_CLOSS,
                 min_max_denormalize=config.MIN_MAX_DENORMALIZE, denormalize_actor_out=config.DENORMALIZE_ACTOR_OUT,
                 acm_ob_idx=None, obs_norm=config.OBS_NORM, max_batch=None, device="cuda", env_spec=None,
                 seed=None, mlp_bf16=False, unbiased_update=False, **loop_kw):
        self._check_kwargs(loop_kw)
        _lib.load()
        ob, ac, ac_high, max_ep = env_spec or config.ENV_SPECS[env_name]
        vanilla = self.VANILLA
        if vanilla:  # SAC (sac.py): no ACM anywhere, the actor emits the env action
            acm_critic, custom_loss, acm_ob_idx = False, 0.0, None
            loop_kw.setdefault("acm_epochs", 0)
        self.env_spec = tuple(env_spec or config.ENV_SPECS[env_name])
        self.env_name, self.ob_dim, self.ac_dim = env_name, ob, ac
        # Q3: AcMOffPolicy never masks time-limit done (off_policy.py:43); RL does (rl.py:185)
        self.max_ep_len = int(max_ep) if vanilla else None
        self.device = torch.device(device)
        self.gamma, self.actor_lr, self.critic_lr, self.alpha_lr, self.acm_lr = gamma, actor_lr, critic_lr, alpha_lr, acm_lr
        self.tau = config.TAU  # Q1: SAC consumes `tau` (sac.py:21) -> DDPG default
        self.act_noise = config.ACT_NOISE  # Q1: likewise (ddpg.py:29,100)
        self.update_batch_size = update_batch_size
        self.acm_critic, self.custom_loss, self.norm_closs = bool(acm_critic), float(custom_loss), bool(norm_closs)
        self.unbiased_update = bool(unbiased_update)  # DDPG_AcM.make_update (ddpg_acm.py:59-79), inherited
        self.min_max_denormalize, self.denormalize_actor_out = bool(min_max_denormalize), bool(denormalize_actor_out)
        self._acm_cols = config.acm_columns(acm_ob_idx, ob)  # (acm.py:94-99; refuses lists the reference can't run)
        self.acm_ob_idx = list(range(ob)) if acm_ob_idx is None else [int(i) for i in acm_ob_idx]
        self.actor_output_dim = ac if vanilla else len(self.acm_ob_idx)
        # acm.py:102-108 actor limit
        if vanilla:
            lim = float(ac_high)  # SAC_Actor(ob, self.ac_lim, ac) (sac.py:97)
        elif self.min_max_denormalize:
            lim = 1.0
        else:
            lim = float(config.MAX_ABS_OBS_VALUE)  # obs spaces of these envs are unbounded
        self.actor_ac_lim = torch.full((self.actor_output_dim,), lim)
        self.ac_lim = torch.full((ac,), float(ac_high))
        self.target_entropy = -float(ac)  # Q4 (sac.py:104-106)
        self.alpha = alpha
        self.max_batch = int(max_batch or config.default_max_batch(update_batch_size, loop_kw))
        aout = self.actor_output_dim
        cin = ob + (ac if self.acm_critic else aout)
        self.layouts = {_lib.SPP_NET_ACTOR: nets.sac_actor_layout(ob, aout),
                        _lib.SPP_NET_CRITIC1: nets.critic_layout(cin), _lib.SPP_NET_CRITIC2: nets.critic_layout(cin),
                        _lib.SPP_NET_CRITIC1_TARG: nets.critic_layout(cin),
                        _lib.SPP_NET_CRITIC2_TARG: nets.critic_layout(cin), _lib.SPP_NET_ACM: nets.acm_layout(2 * ob, ac)}
        cfg = _lib.AgentConfig(self.ALGO, ob, aout, ac, int(self.acm_critic), int(self.min_max_denormalize or vanilla),
                               int(self.norm_closs), self.custom_loss, gamma, self.tau, actor_lr, critic_lr, alpha_lr,
                               acm_lr, self.target_entropy, self.max_batch, int(bool(mlp_bf16)))
        self.mlp_bf16 = bool(mlp_bf16)  # bf16 MFMA MLP layers, fp32 everything else (BASELINE configs[4])
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        call("sppAgentCreate", ctypes.byref(h), ctypes.byref(cfg), dev)
        self._h = h
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        self.params, self.grads, self.exp_avg, self.exp_avg_sq = {}, {}, {}, {}
        sizes = {}
        for net, lay in self.layouts.items():
            n = ctypes.c_int64()
            call("sppAgentNetSize", self._h, net, ctypes.byref(n))
            assert n.value == nets.numel(lay), (net, n.value, nets.numel(lay))
            sizes[net] = n.value
            self.params[net] = nets.linear_init_(torch.empty(n.value, device=self.device), lay, gen)
        # gradient buckets = the data-parallel exchange units (one all-reduce each):
        #   critic: [critic_1 | critic_2], actor: [actor | d alpha operand], acm: [acm]
        c1, c2, na, nm = (sizes[_lib.SPP_NET_CRITIC1], sizes[_lib.SPP_NET_CRITIC2], sizes[_lib.SPP_NET_ACTOR],
                          sizes[_lib.SPP_NET_ACM])
        self.bucket_critic = torch.zeros(c1 + c2, device=self.device)
        self.bucket_actor = torch.zeros(na + 1, device=self.device)
        self.bucket_acm = torch.zeros(nm, device=self.device)
        self.grads = {_lib.SPP_NET_CRITIC1: self.bucket_critic[:c1], _lib.SPP_NET_CRITIC2: self.bucket_critic[c1:],
                      _lib.SPP_NET_ACTOR: self.bucket_actor[:na], _lib.SPP_NET_ACM: self.bucket_acm}
        self.alpha_grad = self.bucket_actor[na:]
        for net in self.grads:
            self.exp_avg[net] = torch.zeros(sizes[net], device=self.device)
            self.exp_avg_sq[net] = torch.zeros(sizes[net], device=self.device)
        # sac.py:127,136: targets start as deep copies of the critics
        self.params[_lib.SPP_NET_CRITIC1_TARG].copy_(self.params[_lib.SPP_NET_CRITIC1])
        self.params[_lib.SPP_NET_CRITIC2_TARG].copy_(self.params[_lib.SPP_NET_CRITIC2])
        for net in self.layouts:
            call("sppAgentBindNet", self._h, net, ptr(self.params[net]), ptr(self.grads.get(net)),
                 ptr(self.exp_avg.get(net)), ptr(self.exp_avg_sq.get(net)))
        a_lim = self.actor_ac_lim.numpy().astype(np.float32)
        m_lim = self.ac_lim.numpy().astype(np.float32)
        call("sppAgentSetLimits", self._h, a_lim.ctypes.data_as(ctypes.c_void_p), m_lim.ctypes.data_as(ctypes.c_void_p))
        self.alpha_state = torch.tensor([math.log(alpha), 0.0, 0.0, alpha], dtype=torch.float64, device=self.device)
        self.alpha_f32 = torch.tensor([alpha], dtype=torch.float32, device=self.device)
        call("sppAgentBindAlpha", self._h, ptr(self.alpha_state), ptr(self.alpha_f32))
        call("sppAgentBindAlphaGrad", self._h, ptr(self.alpha_grad))
        if vanilla:
            # obs_norm (DDPG.__init__, ddpg.py:101-115): the plain ReplayBuffer normalises sampled obs / next obs
            # (z-score, replay_buffer.py:246-249) and the rollout's act input (ddpg.py:203); its statistics start
            # as zeros / ones (replay_buffer.py:113-115), i.e. only the clip, until the first update_obs_mean_std
            self.replay_buffer = ReplayBuffer(buffer_size, ob, ac, device=self.device, obs_norm=bool(obs_norm),
                                              n_envs=int(loop_kw.get("n_envs", 1)))
            # identity denormalisation of the actor output: min-max over [-1, 1] is 0 + x * 1, exact; the z-score
            # pair is the ring's own statistics (the staged batch's obs_norm normalisation, sppAgentStagePost 2)
            self._ident = torch.stack([-torch.ones(ob), torch.ones(ob)]).to(self.device)
            rb = self.replay_buffer
            call("sppAgentBindNormalizer", self._h, ptr(self._ident[0]), ptr(self._ident[1]), ptr(rb.obs_mean),
                 ptr(rb.obs_std))
        else:
            self.replay_buffer = BufferAcMOffPolicy(buffer_size, ob, aout, ac, device=self.device,
                                                    min_max_denormalize=self.min_max_denormalize, obs_norm=obs_norm,
                                                    n_envs=int(loop_kw.get("n_envs", 1)))
            self.bind_normalizer(self.replay_buffer)
            if self._acm_cols is not None:
                self.replay_buffer.set_acm_columns(self._acm_cols)
        self._losses = torch.zeros(_lib.NUM_LOSSES, device=self.device)
        self._init_loop(update_batch_size=update_batch_size, **loop_kw)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sppAgentDestroy(h)
            self._h = None

    # ------------------------------------------------------------------ wiring
    def bind_normalizer(self, buf):
        call("sppAgentBindNormalizer", self._h, ptr(buf.min_obs), ptr(buf.max_obs), ptr(buf.obs_mean),
             ptr(buf.obs_std))

    def net_state(self, net):
        return nets.state_dict(self.params[net], self.layouts[net])

    def load_net(self, net, state):
        nets.load_state(self.params[net], self.layouts[net], state)

    def set_steps(self, actor=0, critic=0, alpha=0, acm=0):
        call("sppAgentSetSteps", self._h, actor, critic, alpha, acm)

    # ------------------------------------------------------------------ update
    def _batch(self, obs, next_obs, action, reward, done, acm_action):
        d = self.device
        t = lambda x, dt=torch.float32: torch.as_tensor(x, dtype=dt).to(d).contiguous()  # noqa: E731
        tens = [t(obs), t(next_obs), t(action) if action is not None else None, t(reward).reshape(-1),
                t(done, torch.int8).reshape(-1), t(acm_action)]
        B = tens[0].shape[0]
        b = _lib.Batch(B, *[ptr(x) for x in tens])
        return b, tens

    def update(self, obs, next_obs, action, reward, done, acm_action, eps_next=None, eps_cur=None):
        """SAC_AcM.update (sac_acm.py:89-162).  eps_* are the rsample draws (sac_acm.py:44, :137);
        when omitted they are drawn from torch's generator on the device."""
        b, keep = self._batch(obs, next_obs, action, reward, done, acm_action)
        shape = (b.B, self.actor_output_dim)
        e1 = torch.as_tensor(eps_next, dtype=torch.float32).to(self.device).contiguous() if eps_next is not None \
            else torch.randn(shape, device=self.device)
        e2 = torch.as_tensor(eps_cur, dtype=torch.float32).to(self.device).contiguous() if eps_cur is not None \
            else torch.randn(shape, device=self.device)
        call("sppSacAcmUpdate", self._h, ctypes.byref(b), ptr(e1), ptr(e2), ptr(self._losses), stream_handle())
        self._keep = (keep, e1, e2)  # inputs must outlive the async work

    def update_from_replay(self, idx, seed, counter):
        """Fused path: gather the sampled transitions on device and update with device eps."""
        idx = torch.as_tensor(idx, dtype=torch.int64).to(self.device).contiguous()
        self._stage(idx)
        call("sppSacAcmUpdateStaged", self._h, seed, counter, ptr(self._losses), stream_handle())

    def update_from_replay_dp(self, idx, seed, counter, allreduce=None, beside=None):
        """The same grad step split at its exchange points: allreduce(bucket) averages a
        flat gradient bucket across data-parallel ranks (RCCL) between grads and apply.  beside()
        enqueues independent work (the ACM step's gradients) under the actor bucket's exchange."""
        st = stream_handle()
        self._stage(idx)
        call("sppSacAcmDrawEps", self._h, seed, counter, st)
        call("sppSacAcmCriticGrads", self._h, None, None, ptr(self._losses), st)
        if allreduce is not None:
            allreduce(self.bucket_critic)
        call("sppSacAcmCriticApply", self._h, st)
        call("sppSacAcmActorGrads", self._h, None, ptr(self._losses), st)
        self._exchange(allreduce, self.bucket_actor, beside)
        call("sppSacAcmActorApply", self._h, ptr(self._losses), st)

    def _fused_update(self, idx, counter, allreduce=None, beside=None):
        self.update_from_replay_dp(idx, self._key_update, counter, allreduce, beside)

    def acm_update_from_replay(self, idx, x, y, loss, allreduce=None):
        """update_acm_batches body (acm.py:356-372) for one device-sampled batch."""
        st = stream_handle()
        B = idx.numel()
        call("sppReplayGatherAcm", self.replay_buffer._h, ptr(idx), B, ptr(x), ptr(y), st)
        call("sppAcmRegressGrads", self._h, ptr(x), ptr(y), B, ptr(loss), st)
        if allreduce is not None:
            allreduce(self.bucket_acm)
        call("sppAcmRegressApply", self._h, st)

    @property
    def loss(self):
        v = self._losses.detach().cpu().numpy()
        out = {"critic_1": float(v[0]), "critic_2": float(v[1]), "actor": float(v[2])}
        if self.custom_loss:
            out["sac"], out["dist"] = float(v[3]), float(v[4])
        return out

    @property
    def log_alpha(self):
        return float(self.alpha_state[0].item())

    def current_alpha(self):
        return float(self.alpha_state[3].item())

    # ------------------------------------------------------------------ ACM regression + acting
    def batch_update_acm(self, x, y):
        """AcMTrainer.batch_update (acm.py:246-258)."""
        x = torch.as_tensor(x, dtype=torch.float32).to(self.device).contiguous()
        y = torch.as_tensor(y, dtype=torch.float32).to(self.device).contiguous()
        loss = torch.zeros(1, device=self.device)
        call("sppAcmRegressStep", self._h, ptr(x), ptr(y), x.shape[0], ptr(loss), stream_handle())
        self._keep_acm = (x, y)
        return loss

    def act(self, obs, eps=None, noise=None, mode=1, act_noise=None):
        """noise_action + process_action for E observations (ddpg_acm.py:40-50, off_policy.py:89-106).
        Returns (target_state [E, aout], env_action [E, ac])."""
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
        # key order of the reference's dict (sac.py:287-296 + acm/off_policy/sac_acm.py collect_params_dict)
        return {"actor": self.net_state(_lib.SPP_NET_ACTOR), "critic_1": self.net_state(_lib.SPP_NET_CRITIC1),
                "critic_2": self.net_state(_lib.SPP_NET_CRITIC2),
                "obs_mean": rb.obs_mean.cpu(), "obs_std": rb.obs_std.cpu(),
                "min_obs": rb.min_obs.cpu() if rb._have_minmax else None,
                "max_obs": rb.max_obs.cpu() if rb._have_minmax else None,
                "acm": self.net_state(_lib.SPP_NET_ACM)}

    def apply_params_dict(self, d):
        for k, net in (("actor", _lib.SPP_NET_ACTOR), ("critic_1", _lib.SPP_NET_CRITIC1),
                       ("critic_2", _lib.SPP_NET_CRITIC2), ("acm", _lib.SPP_NET_ACM)):
            self.load_net(net, d[k])
        rb = self.replay_buffer
        rb.obs_mean.copy_(torch.as_tensor(d["obs_mean"]))
        rb.obs_std.copy_(torch.as_tensor(d["obs_std"]))
        if d.get("min_obs") is not None and d.get("max_obs") is not None:
            rb.min_obs.copy_(torch.as_tensor(d["min_obs"]))
            rb.max_obs.copy_(torch.as_tensor(d["max_obs"]))
            rb._have_minmax = True
