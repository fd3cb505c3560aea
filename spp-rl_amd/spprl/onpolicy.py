"""On-policy (A2C / PPO / PPO_AcM) networks on the MI355X library.

``OnPolicyNets`` holds the reference's 64-wide tanh Actor / Critic
(rltoolkit/basic_model.py:7-76) as flat device buffers and mirrors the
pieces of A2C / PPO that touch them:
  value(x)                       critic(x)                          a2c.py:257-265
  update_critic(obs, next_obs, rew, done)
                                 A2C.update_critic: critic_num_target_updates x
                                 num_critic_updates_per_target full-batch steps   a2c.py:186-225
  update_actor(adv, obs, act, lp_old, next_obs)
                                 PPO.update_actor(_acm): minibatch epochs with KL early stop
                                                                    ppo.py:152-192, on_policy.py:164-216
  act(obs, eps)                  Actor.act (continuous)             basic_model.py:32-51
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib, nets, ppo
from ._lib import call, ptr, stream_handle
from .perm import device_randperm

H = 64


def actor_layout(ob, aout):
    return [("log_scale", (aout,)), ("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)),
            ("fc2.bias", (H,)), ("fc3.weight", (aout, H)), ("fc3.bias", (aout,))]


def critic_layout(ob):
    return [("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc3.weight", (1, H)), ("fc3.bias", (1,))]


class OnPolicyNets:
    def __init__(self, ob, aout, ac_lim=1.0, actor_lr=3e-3, critic_lr=3e-4, ppo_epsilon=0.2, entropy_coef=0.0,
                 gamma=0.99, gae_lambda=0.95, critic_num_target_updates=10, num_critic_updates_per_target=10,
                 max_ppo_epochs=50, ppo_batch_size=1000, kl_div_threshold=0.15, normalize_adv=True,
                 max_batch=4096, device="cuda", seed=None, custom_loss=0.0):
        _lib.load()
        self.ob, self.aout, self.device = ob, aout, torch.device(device)
        self.gamma, self.gae_lambda = gamma, gae_lambda
        self.critic_num_target_updates, self.num_critic_updates_per_target = (critic_num_target_updates,
                                                                              num_critic_updates_per_target)
        self.max_ppo_epochs, self.ppo_batch_size, self.kl_div_threshold = max_ppo_epochs, ppo_batch_size, kl_div_threshold
        self.normalize_adv = normalize_adv
        self.entropy_coef, self.custom_loss = float(entropy_coef), float(custom_loss)
        self.kl_div_updates_counter = 0  # ppo.py:91, += epochs + 1 of each update_actor (ppo.py:192)
        # the device permutations of the minibatch epochs: seed from ``seed`` or torch's global generator
        self._perm_seed = seed if seed is not None else int(torch.randint(0, 2**62, (1,)).item())
        self._perm_ctr = 0
        self.max_batch = int(max_batch)
        cfg = _lib.OnPolicyConfig(ob, aout, actor_lr, critic_lr, ppo_epsilon, entropy_coef, self.max_batch)
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        call("sppOnpCreate", ctypes.byref(h), ctypes.byref(cfg), dev)
        self._h = h
        gen = torch.Generator().manual_seed(seed) if seed is not None else None
        self.layouts = [actor_layout(ob, aout), critic_layout(ob)]
        self.params, self.grads, self.m, self.v = [], [], [], []
        for net, lay in enumerate(self.layouts):
            n = ctypes.c_int64()
            call("sppOnpNetSize", self._h, net, ctypes.byref(n))
            assert n.value == nets.numel(lay)
            p = torch.empty(n.value, device=self.device)
            if net == 0:
                nets.linear_init_(p[aout:], lay[1:], gen)
                p[:aout].fill_(-1.34)  # log_scale init, basic_model.py:18-20
            else:
                nets.linear_init_(p, lay, gen)
            self.params.append(p)
            for lst in (self.grads, self.m, self.v):
                lst.append(torch.zeros(n.value, device=self.device))
            call("sppOnpBindNet", self._h, net, ptr(p), ptr(self.grads[net]), ptr(self.m[net]), ptr(self.v[net]))
        lim = np.full(aout, float(ac_lim), np.float32) if np.ndim(ac_lim) == 0 else np.asarray(ac_lim, np.float32)
        call("sppOnpSetLimits", self._h, lim.ctypes.data_as(ctypes.c_void_p))
        self.loss = {}
        # data parallel (one process per GPU, equal shards): gradient averaging and global sums
        from .dp import make_allreduce, make_allreduce_sum

        self.allreduce, self.allreduce_sum = make_allreduce(), make_allreduce_sum()
        self.world = torch.distributed.get_world_size() if self.allreduce is not None else 1
        self.grad_scale = 1.0 / self.world  # (the fused data-parallel steps write their gradients times this)
        self.shards = self.world  # ranks the global minibatch ppo_batch_size is split over

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sppOnpDestroy(h)
            self._h = None

    def _dev(self, x):
        return torch.as_tensor(x, dtype=torch.float32).to(self.device).contiguous()

    def load_net(self, net, flat):
        self.params[net].copy_(self._dev(flat).reshape(-1))

    # ------------------------------------------------------------------ critic
    def value(self, x):
        x = self._dev(x)
        v = torch.empty(x.shape[0], device=self.device)
        call("sppOnpValue", self._h, ptr(x), x.shape[0], ptr(v), stream_handle())
        self._keep = x
        return v

    def critic_step(self, x, q):
        x, q = self._dev(x), self._dev(q).reshape(-1)
        loss = torch.zeros(1, device=self.device)
        if self.allreduce is not None and self._critic_grads_fused_ok(x.shape[0]):
            # data parallel: the persistent kernel's gradient of this step (one launch, its workgroups' partial
            # gradients summed in a fixed order, written times 1 / ranks) instead of the phase kernel + dW launches
            # of sppOnpCriticGrads; the average is then the plain all-reduce sum
            call("sppOnpCriticStepGrads", self._h, ptr(x), ptr(q), x.shape[0], ptr(loss), self.grad_scale,
                 stream_handle())
            self.allreduce_sum(self.grads[1])
        else:
            call("sppOnpCriticGrads", self._h, ptr(x), ptr(q), x.shape[0], ptr(loss), stream_handle())
            if self.allreduce is not None:  # data parallel: average the critic gradient (RCCL)
                self.allreduce(self.grads[1])
        call("sppOnpCriticApply", self._h, stream_handle())
        self._keep = (x, q)
        return loss

    def update_critic(self, obs, next_obs, rew, done):
        """A2C.update_critic (a2c.py:186-225); returns the advantages of calculate_advantage.  Single-process
        runs make each target's num_critic_updates_per_target full-batch steps in one persistent launch
        (sppOnpCriticSteps); data-parallel ranks all-reduce every step's gradient (critic_step)."""
        obs, next_obs, rew, done = (self._dev(t) for t in (obs, next_obs, rew, done))
        total = torch.zeros(1, device=self.device)
        one_launch = self._critic_kernel_ok(obs.shape[0])
        for _ in range(self.critic_num_target_updates):
            vn = self.value(next_obs)
            q = (rew + self.gamma * (1 - done) * vn).contiguous()
            if one_launch:
                call("sppOnpCriticSteps", self._h, ptr(obs), ptr(q), obs.shape[0], self.num_critic_updates_per_target,
                     ptr(total), stream_handle())
                self._keep_crit = (obs, q)
                continue
            for _ in range(self.num_critic_updates_per_target):
                total += self.critic_step(obs, q)
        if one_launch or (self.allreduce is not None and self._critic_grads_fused_ok(obs.shape[0])):
            self._sync_flag_copy()  # (the persistent launches' timeout flag: sppOnpCriticSteps / StepGrads)
        self.loss["critic"] = float(total.item()) / (self.critic_num_target_updates *
                                                     self.num_critic_updates_per_target)
        self._sync_check()
        with torch.no_grad():
            q = rew + self.gamma * (1 - done) * self.value(next_obs)
            return q - self.value(obs)

    # ------------------------------------------------------------------ actor
    def actor_step(self, x, act, lp_old, adv, next_obs=None, out=None):
        """One minibatch step; ``out`` (4 floats: actor loss, KL, dist, entropy) is written, not
        accumulated, so a caller may hand in rows of a preallocated [steps][4] buffer."""
        x, act, lp_old, adv = (self._dev(t) for t in (x, act, lp_old, adv))
        nxt = self._dev(next_obs) if next_obs is not None else None
        if out is None:
            out = torch.empty(4, device=self.device)
        call("sppOnpActorGrads", self._h, ptr(x), ptr(act), ptr(lp_old.reshape(-1)), ptr(adv.reshape(-1)), ptr(nxt),
             x.shape[0], ptr(out), stream_handle())
        if self.allreduce is not None:  # average the actor gradient and the loss / KL partials
            self.allreduce(self.grads[0])
            self.allreduce(out)
        call("sppOnpActorApply", self._h, stream_handle())
        self._keep = (x, act, lp_old, adv, nxt)
        return out

    def actor_step_fused(self, obs, act, lp_old, adv, nxt, idx, out):
        """One minibatch step (the rows idx of obs / act / lp_old / adv / nxt) through sppOnpActorStepGrads, the
        gradient (and out's 4 partials) all-reduced, then Adam: the data-parallel actor_step."""
        call("sppOnpActorStepGrads", self._h, ptr(obs), ptr(act), ptr(lp_old), ptr(adv), ptr(nxt), ptr(idx),
             idx.shape[0], ptr(out), self.grad_scale, stream_handle())
        if self.allreduce_sum is not None:  # (written times 1 / ranks: the sum is the average)
            self.allreduce_sum(self.grads[0])
            self.allreduce_sum(out)
        call("sppOnpActorApply", self._h, stream_handle())
        return out

    def update_actor(self, advantages, obs, actions, logprobs, next_obs=None, generator=None):
        """PPO minibatch epochs with the KL early stop (ppo.py:152-192); minibatches are a
        random permutation per epoch like the reference's DataLoader(shuffle=True)."""
        adv = self._dev(advantages).reshape(-1)
        if self.normalize_adv:
            if self.allreduce_sum is not None:  # global moments over the ranks' shards
                sums = torch.zeros(2, dtype=torch.float64, device=self.device)
                call("sppAdvSums", ptr(adv), adv.numel(), ptr(sums), stream_handle())
                self.allreduce_sum(sums)
                out = torch.empty_like(adv)
                call("sppAdvNormalizeGlobal", ptr(adv), adv.numel(), ptr(sums), adv.numel() * self.world, ptr(out),
                     stream_handle())
                adv = out
            else:
                adv = ppo.normalize_advantages(adv)
        obs, actions, logprobs = self._dev(obs), self._dev(actions), self._dev(logprobs).reshape(-1)
        nxt = self._dev(next_obs) if next_obs is not None else None
        N = obs.shape[0]
        kl, i = 0.0, 0
        sums = torch.zeros(4, device=self.device)
        self.last_epochs = 0
        mb = max(1, self.ppo_batch_size // self.shards)  # global minibatch = ppo_batch_size
        one_launch = self._epoch_kernel_ok(mb)
        # One-launch epochs keep the device busy across the epoch loop's one host round trip (the KL early stop):
        # the epoch's KL goes to pinned memory by an async copy behind the launch, and the next epoch's permutation
        # (it does not depend on the KL) is enqueued before the host waits for that copy, so its sort runs while the
        # host wakes up instead of after the next launch.  Permutation k uses counter (_perm_ctr + 1 + k) * N, as
        # when each epoch drew its own; the counter advances by the epochs run, so a permutation drawn ahead for an
        # epoch the KL stop skipped is never used and the sequence is the same.
        ahead = generator is None and one_launch
        nxt_perm = device_randperm(N, self._perm_seed, (self._perm_ctr + 1) * N, self.device) if ahead else None
        if ahead and getattr(self, "_kl_host", None) is None:
            self._kl_host = torch.zeros(1).pin_memory()
        for i in range(self.max_ppo_epochs):
            if kl >= self.kl_div_threshold:
                break
            self.last_epochs += 1
            # a CPU generator (tests) keeps its host permutation; by default the permutation is drawn on the
            # device by sppRandPerm (a host randperm + copy, or torch.randperm on the device, would stall the
            # stream every epoch)
            if generator is not None:
                perm = torch.randperm(N, generator=generator).to(self.device)
            elif ahead:
                perm = nxt_perm
            else:
                self._perm_ctr += 1
                perm = device_randperm(N, self._perm_seed, self._perm_ctr * N, self.device)
            outs = torch.empty(-(-N // mb), 4, device=self.device)  # one row per minibatch step
            if one_launch:  # the whole epoch in one persistent launch (the ragged last minibatch included)
                call("sppOnpActorEpoch", self._h, ptr(obs), ptr(actions), ptr(logprobs), ptr(adv), ptr(nxt),
                     ptr(perm), N, mb, ptr(outs), stream_handle())
                if ahead:
                    self._kl_host.copy_(outs[-1, 1:2], non_blocking=True)
                self._sync_flag_copy()
                self._keep = (obs, actions, logprobs, adv, nxt, perm, outs)
            elif self._actor_grads_fused_ok(mb):
                # data parallel: each minibatch step's gradient from the epoch kernel run for that one step, its
                # rows read through the permutation slice (no permuted copies, no phase-kernel + dW launches)
                for k, s in enumerate(range(0, N, mb)):
                    self.actor_step_fused(obs, actions, logprobs, adv, nxt, perm[s:s + mb], out=outs[k])
                self._sync_flag_copy()
                self._keep = (obs, actions, logprobs, adv, nxt, perm, outs)
            else:
                # one permuted copy per epoch: every minibatch is then a contiguous slice
                o_p, a_p, l_p, d_p = obs[perm], actions[perm], logprobs[perm], adv[perm]
                n_p = nxt[perm] if nxt is not None else None
                for k, s in enumerate(range(0, N, mb)):
                    e = s + mb
                    self.actor_step(o_p[s:e], a_p[s:e], l_p[s:e], d_p[s:e], n_p[s:e] if n_p is not None else None,
                                    out=outs[k])
            sums += outs.sum(0)
            if ahead:
                if i + 1 < self.max_ppo_epochs:
                    nxt_perm = device_randperm(N, self._perm_seed, (self._perm_ctr + 2 + i) * N, self.device)
                self._sync_check()  # waits for the event behind the KL copy, not for the permutation drawn ahead
                kl = float(self._kl_host[0])  # KL of the epoch's last minibatch (ppo.py:188)
            else:
                kl = float(outs[-1, 1].item())
                self._sync_check()
        if ahead:
            self._perm_ctr += self.last_epochs
        # the reference divides by i + 1 after the loop: the epochs run when none stopped early, one more than
        # that when the KL check broke the loop (on_policy.py:210-216, ppo.py:190-192)
        s = sums.cpu().numpy().astype(np.float64)
        d = float(i + 1)
        self.loss.update(actor=s[0] / d, entropy=s[3] / d, kl=kl)
        if nxt is not None:  # PPO_AcM: dist = mse(actions, next_obs) (data only: no gradient), and
            # policy = actor - entropy_coef * entropy + custom_loss * dist per minibatch (on_policy.py:188-207)
            self.loss.update(dist=s[2] / d, policy=(s[0] - self.entropy_coef * s[3] + self.custom_loss * s[2]) / d)
        self.kl_div_updates_counter += i + 1
        return kl

    def reserve_workgroups(self, n):
        """Size the persistent critic / actor grids for n workgroup slots taken by a concurrent persistent
        launch on another stream (sppOnpReserveWorkgroups); 0 restores the whole device."""
        call("sppOnpReserveWorkgroups", self._h, int(n))
        self._critic_max_n = self._epoch_max_bs = None
        self._reserved = int(n)

    def _critic_grads_fused_ok(self, n):
        """sppOnpCriticStepGrads takes batches the persistent critic grid covers, while no persistent grid runs
        beside it (the iterations with the ACM epochs on the side stream keep the phase-kernel path: a second
        persistent grid per step starved the ACM grid's arrival waits at the world-8 rehearsal shape, 132 + 103
        workgroups); SPP_ONP_FUSED_GRADS=0: the phase-kernel path always (A/B switch)."""
        if os.environ.get("SPP_ONP_FUSED_GRADS", "1") == "0" or getattr(self, "_reserved", 0) or \
                self.allreduce_sum is None:
            return False
        if getattr(self, "_critic_max_n", None) is None:
            self._critic_max_n = int(_lib.load().sppOnpCriticStepsMaxBatch(self._h))
        return n <= self._critic_max_n

    def _actor_grads_fused_ok(self, mb):
        """sppOnpActorStepGrads for the data-parallel minibatch steps: minibatches whose workgroups are all
        co-resident, while no persistent grid runs beside them (as _critic_grads_fused_ok)."""
        if self.allreduce_sum is None or os.environ.get("SPP_ONP_FUSED_GRADS", "1") == "0" or getattr(self, "_reserved", 0):
            return False
        if getattr(self, "_epoch_max_bs", None) is None:
            self._epoch_max_bs = int(_lib.load().sppOnpActorEpochMaxBatch(self._h))
        return mb <= self._epoch_max_bs

    def _critic_kernel_ok(self, n):
        """The persistent critic steps run single-process batches the co-resident grid covers in <= 8 passes."""
        if self.allreduce is not None:
            return False
        if getattr(self, "_critic_max_n", None) is None:
            self._critic_max_n = int(_lib.load().sppOnpCriticStepsMaxBatch(self._h))
        return n <= self._critic_max_n

    def _epoch_kernel_ok(self, mb):
        """The one-launch epoch (sppOnpActorEpoch) runs single-process epochs of these dims whose minibatch
        workgroups are all co-resident; data-parallel ranks all-reduce each minibatch gradient instead."""
        if self.allreduce is not None:
            return False
        if getattr(self, "_epoch_max_bs", None) is None:
            self._epoch_max_bs = int(_lib.load().sppOnpActorEpochMaxBatch(self._h))
        return mb <= self._epoch_max_bs

    def _sync_flag_copy(self):
        """Enqueue a copy of the persistent launches' timeout flag (sppOnpSyncStatusAsync) into pinned memory on
        the current stream; _sync_check reads it once the stream has passed that point."""
        if getattr(self, "_sync_flag", None) is None:
            self._sync_flag = torch.zeros(1, dtype=torch.int32).pin_memory()
        call("sppOnpSyncStatusAsync", self._h, self._sync_flag.data_ptr(), stream_handle())
        self._sync_ev = torch.cuda.Event()
        self._sync_ev.record()

    def _sync_check(self):
        """Raise SppError if a multi-workgroup sppOnpCriticSteps / sppOnpActorEpoch launch timed out at an arrival
        barrier (its parameters are then invalid).  Called right after the host synchronisation the update makes
        anyway (the critic loss, each epoch's KL), which the flag copy precedes on the stream: no extra wait."""
        ev = getattr(self, "_sync_ev", None)
        if ev is None:
            return
        ev.synchronize()
        self._sync_ev = None
        if int(self._sync_flag[0]):
            raise _lib.SppError("sppOnpCriticSteps / sppOnpActorEpoch: a multi-workgroup step timed out at its arrival "
                                "barrier; the critic / actor parameters are invalid")

    def check_actor_epochs(self):
        """Raise if a multi-workgroup sppOnpActorEpoch launch timed out at an arrival barrier."""
        flag = np.zeros(1, np.int32)
        call("sppOnpActorEpochStatus", self._h, flag.ctypes.data_as(ctypes.c_void_p))
        if flag[0]:
            raise _lib.SppError("sppOnpActorEpoch: a step timed out at its arrival barrier; actor parameters invalid")

    def act(self, obs, eps=None):
        """Actor.act: (action, log_prob); eps None -> deterministic mean."""
        x = self._dev(obs)
        N = x.shape[0]
        a = torch.empty(N, self.aout, device=self.device)
        lp = torch.empty(N, device=self.device)
        e = self._dev(eps) if eps is not None else None
        call("sppOnpAct", self._h, ptr(x), N, ptr(e), ptr(a), ptr(lp), stream_handle())
        self._keep = (x, e)
        return a, lp
