"""PPO_AcM: rltoolkit's SPP-PPO loop on the MI355X library, vectorized over E envs.

Mirrors rltoolkit/acm/on_policy.py (AcMOnPolicyTrainer / A2C_AcM / PPO_AcM) with
A2C (algorithms/a2c/a2c.py) and PPO (algorithms/ppo/ppo.py) underneath:

  collect_batch         a2c.py:144-184 + on_policy.py:32-50 (process_action: denormalise ->
                        AcM -> env), SURVEY.md §8a row a21
  update_critic         a2c.py:186-225 (critic_num_target_updates x num_critic_updates_per_target
                        full-batch steps), row a22
  calculate_gae         ppo.py:117-150 (device scan over [T][E] streams), row a23
  update_actor_acm      on_policy.py:164-216 + advantage_dataset.py:30-42 (clip loss, entropy,
                        custom dist loss on the buffer's (denormalised) actions, KL early stop), row a24
  update_acm(_batches)  acm.py:266-303, 356-372 every acm_update_freq iterations
  update_obs_mean_std   on the ACM ring when denormalize_actor_out (on_policy.py:70-71)
  pre_train             acm.py:234-244

Device pieces: actor / critic = ``OnPolicyNets`` (libspprl sppOnp*), GAE = sppGaeScan, the AcM
(64-32 tanh, basic_model.py:108-132) and its replay ring = the AcM half of an SPP agent handle
(sppPolicyAct mode 3 for the act, sppAcmRegress* for the regression, BufferAcMOffPolicy for the
ring).  Rollout memory is time-major [T][E] on device.

Vectorization: each iteration collects T = ceil(batch_size / E) steps of E lockstep envs
(N = T*E transitions); envs keep running across iterations and the last step of every
iteration is a truncation (end = 1, done = 0), so GAE bootstraps from V(s') there exactly as
the reference does at a time-limit end.  With E = 1 whole episodes are collected until
batch_size frames, as the reference does.
"""
import numpy as np
import torch

from . import config
from ._lib import call, ptr, stream_handle
from .onpolicy import OnPolicyNets
from .ppo import calculate_gae
from .sac_acm import SAC_AcM
from .dp import stream_key
from .trainer import StatsLogger, SynthVecEnv


class PPO_AcM:
    def __init__(self, env_name="HalfCheetah-v2", gamma=0.99, actor_lr=3e-4, critic_lr=3e-4, batch_size=2000,
                 ppo_batch_size=512, kl_div_threshold=0.1, max_ppo_epochs=10, entropy_coef=0.0, ppo_epsilon=0.2,
                 gae_lambda=0.95, critic_num_target_updates=10, num_critic_updates_per_target=10, normalize_adv=True,
                 custom_loss=0.1, norm_closs=config.NORM_CLOSS, min_max_denormalize=True, denormalize_actor_out=True,
                 acm_epochs=5, acm_batch_size=64, acm_update_freq=3, acm_lr=3e-4, acm_update_batches=None,
                 acm_pre_train_samples=100_000, acm_pre_train_epochs=5, acm_scheduler_step=config.ACM_SCHEDULER_STEP,
                 acm_scheduler_gamma=config.ACM_SCHEDULER_GAMMA, acm_keep_pretrain=True, acm_ring_size=None,
                 iterations=1001,
                 stats_freq=1, test_episodes=None, return_done=None, max_frames=None, n_envs=1, env=None,
                 env_spec=None, device="cuda", seed=None, loop_seed=0, epsilon=None, obs_norm=False,
                 rehearse_world=None, dp_update=None, comm=None, acm_ob_idx=None, **unused):
        # unknown keywords raise (the reference's MetaLearner takes no **kwargs, rl.py:17-26); `epsilon` is the
        # reference's name of the clip range (PPO.__init__, ppo.py:17), ppo_epsilon this class's older one
        config.check_kwargs("PPO_AcM", unused, config.ON_POLICY_NO_EFFECT_KWARGS)
        # obs_norm only sets ReplayBufferAcM.obs_norm (acm.py:127-139), read by the ring's normalize() and
        # _sample_batch (replay_buffer.py:77-81, 246-249), neither of which the on-policy loop calls: the rollout
        # normalises through its own Memory (a2c.py:165, on_policy.py:107-112) and the ACM trains on raw ring rows
        # (acm.py:273-282, replay_buffer.py:404-430).  Accepted; it changes nothing computed.
        self.obs_norm = bool(obs_norm)
        if epsilon is not None:
            ppo_epsilon = epsilon
        ob, ac, ac_high, max_ep = env_spec or config.ENV_SPECS[env_name]
        self.env_name, self.ob_dim, self.ac_dim = env_name, ob, ac
        self.device = torch.device(device)
        self.gamma, self.gae_lambda = gamma, gae_lambda
        self.batch_size, self.iterations, self.stats_freq = int(batch_size), int(iterations), int(stats_freq)
        self.test_episodes, self.return_done, self.max_frames = test_episodes, return_done, max_frames
        self.custom_loss, self.norm_closs = float(custom_loss), bool(norm_closs)
        self.min_max_denormalize, self.denormalize_actor_out = bool(min_max_denormalize), bool(denormalize_actor_out)
        self.acm_epochs, self.acm_update_freq, self.acm_update_batches = int(acm_epochs), acm_update_freq, \
            acm_update_batches
        self.actor_output_dim = ob
        lim = 1.0 if self.min_max_denormalize else float(config.MAX_ABS_OBS_VALUE)  # acm.py:102-108
        if env is None:
            env = SynthVecEnv(n_envs, ob, ac, max_episode_steps=max_ep, ac_high=ac_high, seed=loop_seed,
                              device=self.device)
        self.env = env
        self.n_envs = E = env.n
        self.T = 1 if E == 1 else max(1, -(-self.batch_size // E))
        Nmax = max(self.T * E, self.batch_size + (max_ep or 1000) if E == 1 else 0)
        from .dp import make_allreduce

        import torch.distributed as dist

        dp_world = dist.get_world_size() if make_allreduce() is not None else 1  # (union mode: world x N rows)
        # rehearse_world = W (measurement only, one process): the per-rank work of a W-rank job -- the ACM ring
        # written with W ranks' rows per iteration and, for the update, this rank's rollout with the global
        # minibatch split W ways (shard) or the rollout tiled W times, the union's shape (union)
        self.rehearse_world = int(rehearse_world or 0)
        dp_world = max(dp_world, self.rehearse_world)
        # data parallel update (dp_update): "shard" -- each rank updates on its own rollout with one gradient
        # all-reduce per critic / actor step (the reference's per-step losses are batch means, so equal shards
        # average to the union's gradient); "union" -- one all-gather of the rollouts per iteration and every rank
        # runs the whole update on the union (no per-step exchange, replicas equal one process on the union)
        import os

        self.dp_update = dp_update or os.environ.get("SPP_PPO_DP_UPDATE", "shard")
        if self.dp_update not in ("shard", "union"):
            raise ValueError("dp_update must be 'shard' or 'union', got %r" % (self.dp_update,))
        self.nets = OnPolicyNets(ob, ob, ac_lim=lim, actor_lr=actor_lr, critic_lr=critic_lr, ppo_epsilon=ppo_epsilon,
                                 entropy_coef=entropy_coef, gamma=gamma, gae_lambda=gae_lambda,
                                 critic_num_target_updates=critic_num_target_updates,
                                 num_critic_updates_per_target=num_critic_updates_per_target,
                                 max_ppo_epochs=max_ppo_epochs, ppo_batch_size=ppo_batch_size,
                                 kl_div_threshold=kl_div_threshold, normalize_adv=normalize_adv,
                                 max_batch=max((dp_world if self.dp_update == "union" else 1) * Nmax,
                                               ppo_batch_size),
                                 device=self.device, seed=seed, custom_loss=custom_loss)
        # the AcM and its replay ring (acm.py:127-141: size = pre-train samples * 1.1)
        ring = int(acm_ring_size or acm_pre_train_samples * 1.1)
        self.acm = SAC_AcM(env_name=env_name, env_spec=(ob, ac, ac_high, max_ep), acm_lr=acm_lr, buffer_size=ring,
                           max_batch=max(acm_batch_size, 64), min_max_denormalize=min_max_denormalize,
                           denormalize_actor_out=denormalize_actor_out, device=self.device, seed=seed, env=env,
                           acm_epochs=acm_epochs, acm_batch_size=acm_batch_size, acm_update_freq=1,
                           acm_update_batches=acm_update_batches, acm_pre_train_samples=acm_pre_train_samples,
                           acm_pre_train_epochs=acm_pre_train_epochs, acm_scheduler_step=acm_scheduler_step,
                           acm_scheduler_gamma=acm_scheduler_gamma, acm_keep_pretrain=acm_keep_pretrain,
                           acm_ob_idx=acm_ob_idx, loop_seed=loop_seed + 17)
        self.replay_buffer = self.acm.replay_buffer
        # Data parallel: the ACM ring is REPLICATED (every rank writes every rank's transitions, in rank
        # order, at the end of each iteration: ReplayBufferAcM.add_buffer, replay_buffer.py:284-297), so the
        # ACM epochs (acm.py:266-303) run on identical rings with one permutation stream and need no
        # per-batch collective, and the ring's obs statistics are global without a collective either.
        # Data parallel (self.dp: a process group with more than one rank, or SPP_DP_FORCE=1's one-rank rehearsal),
        # the on-policy update (acm/on_policy.py:72-75, a2c.py:186-225, ppo.py:152-192):
        #   "shard" (default) -- each rank's own rollout, one gradient all-reduce per critic / clip-loss step (on
        #     the communicator's compute stream when comm is passed), advantages normalised with global moments;
        #   "union" -- one all-gather of the rollouts per iteration ([T][world * E], rank-major along the env axis)
        #     and the persistent single-process launches on the identical union with one permutation stream.
        # Either way the replicas stay bit-identical.
        self.dp = self.nets.allreduce is not None or self.rehearse_world > 1
        self.world = dist.get_world_size() if self.nets.allreduce is not None else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        if self.dp_update == "union":
            self.nets.allreduce = self.nets.allreduce_sum = None  # (the nets see the union: no per-step exchange)
            self.nets.world = self.nets.shards = 1
        else:
            if comm is not None and self.nets.allreduce is not None:  # the per-step exchange on the compute stream
                inv = 1.0 / comm.world

                def allreduce(t):
                    comm.allreduce_sum(t)
                    t.mul_(inv)

                self.nets.allreduce, self.nets.allreduce_sum = allreduce, comm.allreduce_sum
                self.nets.grad_scale = inv
            # the global minibatch ppo_batch_size is split over the ranks (a rehearsal: over rehearse_world)
            self.nets.shards = max(self.world, self.rehearse_world)
        if self.world > 1 and E == 1:
            # one env per rank collects whole episodes: the ranks' ring-write records ("start" per episode)
            # then differ in count and kind, which the rank-major all-gather of _flush_ring cannot carry
            raise ValueError("PPO_AcM data parallel needs n_envs > 1 per rank (vectorized lockstep envs); "
                             "got n_envs = 1 with world = %d" % self.world)
        if self.dp:  # the replicated ring needs no gradient or statistics exchange either
            self.acm.allreduce = self.acm.allreduce_sum = self.acm.host_sum = None
        self.acm._perm_seed = int(seed or 0) * 7919 + 17  # rank-independent epoch permutations
        self._ring_log = []  # this iteration's ring writes (applied by _flush_ring)
        self._prev_all = None  # per rank: the ring slot of each env's last obs
        self.stats_logger = StatsLogger()
        self.iteration = 0
        self.loop_seed, self._ctr = int(loop_seed), 0
        self._key_policy = stream_key(loop_seed, "policy")
        self.loss = {}
        d = self.device
        self._ep_ret = torch.zeros(E, device=d)
        self._ret_sums = torch.zeros(2, dtype=torch.float64, device=d)
        self._obs = None
        self._prev_slots = None

    @property
    def kl_div_updates_counter(self):  # ppo.py:91, on_policy.py:216 (epochs + 1 per update_actor_acm)
        return self.nets.kl_div_updates_counter

    @kl_div_updates_counter.setter
    def kl_div_updates_counter(self, v):  # ppo.py:226 resets it after logging
        self.nets.kl_div_updates_counter = int(v)

    # ---------------------------------------------------------------- helpers
    def _randn(self, t):
        self._ctr += 1
        call("sppRandNormal", ptr(t), t.numel(), self._key_policy, self._ctr, stream_handle())
        return t

    def normalize(self, x):
        """MemoryAcM.normalize with the ring's statistics (memory.py:76-88)."""
        rb = self.replay_buffer
        if self.min_max_denormalize and not rb._have_minmax:
            return x.clone()  # the caller keeps it: never alias the env's double-buffered obs
        return rb._norm(x, 0)

    def denormalize(self, x):
        return self.replay_buffer._norm(x, 1)

    def process_action(self, action, norm_obs):
        """on_policy.py:32-50: denormalise (if denormalize_actor_out) -> AcM(cat(obs, a)) -> env action."""
        _, env_act = self.acm.act(norm_obs, eps=action, mode=3)
        return env_act

    # ---------------------------------------------------------------- RL.train / perform_iteration
    def pre_train(self):
        """acm.py:234-244.  Data parallel: the random-action samples of every rank go into every rank's
        ring (replicated, as the iteration's writes), then the same epochs run on every rank."""
        if self.world == 1:
            self.acm.pre_train()
            self._obs = None
            return
        acm, E = self.acm, self.n_envs
        obs = self.env.reset()
        self._ring_log.append(("start", obs.clone()))
        act = torch.empty(E, self.ac_dim, device=self.device)
        collected = 0
        while collected < acm.acm_pre_train_samples:  # AcMOffPolicy.collect_samples (off_policy.py:56-87)
            self.env.sample_actions(act)
            nobs, rew, end, end_dev = self.env.step(act)
            mask, robs = None, None
            if end.any():
                obs = self.env.reset(end)
                mask, robs = end.copy(), obs.clone()
            # the buffer's action slot holds the next obs; time-limit ends are kept as done
            self._ring_log.append(("step", nobs.clone(), rew.clone(), end_dev.clone(), end_dev.clone(), act.clone(),
                                   mask, robs))
            collected += E
        self._flush_ring()
        acm.update_acm(epochs=acm.acm_pre_train_epochs, pretrain=True)
        acm.update_obs_stats()
        if not acm.acm_keep_pretrain:
            self.replay_buffer.reset_idx()
        self._obs = None

    def train(self, iterations=None):
        if iterations:
            self.iterations += iterations
        while self.iteration < self.iterations:
            ret = self.perform_iteration()
            running = self.stats_logger.calc_running_return(ret)
            if self.return_done is not None and running is not None and running >= self.return_done:
                break
            if self.test_episodes and self.iteration % self.stats_freq == 0:
                self.stats_logger.test_return = self.test()
            self.iteration += 1
            if self.max_frames is not None and self.max_frames < self.stats_logger.frames:
                break
        return self.stats_logger.running_return

    def perform_iteration(self, sync=True):
        """on_policy.py:52-75.  Returns the mean return of the episodes completed (None if none).

        update(mem) (critic, GAE, actor) and update_acm touch disjoint networks and data: the ACM trains on
        the ring, already flushed by collect_batch, and nothing in update(mem) reads the ACM.  A single-process
        run therefore enqueues the ACM epochs on a side stream first and runs update(mem) beside them (the
        persistent critic / actor grids leave the ACM grid's workgroup slots free); the obs statistics and the
        next rollout wait for both, as in the reference's order.  The results are the serial order's."""
        self._ret_sums.zero_()
        mem = self.collect_batch()
        if self.dp and self.dp_update == "union":
            mem = self._union(mem)  # every rank's rollout, before the ACM's side stream starts
        acm_now = bool(self.acm_update_freq) and self.iteration % self.acm_update_freq == 0
        side = self._acm_side_stream() if acm_now else None
        if side is not None:
            ready = torch.cuda.Event()
            ready.record()
            side.wait_event(ready)
            self.nets.reserve_workgroups(self.acm.acm_sgd_workgroups())
            with torch.cuda.stream(side):
                self._update_acm()
            done = torch.cuda.Event()
            done.record(side)
            try:
                self.update(mem)
            finally:
                torch.cuda.current_stream().wait_event(done)
                self.nets.reserve_workgroups(0)
        else:
            self.update(mem)
            if acm_now:
                self._update_acm()
        if self.denormalize_actor_out:
            self.acm.update_obs_stats()
        if not sync:
            return None
        s = self._ret_sums.cpu().numpy()
        return float(s[0] / s[1]) if s[1] > 0 else None

    def _update_acm(self):
        if self.acm_update_batches:
            self.acm.update_acm_batches(self.acm_update_batches)
        else:
            self.acm.update_acm(self.acm_epochs)

    def _acm_side_stream(self):
        """The side stream of the concurrent ACM update, or None: CUDA device, persistent ACM SGD eligible (one
        launch per epoch), and the env var SPP_PPO_ACM_OVERLAP not 0.  Data parallel too: the iteration's
        collectives (the ring flush, the rollout union) are all issued before the side stream starts, and the
        ACM epochs themselves exchange nothing (replicated ring)."""
        import os

        if os.environ.get("SPP_PPO_ACM_OVERLAP", "1") == "0" or self.device.type != "cuda":
            return None
        if not self.acm._acm_sgd_ok(self.acm.acm_batch_size):
            return None
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    # ---------------------------------------------------------------- A2C.collect_batch
    def _start(self):
        self._obs = self.env.reset()
        self._ring_log.append(("start", self._obs.clone()))
        self._ep_ret.zero_()
        self._ep_len = np.zeros(self.n_envs, np.int64)

    # ---------------------------------------------------------------- the ACM ring (add_buffer)
    def _flush_ring(self):
        """Apply the iteration's ring writes (ReplayBufferAcM.add_buffer at the iteration's end,
        replay_buffer.py:284-297): locally, or -- data parallel -- every rank's writes in rank order
        after one all-gather of the iteration's records, so every rank holds the same ring."""
        log, self._ring_log = self._ring_log, []
        if not log:
            return
        E, ob, ac = self.n_envs, self.ob_dim, self.ac_dim
        W = self.world
        R = self.rehearse_world if W == 1 and self.rehearse_world > 1 else 1
        if self._prev_all is None:
            self._prev_all = [None] * max(W, R)
        if W == 1:
            # (a rehearsal of R ranks: the replicated ring takes R ranks' writes per iteration -- this rank's R times)
            blocks = [log] * R
        else:
            import torch.distributed as dist

            F = 2 * ob + ac + 4  # obs | rew | done | end | env action | reset obs | reset mask
            buf = torch.zeros(len(log), E, F, device=self.device)
            for i, rec in enumerate(log):
                if rec[0] == "start":
                    buf[i, :, :ob] = rec[1]
                else:
                    _, nobs, rew, done, end, act, mask, robs = rec
                    buf[i, :, :ob] = nobs
                    buf[i, :, ob] = rew
                    buf[i, :, ob + 1] = done.float()
                    buf[i, :, ob + 2] = end.float()
                    buf[i, :, ob + 3:ob + 3 + ac] = act
                    if mask is not None:
                        buf[i, :, ob + 3 + ac:2 * ob + 3 + ac] = robs
                        buf[i, :, 2 * ob + 3 + ac] = torch.from_numpy(mask.astype(np.float32)).to(self.device)
            allb = torch.empty(W * buf.shape[0], *buf.shape[1:], device=self.device)
            dist.all_gather_into_tensor(allb, buf)  # rank-major along dim 0
            allb = allb.view(W, *buf.shape)
            masks = allb[:, :, :, 2 * ob + 3 + ac].cpu().numpy() > 0.5  # one host copy for every rank's masks
            blocks = []
            for r in range(W):
                recs = []
                for i, rec in enumerate(log):
                    b = allb[r, i]
                    if rec[0] == "start":
                        recs.append(("start", b[:, :ob]))
                    else:
                        m = masks[r, i]
                        recs.append(("step", b[:, :ob], b[:, ob], b[:, ob + 1].to(torch.uint8),
                                     b[:, ob + 2].to(torch.uint8), b[:, ob + 3:ob + 3 + ac],
                                     m if m.any() else None, b[:, ob + 3 + ac:2 * ob + 3 + ac]))
                blocks.append(recs)
        rb = self.replay_buffer
        for r, recs in enumerate(blocks):
            prev = self._prev_all[r]
            for rec in recs:
                if rec[0] == "start":
                    prev = rb.add_obs_batch(rec[1])
                    continue
                _, nobs, rew, done, end, act, mask, robs = rec
                slots = rb.add_obs_batch(nobs)
                rb.add_timestep_batch(prev, slots, nobs, rew, done, end, act)  # ReplayBufferAcM ring
                prev = slots
                if mask is not None:
                    idx = np.flatnonzero(mask)
                    rs = rb.add_obs_batch(robs[torch.as_tensor(idx, device=self.device)])
                    prev = prev.copy()
                    prev[idx] = rs
            self._prev_all[r] = prev

    def collect_batch(self):
        """Rollout memory, time-major [T][E]: normalised obs, actions, log-probs, rewards, done,
        end, next obs (raw)."""
        E = self.n_envs
        if E == 1:  # whole episodes until batch_size frames (a2c.py:155-184)
            steps = []
            while sum(len(s) for s in steps) < self.batch_size:
                self.stats_logger.rollouts += 1
                self._start()
                seg, end = [], False
                while not end:
                    step = self._step()
                    end = bool(step[-1])
                    seg.append(step[:-1])
                steps.append(seg)
            flat = [x for s in steps for x in s]
        else:
            if self._obs is None:
                self._start()
                self.stats_logger.rollouts += E
            flat = [self._step()[:-1] for _ in range(self.T)]
        self._flush_ring()
        T = len(flat)
        cat = lambda k: torch.stack([f[k] for f in flat])  # noqa: E731
        mem = {"obs": cat(0), "act": cat(1), "lp": cat(2), "rew": cat(3), "done": cat(4), "end": cat(5),
               "next_obs": cat(6), "T": T}
        if E > 1:
            mem["end"][-1].fill_(1)  # segment truncation: GAE bootstraps from V(s') (ppo.py:136-148)
        self.stats_logger.frames += T * E
        return mem

    def _step(self):
        E, rb = self.n_envs, self.replay_buffer
        norm_obs = self.normalize(self._obs)
        eps = self._randn(torch.empty(E, self.actor_output_dim, device=self.device))
        act, lp = self.nets.act(norm_obs, eps)
        env_act = self.process_action(act, norm_obs)
        nobs, rew, end, end_dev = self.env.step(env_act)
        # a2c.py:168-171: end = env done; done = False when the episode hit max_ep_len (a time-limit end)
        self._ep_len += 1
        max_ep = getattr(self.env, "_max_episode_steps", None)
        done_h = end & (self._ep_len != max_ep) if max_ep else end.copy()
        self._ep_len[end] = 0
        done = (torch.from_numpy(done_h.astype(np.uint8)).to(self.device) if done_h.any()
                else torch.zeros(E, dtype=torch.uint8, device=self.device))
        any_end = bool(end.any())
        call("sppEpisodeAccum", ptr(rew), ptr(end_dev) if any_end else None, E, ptr(self._ep_ret),
             ptr(self._ret_sums), stream_handle())
        out = (norm_obs, act, lp, rew.clone(), done, end_dev.clone(), nobs.clone(), end.any() if E == 1 else False)
        self._obs = nobs
        mask, robs = None, None
        if any_end and E > 1:
            self.stats_logger.rollouts += int(end.sum())
            self._obs = self.env.reset(end)
            mask, robs = end.copy(), self._obs.clone()
        # ring writes of this step (applied at the iteration's end, _flush_ring)
        self._ring_log.append(("step", out[6], out[3], done, out[5], env_act.clone(), mask, robs))
        return out

    # ---------------------------------------------------------------- data parallel: the rollout union
    def _union(self, mem):
        """All-gather the ranks' rollouts [T][E] into the union [T][world * E] (rank-major along the env axis),
        in one collective of one packed tensor: normalised obs | action | log-prob | reward | done | end | next
        obs.  Every rank then holds the same batch."""
        import torch.distributed as dist

        if mem.get("union"):
            return mem
        T, E, ob, W = mem["T"], self.n_envs, self.ob_dim, self.world
        if self.rehearse_world > 1:  # (measurement: a W-rank union's shape from this rank's rollout)
            R = self.rehearse_world
            tile = lambda x: x.repeat(1, R, *([1] * (x.dim() - 2)))  # noqa: E731
            out = {k: tile(mem[k]) for k in ("obs", "act", "lp", "rew", "done", "end", "next_obs")}
            out.update(T=T, E=R * E, union=True)
            return out
        F = 3 * ob + 4
        pk = torch.empty(T, E, F, device=self.device)
        pk[:, :, :ob] = mem["obs"]
        pk[:, :, ob:2 * ob] = mem["act"]
        pk[:, :, 2 * ob] = mem["lp"]
        pk[:, :, 2 * ob + 1] = mem["rew"]
        pk[:, :, 2 * ob + 2] = mem["done"].float()
        pk[:, :, 2 * ob + 3] = mem["end"].float()
        pk[:, :, 2 * ob + 4:] = mem["next_obs"]
        allp = torch.empty(W, T, E, F, device=self.device)
        dist.all_gather_into_tensor(allp.view(W * T, E, F), pk.view(T, E, F))
        u = allp.permute(1, 0, 2, 3).reshape(T, W * E, F)  # [T][rank][env] -> [T][rank * E + env]
        return {"obs": u[:, :, :ob], "act": u[:, :, ob:2 * ob], "lp": u[:, :, 2 * ob].contiguous(),
                "rew": u[:, :, 2 * ob + 1].contiguous(), "done": u[:, :, 2 * ob + 2].to(torch.uint8),
                "end": u[:, :, 2 * ob + 3].to(torch.uint8), "next_obs": u[:, :, 2 * ob + 4:], "T": T, "E": W * E,
                "union": True}

    # ---------------------------------------------------------------- update (critic, GAE, actor)
    def update(self, mem):
        """critic, GAE, actor on the iteration's batch: this rank's rollout, or (data parallel) the union of every
        rank's (self._union; a caller may pass the union itself)."""
        if self.dp and self.dp_update == "union":
            mem = self._union(mem)
        T, E, ob = mem["T"], mem.get("E", self.n_envs), self.ob_dim
        N = T * E
        obs = mem["obs"].reshape(N, ob)
        nobs = self.normalize(mem["next_obs"].reshape(N, ob))
        rew, done = mem["rew"].reshape(N), mem["done"].reshape(N).float()
        self.nets.update_critic(obs, nobs, rew, done)  # a2c.py:186-225
        v = self.nets.value(obs).reshape(T, E)
        v_next = self.nets.value(nobs).reshape(T, E)
        _, adv = calculate_gae(mem["rew"].reshape(T, E), v, v_next, mem["done"].reshape(T, E),
                               mem["end"].reshape(T, E), self.gamma, self.gae_lambda)
        acts = mem["act"].reshape(N, ob)
        nxt = nobs
        if not self.norm_closs:  # on_policy.py:191-193
            nxt, acts = self.denormalize(nobs), self.denormalize(acts)
        self.nets.update_actor(adv.reshape(N), obs, acts, mem["lp"].reshape(N), nxt)
        self.loss.update(self.nets.loss)
        self.loss["acm"] = None

    # ---------------------------------------------------------------- test (a2c.py test)
    def test(self, episodes=None):
        episodes = episodes or self.test_episodes or 1
        env = self.env.spawn(episodes, seed=self.loop_seed + 99991)
        obs = env.reset()
        ret = torch.zeros(episodes, device=self.device)
        sums = torch.zeros(2, dtype=torch.float64, device=self.device)
        alive = np.ones(episodes, bool)
        while alive.any():
            n_obs = self.normalize(obs)
            act, _ = self.nets.act(n_obs, None)  # deterministic mean
            obs, rew, end, _ = env.step(self.process_action(act, n_obs))
            m = torch.as_tensor((end & alive).astype(np.uint8), device=self.device)
            call("sppEpisodeAccum", ptr(rew), ptr(m), episodes, ptr(ret), ptr(sums), stream_handle())
            alive &= ~end
            if end.any() and alive.any():
                obs = env.reset(end)
        s = sums.cpu().numpy()
        return float(s[0] / s[1])

    # ---------------------------------------------------------------- checkpoints (rl.py:263-301)
    def collect_params_dict(self):
        from .onpolicy import actor_layout, critic_layout
        from . import nets as _nets

        rb = self.replay_buffer
        return {"actor": _nets.state_dict(self.nets.params[0], actor_layout(self.ob_dim, self.ob_dim)),
                "critic": _nets.state_dict(self.nets.params[1], critic_layout(self.ob_dim)),
                "obs_mean": rb.obs_mean.cpu(), "obs_std": rb.obs_std.cpu(),
                "min_obs": rb.min_obs.cpu() if rb._have_minmax else None,
                "max_obs": rb.max_obs.cpu() if rb._have_minmax else None,
                "acm": self.acm.net_state(5)}

    def apply_params_dict(self, d):  # rl.py:263-279 + ACM (acm/on_policy.py)
        from .onpolicy import actor_layout, critic_layout
        from . import nets as _nets

        for i, (k, lay) in enumerate((("actor", actor_layout(self.ob_dim, self.ob_dim)),
                                      ("critic", critic_layout(self.ob_dim)))):
            _nets.load_state(self.nets.params[i], lay, d[k])
        self.acm.apply_params_dict({"actor": self.acm.net_state(0), "critic_1": self.acm.net_state(1),
                                    "critic_2": self.acm.net_state(2), "acm": d["acm"], "obs_mean": d["obs_mean"],
                                    "obs_std": d["obs_std"], "min_obs": d.get("min_obs"),
                                    "max_obs": d.get("max_obs")})

    def save(self, path):  # rl.py:281-292
        from .checkpoint import save_params

        save_params(path, self.collect_params_dict())

    def load(self, path):  # rl.py:294-301
        from .checkpoint import load_params

        self.apply_params_dict(load_params(path))
