"""Vectorized rollout -> HBM replay -> update loop (the callers either side of the update).

Mirrors the reference's control plane for the SPP off-policy agents, batched over
E lockstep env instances per GPU:

  RL.train                      rltoolkit/rl.py:192-229        -> OffPolicyLoop.train
  DDPG.perform_iteration        algorithms/ddpg/ddpg.py:159-170 -> perform_iteration
  DDPG.collect_batch_and_train  ddpg.py:182-223                -> collect_batch_and_train
  DDPG(_AcM).make_update        ddpg.py:225-237, acm/off_policy/ddpg_acm.py:52-85
  AcMTrainer.pre_train          acm/acm.py:234-244 (+ AcMOffPolicy.collect_samples, off_policy.py:56-87)
  AcMTrainer.update_acm         acm.py:266-303 (shuffled full-buffer epochs, StepLR)
  AcMTrainer.update_acm_batches acm.py:356-372
  DDPG.test                     ddpg.py:385-410
  StatsLogger                   stats_logger.py:9-26

Two schedules:
  * "reference" (E == 1): the reference cadence frame by frame -- grad_steps updates of
    update_batch_size samples every update_freq frames, indices from numpy's global
    MT19937 stream (np.random.randint, replay_buffer.py:234), episodes run to their end
    inside an iteration.
  * "fused" (E > 1): each vector step of E frames does one grad step on
    rho*E device-sampled transitions, rho = update_batch_size*grad_steps/update_freq, and
    (acm_update_batches mode) one ACM step on sigma*E samples, sigma =
    acm_update_batches*acm_batch_size/acm_update_freq.  FLOPs per env-step equal the
    reference's.  With a host (CPU) env the update of step t is enqueued before the CPU
    envs step, so GPU work overlaps the simulator ("pipelined": the update sees the
    transitions up to t-1).

Envs: ``SynthVecEnv`` (SURVEY.md Appendix A dynamics, on device) or ``HostVecEnv``
(gym-style envs stepped on the host CPU -- MuJoCo when available -- with pinned staging
buffers and H2D/D2H copies on a side stream).  Everything device-side runs in
libspprl.so; this module only sequences calls.
"""
import ctypes
import os
import time

import numpy as np
import torch

from . import config
from ._lib import SppError, call, load, ptr, stream_handle
from .perm import device_randperm
from .dp import make_allgather, make_allreduce, make_allreduce_sum, make_host_allreduce_sum, stream_key

# ---------------------------------------------------------------- stats


class StatsLogger:
    """rltoolkit/stats_logger.py:9-26 (running return with alpha = 0.9)."""

    def __init__(self, alpha=0.9):
        self.running_return = None
        self.test_return = None
        self._alpha = 0.9  # the reference ignores its argument (stats_logger.py:13)
        self.frames = 0
        self.rollouts = 0
        self.time_list = []
        self.stats = []

    def calc_running_return(self, new_mean_return):
        if new_mean_return is None:
            return self.running_return
        if self.running_return is None:
            self.running_return = new_mean_return
        else:
            self.running_return *= self._alpha
            self.running_return += (1 - self._alpha) * new_mean_return
        return self.running_return


# ---------------------------------------------------------------- envs


class SynthVecEnv:
    """E SynthEnv instances stepped in lockstep on device:
    s' = tanh(A s) + 0.1 resize(a, ob), r = -|a|^2 + s'[0], episodes of ``max_episode_steps``.
    ``A`` is shared (seeded by ``dyn_seed``) so data-parallel ranks simulate the same MDP."""

    is_host = False

    def __init__(self, n_envs, ob, ac, max_episode_steps=1000, ac_high=1.0, seed=0, dyn_seed=1234, device="cuda"):
        self.n, self.ob, self.ac = int(n_envs), int(ob), int(ac)
        self.device = torch.device(device)
        self._max_episode_steps = int(max_episode_steps)
        g = torch.Generator(device="cpu").manual_seed(dyn_seed)
        self.A = (torch.randn(ob, ob, generator=g) * 0.05).to(self.device)
        self.ac_low = torch.full((ac,), -float(ac_high), device=self.device)
        self.ac_high = torch.full((ac,), float(ac_high), device=self.device)
        self.seed, self._ctr = int(seed), 0
        self._key_reset, self._key_action = stream_key(seed, "env"), stream_key(seed, "env_action")
        self.obs = torch.empty(self.n, ob, device=self.device)
        self.nobs = torch.empty(self.n, ob, device=self.device)
        self.rew = torch.empty(self.n, device=self.device)
        self.end_dev = torch.empty(self.n, dtype=torch.uint8, device=self.device)
        self.t = 0

    def _next(self):
        self._ctr += 1
        return self._ctr

    def reset(self, mask=None):
        """Reset all envs (mask None) or those with mask[e]; returns the device obs [E, ob]."""
        m = None
        if mask is not None:
            m = torch.as_tensor(np.asarray(mask, np.uint8)).to(self.device)
        call("sppSynthEnvReset", ptr(self.obs), ptr(m), self.n, self.ob, self._key_reset, self._next(),
             stream_handle())
        self._keep = m
        if mask is None:
            self.t = 0
        return self.obs

    def step(self, action):
        """action [E, ac] device -> (next_obs [E, ob], rew [E], end host bool [E], end device u8 [E])."""
        call("sppSynthEnvStep", ptr(self.A), ptr(self.obs), ptr(action), self.n, self.ob, self.ac, ptr(self.nobs),
             ptr(self.rew), stream_handle())
        self.obs, self.nobs = self.nobs, self.obs
        self.t += 1
        end = self.t >= self._max_episode_steps
        self.end_dev.fill_(1 if end else 0)
        if end:
            self.t = 0
        return self.obs, self.rew, np.full(self.n, end), self.end_dev

    def sample_actions(self, out):
        """action_space.sample() for every env, on device (pre-train collector)."""
        call("sppRandUniform", ptr(out), out.numel(), ptr(self.ac_low), ptr(self.ac_high), self.ac, self._key_action,
             self._next(), stream_handle())
        return out

    def spawn(self, n_envs, seed):
        return SynthVecEnv(n_envs, self.ob, self.ac, self._max_episode_steps, float(self.ac_high[0]), seed=seed,
                           device=self.device)


class HostVecEnv:
    """gym-style envs stepped on the host CPU (MuJoCo when installed).

    Actions go device -> pinned host on a side stream; observations/rewards come back
    pinned host -> device on the same side stream; the compute stream waits on an event,
    so the copies overlap whatever the compute stream has queued (the update).

    The pinned staging is a ring of ``n_stage`` buffer sets, each with the event of the
    upload that last read it: the host only writes a set once that upload has completed,
    so a queued (not yet executed) H2D copy never sees the next step's or a reset's rows."""

    is_host = True

    def __init__(self, envs, device="cuda", env_fn=None, n_stage=4):
        self.env_fn = env_fn
        self.envs = list(envs)
        e0 = self.envs[0]
        self._init_staging(len(self.envs), int(np.prod(e0.observation_space.shape)),
                           int(np.prod(e0.action_space.shape)), getattr(e0, "_max_episode_steps", None), device,
                           n_stage)

    def _init_staging(self, n, ob, ac, max_episode_steps, device, n_stage):
        self.n, self.ob, self.ac = int(n), int(ob), int(ac)
        self._max_episode_steps = max_episode_steps
        self.device = torch.device(device)
        self.side = torch.cuda.Stream(device=self.device)
        pin = dict(pin_memory=True)
        self._stage = [(torch.zeros(self.n, self.ob, **pin), torch.zeros(self.n, **pin),
                        torch.zeros(self.n, dtype=torch.uint8, **pin)) for _ in range(int(n_stage))]
        self._stage_ev = [None] * len(self._stage)
        self._cur = 0
        self.h_act = torch.empty(self.n, self.ac, **pin)
        self.obs = torch.empty(self.n, self.ob, device=self.device)
        self.rew = torch.empty(self.n, device=self.device)
        self.end_dev = torch.empty(self.n, dtype=torch.uint8, device=self.device)
        self._act_ev = torch.cuda.Event()
        self._pending = False

    def _writable(self, carry):
        """Advance to the next staging set, wait for its last upload, and (carry) copy the
        current set's rows into it (a partial reset keeps the other envs' observations)."""
        prev = self._stage[self._cur]
        self._cur = (self._cur + 1) % len(self._stage)
        ev = self._stage_ev[self._cur]
        if ev is not None:
            ev.synchronize()
        cur = self._stage[self._cur]
        if carry:
            for dst, src in zip(cur, prev):
                dst.copy_(src)
        return cur

    def _upload(self):
        h_obs, h_rew, h_end = self._stage[self._cur]
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.side):
            self.side.wait_stream(main)  # do not overwrite obs still being read by queued kernels
            self.obs.copy_(h_obs, non_blocking=True)
            self.rew.copy_(h_rew, non_blocking=True)
            self.end_dev.copy_(h_end, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.side)
        self._stage_ev[self._cur] = ev
        main.wait_stream(self.side)

    def reset(self, mask=None):
        h_obs, _, _ = self._writable(carry=mask is not None)
        idx = np.arange(self.n) if mask is None else np.flatnonzero(mask)
        self._reset_rows(idx, h_obs)
        self._upload()
        return self.obs

    def _reset_rows(self, idx, h_obs):
        for e in idx:
            h_obs[e] = torch.as_tensor(np.asarray(self.envs[e].reset(), np.float32).reshape(-1))

    def _step_rows(self, act, h_obs, h_rew):
        end = np.zeros(self.n, bool)
        for e, env in enumerate(self.envs):
            o, r, d, _ = env.step(act[e])
            h_obs[e] = torch.as_tensor(np.asarray(o, np.float32).reshape(-1))
            h_rew[e] = float(r)
            end[e] = bool(d)
        return end

    def send(self, action):
        """Start the D2H copy of the actions (non-blocking)."""
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.side):
            self.side.wait_stream(main)
            self.h_act.copy_(action, non_blocking=True)
            self._act_ev.record(self.side)
        self._pending = True

    def recv(self):
        self._act_ev.synchronize()
        self._pending = False
        act = self.h_act.numpy()
        h_obs, h_rew, h_end = self._writable(carry=False)
        end = self._step_rows(act, h_obs, h_rew)
        h_end.copy_(torch.from_numpy(end.astype(np.uint8)))
        self._upload()
        return self.obs, self.rew, end, self.end_dev

    def step(self, action):
        self.send(action)
        return self.recv()

    def spawn(self, n_envs, seed):
        if self.env_fn is None:
            raise NotImplementedError("HostVecEnv.spawn needs env_fn")
        return HostVecEnv([self.env_fn() for _ in range(n_envs)], self.device, self.env_fn)

    def sample_actions(self, out):
        a = np.stack([np.asarray(env.action_space.sample(), np.float32).reshape(-1) for env in self.envs])
        out.copy_(torch.from_numpy(a))
        return out


class HostSynthEnv(HostVecEnv):
    """E SynthEnv instances (SURVEY.md Appendix A dynamics, as SynthVecEnv) stepped on the HOST in
    one vectorised numpy call per step -- the stand-in for a CPU simulator pool (MuJoCo is not in
    this image) behind HostVecEnv's pinned staging and side-stream copies, so the loop measures the
    host-env boundary: D2H actions, the host step overlapped with the queued update, H2D obs."""

    def __init__(self, n_envs, ob, ac, max_episode_steps=1000, ac_high=1.0, seed=0, dyn_seed=1234, device="cuda",
                 n_stage=4):
        self.envs, self.env_fn = [], None
        self._init_staging(n_envs, ob, ac, int(max_episode_steps), device, n_stage)
        g = torch.Generator(device="cpu").manual_seed(dyn_seed)
        self.A = (torch.randn(ob, ob, generator=g) * 0.05).numpy()
        self.ac_high = float(ac_high)
        self._rng = np.random.RandomState(seed)
        self._s = np.zeros((self.n, ob), np.float32)
        self._t = np.zeros(self.n, np.int64)
        self._seed = seed

    def _reset_rows(self, idx, h_obs):
        self._s[idx] = self._rng.randn(len(idx), self.ob).astype(np.float32)
        self._t[idx] = 0
        h_obs.numpy()[idx] = self._s[idx]

    def _step_rows(self, act, h_obs, h_rew):
        a = np.asarray(act, np.float32)  # s'_i = tanh(A_i . s) + 0.1 a[i % ac] (k_synth_env)
        s = np.tanh(self._s @ self.A.T) + np.float32(0.1) * a[:, np.arange(self.ob) % self.ac]
        self._s = s.astype(np.float32)
        h_obs.numpy()[:] = self._s
        h_rew.numpy()[:] = -(a * a).sum(1) + self._s[:, 0]
        self._t += 1
        return self._t >= self._max_episode_steps

    def spawn(self, n_envs, seed):
        return HostSynthEnv(n_envs, self.ob, self.ac, self._max_episode_steps, self.ac_high, seed=seed,
                            device=self.device)

    def sample_actions(self, out):
        out.copy_(torch.from_numpy(self._rng.uniform(-self.ac_high, self.ac_high, (self.n, self.ac)).astype(
            np.float32)))
        return out


# ---------------------------------------------------------------- loop


class OffPolicyLoop:
    """Trainer mixin of SAC_AcM / DDPG_AcM.  The host class provides ``act``,
    ``update``, ``replay_buffer``, ``bucket_acm``, ``_h`` and ``_fused_update(idx, ctr, allreduce, beside)``."""

    def _init_loop(self, iterations=config.ITERATIONS, batch_size=config.BATCH_SIZE, stats_freq=config.STATS_FREQ,
                   test_episodes=None, return_done=None, max_frames=None, random_frames=config.RANDOM_FRAMES,
                   update_freq=config.UPDATE_FREQ, grad_steps=config.GRAD_STEPS, acm_epochs=config.ACM_EPOCHS,
                   acm_batch_size=config.ACM_BATCH_SIZE, acm_update_freq=config.ACM_UPDATE_FREQ,
                   acm_update_batches=config.ACM_UPDATE_BATCHES, acm_pre_train_samples=config.ACM_PRE_TRAIN_SAMPLES,
                   acm_pre_train_epochs=config.ACM_PRE_TRAIN_N_EPOCHS, acm_scheduler_step=config.ACM_SCHEDULER_STEP,
                   acm_scheduler_gamma=config.ACM_SCHEDULER_GAMMA, acm_keep_pretrain=config.ACM_KEEP_PRE_TRAIN,
                   n_envs=1, env=None, schedule=None, loop_seed=0, allreduce=None, allreduce_sum=None, host_sum=None,
                   tensorboard_dir=None, debug_mode=False, update_batch_size=None, **rest):
        config.check_kwargs(type(self).__name__, rest)  # (update_batch_size: already set by the agent)
        if max_frames is not None and max_frames > iterations * batch_size:
            raise AssertionError("max_frames should be smaller or equal than iterations * batch_size")  # rl.py:166
        self.iterations, self.batch_size, self.stats_freq = int(iterations), int(batch_size), int(stats_freq)
        self.test_episodes, self.return_done, self.max_frames = test_episodes, return_done, max_frames
        self.random_frames, self.update_freq, self.grad_steps = int(random_frames), int(update_freq), int(grad_steps)
        self.acm_epochs, self.acm_batch_size, self.acm_update_freq = int(acm_epochs), int(acm_batch_size), int(
            acm_update_freq)
        self.acm_update_batches = acm_update_batches
        self.acm_pre_train_samples, self.acm_pre_train_epochs = int(acm_pre_train_samples), int(acm_pre_train_epochs)
        self.acm_scheduler_step, self.acm_scheduler_gamma = int(acm_scheduler_step), float(acm_scheduler_gamma)
        self.acm_keep_pretrain = bool(acm_keep_pretrain)
        self._acm_sched_epochs = 0  # StepLR.last_epoch
        self.iteration = 0
        self.stats_logger = StatsLogger()
        # rl.py:67-83: a TensorBoard writer when tensorboard_dir is given (scalar panels, spprl/tb.py)
        self.tensorboard_dir, self.debug_mode = tensorboard_dir, bool(debug_mode)
        self.tensorboard_writer = None
        if tensorboard_dir is not None:
            from .tb import TensorboardWriter

            self.tensorboard_writer = TensorboardWriter(tensorboard_dir)
        ob, ac = self.ob_dim, self.ac_dim
        if env is None:
            spec = getattr(self, "env_spec", None) or config.ENV_SPECS.get(self.env_name, (ob, ac, 1.0, 1000))
            env = SynthVecEnv(n_envs, ob, ac, max_episode_steps=spec[3], ac_high=spec[2], seed=loop_seed,
                              device=self.device)
        self.env = env
        self.n_envs = env.n
        self.schedule = schedule or ("reference" if self.n_envs == 1 else "fused")
        if self.schedule not in ("reference", "fused"):
            raise ValueError("schedule must be 'reference' or 'fused'")
        self.allreduce = allreduce if allreduce is not None else make_allreduce()
        self.allreduce_sum = self.host_sum = self.allgather = None
        if self.allreduce is not None:
            # the obs statistics must be global whenever the gradients are (else the replicas' normalisers
            # drift apart): an explicit gradient exchange needs its statistics exchange too
            self.allreduce_sum = allreduce_sum if allreduce_sum is not None else make_allreduce_sum()
            self.host_sum = host_sum if host_sum is not None else make_host_allreduce_sum()
            self.allgather = make_allgather()  # one-pass statistics (None: the stepwise protocol)
            if self.allreduce_sum is None:
                raise ValueError("an explicit allreduce needs allreduce_sum (and host_sum) for the global obs "
                                 "statistics, e.g. spprl.dp.NativeComm(...).attach(agent) or torch.distributed")
        self.loop_seed = int(loop_seed)
        # one Philox key per random-stream consumer (never a shared (key, counter) pair)
        self._key_policy, self._key_index = stream_key(loop_seed, "policy"), stream_key(loop_seed, "index")
        self._key_update = stream_key(loop_seed, "update_eps")
        self._ctr = 0
        E = self.n_envs
        self.rho = self.update_batch_size * self.grad_steps / self.update_freq
        self.sigma = (self.acm_update_batches * self.acm_batch_size / self.acm_update_freq
                      if self.acm_update_batches else 0.0)
        d = self.device
        self._eps = torch.empty(E, self.actor_output_dim, device=d)
        self._noise = torch.empty(E, self.actor_output_dim, device=d)
        self._ep_ret = torch.zeros(E, device=d)
        self._ret_sums = torch.zeros(2, dtype=torch.float64, device=d)
        self._acm_loss = torch.zeros(1, device=d)
        self._acm_loss_acc = torch.zeros(1, device=d)
        self._obs = None
        self._prev_slots = None
        self._ep_len = np.zeros(E, np.int64)  # frames into the current episode, per env (time-limit done, Q3)

    def _check_kwargs(self, kw):
        """At the top of an agent constructor: every keyword it hands to _init_loop is a loop keyword or one of
        config.NO_EFFECT_KWARGS, else TypeError (before any device allocation)."""
        import inspect

        taken = set(inspect.signature(OffPolicyLoop._init_loop).parameters) - {"self", "rest"}
        config.check_kwargs(type(self).__name__, {k: v for k, v in kw.items() if k not in taken})

    # ---------------------------------------------------------- helpers
    def _next(self):
        self._ctr += 1
        return self._ctr

    def _randn(self, t):
        call("sppRandNormal", ptr(t), t.numel(), self._key_policy, self._next(), stream_handle())
        return t

    def _set_acm_lr(self, lr):
        call("sppAgentSetLr", self._h, -1.0, -1.0, -1.0, float(lr))

    # ---------------------------------------------------------- RL.train (rl.py:192-229)
    def train(self, iterations=None):
        if iterations:
            self.iterations += iterations
        ret = None
        while self.iteration < self.iterations:
            t0 = time.perf_counter()
            ret = self.perform_iteration()
            self.stats_logger.time_list.append(time.perf_counter() - t0)
            running = self.stats_logger.calc_running_return(ret)
            if self.return_done is not None and running is not None and running >= self.return_done:
                break
            if self.iteration % self.stats_freq == 0:
                self.logs_after_iteration(ret)
            self.iteration += 1
            if self.max_frames is not None and self.max_frames < self.stats_logger.frames:
                break
        self.logs_after_iteration(ret, done=True)
        return self.stats_logger.running_return

    def logs_after_iteration(self, ret, done=False):  # rl.py:320-368
        if self.test_episodes:
            self.stats_logger.test_return = self.test()
        loss = dict(self.loss)
        self.stats_logger.stats.append({"iteration": self.iteration, "frames": self.stats_logger.frames,
                                        "running_return": self.stats_logger.running_return,
                                        "test_return": self.stats_logger.test_return, "loss": loss})
        w = self.tensorboard_writer
        if w is not None:  # add_tensorboard_logs (rl.py:344-368): the scalar panels
            sl = self.stats_logger
            if sl.running_return is not None:
                w.log_running_return(self.iteration, sl.frames, sl.rollouts, sl.running_return)
            if self.test_episodes:
                w.log_test_return(self.iteration, sl.frames, sl.rollouts, sl.test_return)
            w.log_loss(self.iteration, loss)
            if self.debug_mode and hasattr(self, "current_alpha"):  # sac.py:233-236
                w.log_sac_alpha(self.iteration, self.current_alpha())
            w.flush()
            if done:
                w.close()

    # ---------------------------------------------------------- DDPG.perform_iteration (ddpg.py:159-170)
    def perform_iteration(self):
        """Collect batch_size frames (training as they arrive), then update the obs stats.
        Returns the mean return of the episodes completed in this iteration (None if none)."""
        self._ret_sums.zero_()
        self.collect_batch_and_train(self.batch_size)
        self.update_obs_stats()
        s = self._ret_sums.cpu().numpy()
        return float(s[0] / s[1]) if s[1] > 0 else None

    def update_obs_stats(self):
        """update_obs_mean_std (rl.py:93-112); global over the ranks' shards under DP."""
        if self.allreduce is not None and self.allreduce_sum is None:
            raise RuntimeError("data-parallel gradients without a statistics exchange (allreduce_sum): "
                               "use NativeComm.attach(agent) or torch.distributed")
        if self.allreduce_sum is not None:
            # shard lengths differ across ranks once resets (early terminations) advance the
            # obs rings unevenly: the global row count is all-reduced, never assumed
            # (counted on the host and exchanged over gloo: no device synchronisation per step)
            self.replay_buffer.update_obs_mean_std_dp(self.allreduce_sum, host_sum=getattr(self, "host_sum", None),
                                                      allgather=getattr(self, "allgather", None))
        else:
            self.replay_buffer.update_obs_mean_std()

    def _start_episodes(self):
        self._ep_len[:] = 0
        obs = self.env.reset()
        self._obs = obs
        self._prev_slots = self.replay_buffer.add_obs_batch(obs)
        self._ep_ret.zero_()

    def collect_batch_and_train(self, batch_size):
        collected = 0
        if self.schedule == "reference":
            while collected < batch_size:  # whole episodes (ddpg.py:192-223)
                self.stats_logger.rollouts += 1
                self._start_episodes()
                end = False
                while not end:
                    end = bool(self._vector_step()[0])
                    collected += 1
                    self.make_update()
            return
        if self._obs is None:
            self._start_episodes()
            self.stats_logger.rollouts += self.n_envs
        while collected < batch_size:
            self._vector_step()
            collected += self.n_envs

    def _vector_step(self):
        """One step of every env: act -> env -> replay writes (-> fused update)."""
        E = self.n_envs
        rb = self.replay_buffer
        mode = 0 if self.stats_logger.frames < self.random_frames else 1  # initial_act (off_policy.py:50-54)
        vanilla = getattr(self, "VANILLA", False)
        if mode == 0 and vanilla:
            self.env.sample_actions(self._eps)  # DDPG.initial_act: env.action_space.sample() (ddpg.py:178-180)
        else:
            self._randn(self._eps)
        if mode == 1:
            self._randn(self._noise)
        obs_in = rb.normalize(self._obs)
        tgt, env_act = self.act(obs_in, eps=self._eps, noise=self._noise, mode=mode)
        pipelined = self.schedule == "fused" and self.env.is_host
        if pipelined:
            self.env.send(env_act)
            self._fused_make_update()  # overlaps the CPU envs
            nobs, rew, end, end_dev = self.env.recv()
        else:
            nobs, rew, end, end_dev = self.env.step(env_act)
        any_end = bool(end.any())
        call("sppEpisodeAccum", ptr(rew), ptr(end_dev) if any_end else None, E, ptr(self._ep_ret),
             ptr(self._ret_sums), stream_handle())
        slots = rb.add_obs_batch(nobs)
        # done = end, except at the time limit when max_ep_len is set (Q3, ddpg.py:210-212);
        # AcMOffPolicy keeps max_ep_len None (off_policy.py:43)
        done_dev = end_dev
        max_ep = getattr(self, "max_ep_len", None)
        if max_ep is not None:
            self._ep_len += 1
            if any_end:
                done_h = end & (self._ep_len != max_ep)
                done_dev = torch.from_numpy(done_h.astype(np.uint8)).to(self.device, non_blocking=False)
            else:
                done_dev = end_dev  # all zero
            self._ep_len[end] = 0
        rb.add_timestep_batch(self._prev_slots, slots, tgt, rew, done_dev, end_dev, None if vanilla else env_act)
        self._prev_slots = slots
        self._obs = nobs
        self.stats_logger.frames += E
        if any_end and self.schedule == "fused":
            self.stats_logger.rollouts += int(end.sum())
            self._obs = self.env.reset(end)
            rs = rb.add_obs_batch(self._obs[torch.as_tensor(np.flatnonzero(end), device=self.device)])
            self._prev_slots = self._prev_slots.copy()
            self._prev_slots[np.flatnonzero(end)] = rs
        if self.schedule == "fused" and not pipelined:
            self._fused_make_update()
        return end

    # ---------------------------------------------------------- make_update
    def update_condition(self):  # ddpg.py:225-229
        return len(self.replay_buffer) > self.update_batch_size and self.stats_logger.frames % self.update_freq == 0

    def acm_update_condition(self):  # ddpg_acm.py:52-57
        return self.iteration > 0 and self.acm_epochs > 0 and self.stats_logger.frames % self.acm_update_freq == 0

    def make_update(self):
        """Reference cadence (ddpg.py:231-237, ddpg_acm.py:75-85), one frame at a time.  unbiased_update
        (make_unbiased_update, ddpg_acm.py:59-73): the sampled next obs is the critic's action."""
        if self.update_condition():
            unbiased = getattr(self, "unbiased_update", False)
            rb = self.replay_buffer
            # vanilla SAC on the device: the same MT19937 index draw as sample_batch (replay_buffer.py:234), staged
            # feature-major straight from the ring (one gather kernel instead of a row-major gather + restage) with
            # the rsample noise drawn on the device
            staged = getattr(self, "VANILLA", False) and self.device.type == "cuda"
            for _ in range(self.grad_steps):
                if staged:
                    idx = np.random.randint(0, len(rb), self.update_batch_size)
                    self.update_from_replay(rb._idx_dev(idx), self._key_update, self._next())
                    continue
                batch = rb.sample_batch(self.update_batch_size, self.device)
                if unbiased:
                    batch[2] = batch[1]
                self.update(*batch)
        if self.acm_update_condition():
            if self.acm_update_batches:
                self.update_acm_batches(self.acm_update_batches)
            else:
                self.update_acm(self.acm_epochs)

    def _fused_make_update(self):
        """Batched cadence: rho*E transitions in one grad step, sigma*E in one ACM step."""
        rb = self.replay_buffer
        n = len(rb)
        B, BA = self.fused_batch_sizes()
        acm_batch = self.iteration > 0 and self.acm_epochs > 0 and bool(self.acm_update_batches)
        if n > self.update_batch_size:
            idx = torch.empty(B, dtype=torch.int64, device=self.device)
            ctr = self._next()
            call("sppRandIndex", ptr(idx), B, n, self._key_index, ctr, stream_handle())
            beside = None
            if acm_batch and self._exchange_overlap():
                # the ACM step's gather and gradients (they read only the ACM and the replay, which the actor
                # update leaves alone) run while the actor bucket is exchanged; its indices are the same draw
                # (the next counter) as in the serial order below
                ia = self._rand_idx(BA, n)
                beside = lambda: self._acm_grads_from_idx(ia)  # noqa: E731
            self._fused_update(idx, ctr, self.allreduce, beside)  # (eps counter: the index draw's, as serial)
            self._keep_idx = idx
            if beside is not None:
                self._acm_exchange_apply()
                self._acm_loss_acc.copy_(self._acm_loss)
                return
        if self.iteration > 0 and self.acm_epochs > 0:
            if self.acm_update_batches:
                self._acm_step_from_idx(self._rand_idx(BA, n))
                self._acm_loss_acc.copy_(self._acm_loss)
            else:  # epoch mode at every crossed multiple of acm_update_freq
                f1 = self.stats_logger.frames
                if f1 // self.acm_update_freq > (f1 - self.n_envs) // self.acm_update_freq:
                    self.update_acm(self.acm_epochs)

    def _stage(self, idx):
        """sample_batch of the fused schedule on device: gather the transitions idx into the agent's staging
        area (sppAgentStageFromReplay), then the normalisation of obs_norm buffers (replay_buffer.py:247-249)
        and, with unbiased_update, action := next obs (ddpg_acm.py:59-73), in place (sppAgentStagePost)."""
        st = stream_handle()
        rb = self.replay_buffer
        call("sppAgentStageFromReplay", self._h, rb._h, ptr(idx), idx.numel(), st)
        norm = bool(rb.obs_norm) and not (rb.min_max_denormalize and not rb._have_minmax)  # normalize() no-ops
        if norm and not rb.HAS_ACM:  # the plain ReplayBuffer (vanilla SAC): z-score (zeros / ones before any stats)
            norm = 2
        unbiased = bool(getattr(self, "unbiased_update", False)) and not self.acm_critic  # acm_critic: acm_action
        if norm or unbiased:
            call("sppAgentStagePost", self._h, int(norm), int(unbiased), st)

    def fused_batch_sizes(self):
        """(grad-step batch, ACM batch) of one fused vector step: rho*E and sigma*E."""
        E = self.n_envs
        return max(1, int(round(self.rho * E))), max(1, int(round(self.sigma * E))) if self.sigma else 0

    def _rand_idx(self, B, n):
        idx = torch.empty(B, dtype=torch.int64, device=self.device)
        call("sppRandIndex", ptr(idx), B, n, self._key_index, self._next(), stream_handle())
        return idx

    # ---------------------------------------------------------- ACM regression
    def _acm_step_from_idx(self, idx):
        """acm_cat + batch_update (acm.py:246-264) on gathered replay rows."""
        self._acm_grads_from_idx(idx)
        self._acm_exchange_apply()

    def _acm_grads_from_idx(self, idx):
        B = idx.numel()
        st = stream_handle()
        x = torch.empty(B, 2 * self.ob_dim, device=self.device)
        y = torch.empty(B, self.ac_dim, device=self.device)
        call("sppReplayGatherAcm", self.replay_buffer._h, ptr(idx), B, ptr(x), ptr(y), st)
        call("sppAcmRegressGrads", self._h, ptr(x), ptr(y), B, ptr(self._acm_loss), st)
        self._keep_acm_xy = (idx, x, y)

    def _acm_exchange_apply(self):
        if self.allreduce is not None:
            self.allreduce(self.bucket_acm)
        call("sppAcmRegressApply", self._h, stream_handle())

    # ---------------------------------------------------------- exchange overlap
    def _exchange_overlap(self):
        """Data-parallel bucket exchange beside independent compute: opt-in (SPP_DP_OVERLAP=1).  Measured on the
        one-rank RCCL rehearsal (profiles/r05/dp_overlap/): with the exchange on its own stream every kernel of
        the step dispatched slowly (Adam / pack / finalize 40-55 us instead of 4-9 us in the kernel trace), SAC
        Hopper 12.69 ms per step against 9.77 ms in the serial order, so the serial order is the default."""
        return (self.allreduce is not None and torch.device(self.device).type == "cuda"
                and os.environ.get("SPP_DP_OVERLAP", "0") == "1")

    def _exchange(self, allreduce, bucket, beside=None):
        """allreduce(bucket), averaged in place.  With ``beside`` the exchange is enqueued on the agent's
        exchange stream (after everything already on the current stream) while ``beside()`` enqueues work that
        neither reads nor writes the bucket on the current stream; the current stream then waits for the
        exchange.  The same operations on the same data as the serial order, so the results are identical."""
        if beside is None:
            if allreduce is not None:
                allreduce(bucket)
            return
        if allreduce is None:
            beside()
            return
        main = torch.cuda.current_stream(self.device)
        side = getattr(self, "_xstream", None)
        if side is None:
            side = self._xstream = torch.cuda.Stream(device=self.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            allreduce(bucket)
        beside()
        main.wait_stream(side)

    def _acm_sgd_ok(self, bs):
        """The persistent one-launch SGD kernel (sppAcmSgd) covers the AcM of these dims, one rank, and
        batches whose workgroups are all co-resident on this device (sppAcmSgdMaxBatch)."""
        if not (getattr(self, "acm_kind", "acm") == "acm" and self.allreduce is None
                and (self.ob_dim, self.ac_dim) in ((11, 3), (17, 6), (3, 1))):
            return False
        if getattr(self, "_sgd_max_bs", None) is None:
            self._sgd_max_bs = int(load().sppAcmSgdMaxBatch(self._h))
        return bs <= self._sgd_max_bs

    def acm_sgd_workgroups(self):
        """Workgroups (one per CU) of one sppAcmSgd step at acm_batch_size (sppAcmSgdWorkgroups)."""
        return max(1, int(load().sppAcmSgdWorkgroups(self._h, int(self.acm_batch_size))))

    def _acm_sgd(self, idx, nsteps, bs, nrows=None):
        """nsteps AcM regression steps in one launch on the rows idx[k*bs:(k+1)*bs] (sppAcmSgd); with nrows,
        one epoch over idx[:nrows] whose last batch is the ragged remainder (sppAcmSgdEpoch)."""
        n = nsteps * bs if nrows is None else nrows
        x, y = self._acm_gather(idx, n)
        self._acm_sgd_xy(x, y, nsteps, bs, nrows)
        self._keep_sgd = (idx, x, y)

    def _acm_gather(self, idx, n):
        """The AcM regression rows of idx[:n] (sppReplayGatherAcm: x = [obs | next obs], y = the ACM action)."""
        x = torch.empty(n, 2 * self.ob_dim, device=self.device)
        y = torch.empty(n, self.ac_dim, device=self.device)
        call("sppReplayGatherAcm", self.replay_buffer._h, ptr(idx), n, ptr(x), ptr(y), stream_handle())
        return x, y

    def _acm_sgd_xy(self, x, y, nsteps, bs, nrows=None):
        st = stream_handle()
        ev = getattr(self, "sgd_events", None)  # measurement: HIP events around each sppAcmSgd launch
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if nrows is None:
            call("sppAcmSgd", self._h, ptr(x), ptr(y), nsteps, bs, ptr(self._acm_loss_acc), st)
        else:
            call("sppAcmSgdEpoch", self._h, ptr(x), ptr(y), nrows, bs, ptr(self._acm_loss_acc), st)
        if ev is not None:
            e1.record()
            ev.append((e0, e1, x.shape[0]))

    def _acm_sgd_check(self):
        """Raise if a multi-workgroup sppAcmSgd launch timed out at its arrival barrier (its AcM
        weights are then invalid).  The flag is copied stream-ordered into pinned memory after each
        update_acm and read at the next one (or by check_acm_sgd(sync=True)), so no call blocks."""
        ev = getattr(self, "_sgd_flag_ev", None)
        if ev is not None:
            ev.synchronize()
            if int(self._sgd_flag[0]):
                raise SppError("sppAcmSgd: a multi-workgroup step timed out at its arrival barrier; the AcM "
                               "parameters are invalid")
        if getattr(self, "_sgd_flag", None) is None:
            self._sgd_flag = torch.zeros(1, dtype=torch.int32).pin_memory()
        call("sppAcmSgdStatusAsync", self._h, self._sgd_flag.data_ptr(), stream_handle())
        self._sgd_flag_ev = torch.cuda.Event()
        self._sgd_flag_ev.record()

    def check_acm_sgd(self):
        """Synchronous form of the timeout check (tests, end of training)."""
        self._acm_sgd_check()
        self._acm_sgd_check()

    def update_acm_batches(self, n_batches):
        """acm.py:356-372: n batches of acm_batch_size uniform samples; loss = batch mean."""
        n = len(self.replay_buffer)
        self._acm_loss_acc.zero_()
        if self._acm_sgd_ok(self.acm_batch_size):
            self._acm_sgd(self._rand_idx(n_batches * self.acm_batch_size, n), n_batches, self.acm_batch_size)
            if self.acm_sgd_workgroups() > 1:
                self._acm_sgd_check()
        else:
            for _ in range(n_batches):
                self._acm_step_from_idx(self._rand_idx(self.acm_batch_size, n))
                self._acm_loss_acc += self._acm_loss
        self._acm_loss_acc /= n_batches

    def update_acm(self, epochs, pretrain=False):
        """acm.py:266-303: shuffled epochs over every live row, batches of acm_batch_size,
        StepLR(acm_scheduler_step, acm_scheduler_gamma) stepped once per epoch."""
        n = len(self.replay_buffer)
        if n == 0:
            return
        # epoch permutations drawn on the device (DataLoader(shuffle=True), acm.py:275) by sppRandPerm (a
        # host randperm and its copy, or torch.randperm on the device, would hold the stream every epoch)
        # (_perm_seed: a seed shared by data-parallel ranks that run the epochs replicated, spprl/ppo_acm.py)
        ps = getattr(self, "_perm_seed", None)
        if ps is None:
            seed = self.loop_seed * 7919 + self._next()
        else:
            self._perm_ctr = getattr(self, "_perm_ctr", 0) + 1
            seed = ps + 104729 * self._perm_ctr
        bs = self.acm_batch_size
        nb = -(-n // bs)
        for e in range(epochs):
            lr = self.acm_lr * self.acm_scheduler_gamma ** (self._acm_sched_epochs // self.acm_scheduler_step)
            self._set_acm_lr(lr)
            self._acm_loss_acc.zero_()
            perm = device_randperm(n, seed, e * n, self.device)
            if self._acm_sgd_ok(bs):  # the whole epoch in one launch, the ragged last batch included
                self._acm_sgd(perm, nb, bs, nrows=n)
            else:
                for s in range(0, n, bs):
                    self._acm_step_from_idx(perm[s:s + bs].contiguous())
                    self._acm_loss_acc += self._acm_loss
            self._acm_loss_acc /= max(nb, 1)
            self._acm_sched_epochs += 1
        if self.acm_sgd_workgroups() > 1 and self._acm_sgd_ok(self.acm_batch_size):  # a multi-workgroup launch ran
            self._acm_sgd_check()
        self._set_acm_lr(self.acm_lr * self.acm_scheduler_gamma ** (self._acm_sched_epochs // self.acm_scheduler_step))

    # ---------------------------------------------------------- pre-train (acm.py:234-244)
    def collect_samples(self):
        """AcMOffPolicy.collect_samples (off_policy.py:56-87): random env actions; the
        buffer's ``action`` slot holds the next obs; time-limit ends are kept as done."""
        rb, E = self.replay_buffer, self.n_envs
        collected = 0
        obs = self.env.reset()
        prev = rb.add_obs_batch(obs)
        act = torch.empty(E, self.ac_dim, device=self.device)
        while collected < self.acm_pre_train_samples:
            self.env.sample_actions(act)
            nobs, rew, end, end_dev = self.env.step(act)
            slots = rb.add_obs_batch(nobs)
            rb.add_timestep_batch(prev, slots, nobs, rew, end_dev, end_dev, act)
            prev = slots
            collected += E
            if end.any():
                obs = self.env.reset(end)
                rs = rb.add_obs_batch(obs[torch.as_tensor(np.flatnonzero(end), device=self.device)])
                prev = prev.copy()
                prev[np.flatnonzero(end)] = rs
        self._obs = None

    def pre_train(self):
        self.collect_samples()
        self.update_acm(epochs=self.acm_pre_train_epochs, pretrain=True)
        self.update_obs_stats()
        if not self.acm_keep_pretrain:
            self.replay_buffer.reset_idx()

    # ---------------------------------------------------------- DDPG.test (ddpg.py:385-410)
    def test(self, episodes=None):
        """Deterministic policy (act_noise 0, mode det) for ``episodes`` env instances run in
        parallel, one episode each; returns the mean episode return."""
        episodes = episodes or self.test_episodes or 1
        env = self.env.spawn(episodes, seed=self.loop_seed + 99991)
        obs = env.reset()
        ret = torch.zeros(episodes, device=self.device)
        sums = torch.zeros(2, dtype=torch.float64, device=self.device)
        alive = np.ones(episodes, bool)
        while alive.any():
            _, env_act = self.act(self.replay_buffer.normalize(obs), mode=2, act_noise=0.0)
            obs, rew, end, _ = env.step(env_act)
            first = end & alive
            m = torch.as_tensor(first.astype(np.uint8), device=self.device)
            call("sppEpisodeAccum", ptr(rew), ptr(m), episodes, ptr(ret), ptr(sums), stream_handle())
            alive &= ~end
            if end.any() and alive.any():
                obs = env.reset(end)
        s = sums.cpu().numpy()
        return float(s[0] / s[1])

    @property
    def acm_loss(self):
        return float(self._acm_loss_acc.item())

    # ---------------------------------------------------------- per-kernel device timing
    def set_timing(self, on=True):
        call("sppAgentSetTiming", self._h, int(on))

    def get_timing(self):
        """(total ms, launch count) per kind: critic phase, actor phase, dW, Adam, ACM regression."""
        ms = np.zeros(5, np.float64)
        cnt = np.zeros(5, np.int64)
        call("sppAgentGetTiming", self._h, ms.ctypes.data_as(ctypes.c_void_p), cnt.ctypes.data_as(ctypes.c_void_p))
        return ms, cnt

    # ---------------------------------------------------------- checkpoints (rl.py:281-301)
    def save(self, path):
        from .checkpoint import save_params

        save_params(path, self.collect_params_dict())

    def load(self, path):
        from .checkpoint import load_params

        self.apply_params_dict(load_params(path))


def acm_lr_at(acm_lr, gamma, step, epochs_done):
    """StepLR value after ``epochs_done`` scheduler steps (torch.optim.lr_scheduler.StepLR)."""
    return acm_lr * gamma ** (epochs_done // step)

