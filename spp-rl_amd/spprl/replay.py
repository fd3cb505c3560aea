"""HBM-resident BufferAcMOffPolicy (rltoolkit/buffer/replay_buffer.py:303-401).

Same method names and semantics as the reference, including the obs-index ring
and its wrap rule (Q6).  Batched variants (``add_obs_batch`` / ``add_timestep_batch``)
apply the reference recurrence to E lockstep envs in env order.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_handle


class Memory:
    """What rltoolkit's last_rollout returns (buffer/memory.py:131-270 Memory / MemoryAcM, one
    rollout): ``obs`` [T, ob] and ``next_obs`` [T, ob] of the episode, ``actions`` [T, aout],
    ``rewards`` [T], ``done`` / ``end`` [T] (the end flags; the last is set), ``actions_acm`` [T, ac]
    and the buffer's normaliser state (``normalize`` / ``denormalize`` as the buffer's)."""

    def __init__(self, obs_all, actions, rewards, end, actions_acm, buffer):
        self._obs_all = obs_all  # [T + 1, ob]: the episode's observations and the final next_obs
        self.actions, self.rewards, self.actions_acm = actions, rewards, actions_acm
        self.done = self.end = end
        self.min_max_denormalize = buffer.min_max_denormalize
        self.obs_mean, self.obs_std = buffer.obs_mean.clone(), buffer.obs_std.clone()
        self.min_obs, self.max_obs = buffer.min_obs.clone(), buffer.max_obs.clone()
        self._buffer = buffer

    @property
    def obs(self):
        return self._obs_all[:-1]

    @property
    def next_obs(self):
        return self._obs_all[1:]

    @property
    def norm_obs(self):
        return self._buffer.normalize(self.obs, force=True)

    @property
    def norm_next_obs(self):
        return self._buffer.normalize(self.next_obs, force=True)

    def __len__(self):
        return int(self.rewards.shape[0])

    @property
    def returns_rollouts(self):  # memory.py:202-212
        return np.array([float(self.rewards.double().sum())])

    @property
    def rollouts_no(self):  # memory.py:214-216
        return int(self.end.sum())

    @property
    def average_returns_per_rollout(self):
        return float(self.returns_rollouts.sum()) / self.rollouts_no


class BufferAcMOffPolicy:
    HAS_ACM = True

    def __init__(self, size, obs_shape, act_shape, acm_act_shape, device="cuda", min_max_denormalize=False,
                 obs_mean=None, obs_std=None, max_obs=None, min_obs=None, obs_norm=False, dtype=torch.float32,
                 n_envs=1):
        _lib.load()
        self.size, self.obs_shape, self.act_shape, self.acm_act_shape = int(size), obs_shape, act_shape, acm_act_shape
        self.device = torch.device(device)
        self.dtype = dtype
        self.obs_norm = obs_norm
        self.min_max_denormalize = min_max_denormalize
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = ctypes.c_void_p()
        call("sppReplayCreateEx", ctypes.byref(h), self.size, obs_shape, act_shape, acm_act_shape, int(n_envs), 1, 0,
             dev)
        self._h = h
        z = lambda v: None if v is None else torch.as_tensor(v, dtype=torch.float32, device=self.device)  # noqa
        # ReplayBuffer.__init__ :113-115: identity z-score normaliser until the first stats update
        self.obs_mean = z(obs_mean) if obs_mean is not None else torch.zeros(obs_shape, device=self.device)
        self.obs_std = z(obs_std) if obs_std is not None else torch.ones(obs_shape, device=self.device)
        self.max_obs = z(max_obs) if max_obs is not None else torch.zeros(obs_shape, device=self.device)
        self.min_obs = z(min_obs) if min_obs is not None else torch.zeros(obs_shape, device=self.device)
        self._have_minmax = max_obs is not None and min_obs is not None
        self._pending_acm = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sppReplayDestroy(h)
            self._h = None

    def set_acm_columns(self, cols):
        """AcMTrainer.acm_ob_idx (acm.py:94-99, 260-264): the ob columns of acm_cat's obs / next_obs in every ACM
        gather (sppReplaySetAcmColumns); None restores the whole observation vector."""
        n = 0 if cols is None else len(cols)
        arr = np.asarray(cols if cols is not None else [0], np.int32)
        call("sppReplaySetAcmColumns", self._h, arr.ctypes.data_as(ctypes.c_void_p) if n else None, n)
        self.acm_cols = None if cols is None else list(cols)

    # ------------------------------------------------------------------ state
    def _state(self):
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        call("sppReplayState", self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    @property
    def obs_idx(self):
        return self._state()[0]

    @property
    def ts_idx(self):
        return self._state()[1]

    @property
    def current_len(self):
        return self._state()[2]

    def __len__(self):
        return self._state()[2]

    def reset_idx(self):
        call("sppReplayReset", self._h)
        self._gen = getattr(self, "_gen", 0) + 1

    def view(self):
        v = _lib.ReplayView()
        call("sppReplayGetView", self._h, ctypes.byref(v))
        return v

    # ------------------------------------------------------------------ writes
    def _dev(self, x, dtype=torch.float32):
        return torch.as_tensor(x, dtype=dtype).to(self.device).contiguous()

    def add_obs_batch(self, obs):
        """obs [E, ob] -> slots (numpy int64 [E])"""
        o = self._dev(obs).reshape(-1, self.obs_shape)
        slots = np.empty(o.shape[0], np.int64)
        call("sppReplayAddObs", self._h, ptr(o), o.shape[0], slots.ctypes.data_as(ctypes.c_void_p), stream_handle())
        return slots

    def add_obs(self, obs):
        """MetaReplayBuffer.add_obs (:56-60)"""
        return int(self.add_obs_batch(torch.as_tensor(obs).reshape(1, -1))[0])

    def add_acm_action(self, acm_action):
        """BufferAcMOffPolicy.add_acm_action (:332-333): stored at ts_idx by the next add_timestep."""
        self._pending_acm = self._dev(acm_action).reshape(1, self.acm_act_shape)

    def add_timestep_batch(self, prev, nxt, action, rew, done, end, acm_action=None):
        E = len(prev)
        prev = np.ascontiguousarray(prev, np.int64)
        nxt = np.ascontiguousarray(nxt, np.int64)
        act = self._dev(action).reshape(E, self.act_shape)
        acm = self._dev(acm_action).reshape(E, self.acm_act_shape) if acm_action is not None else None
        r = self._dev(rew).reshape(E)
        d = self._dev(done, torch.uint8).reshape(E)
        e = self._dev(end, torch.uint8).reshape(E)
        call("sppReplayAddStep", self._h, prev.ctypes.data_as(ctypes.c_void_p), nxt.ctypes.data_as(ctypes.c_void_p),
             E, ptr(act), ptr(acm), ptr(r), ptr(d), ptr(e), stream_handle())
        self._gen = getattr(self, "_gen", 0) + 1  # timestep writes so far (the DP stats' row-count cache key)

    def add_timestep(self, obs_idx, next_obs_idx, action, rew, done, end):
        """add_timestep (:65-75) + ReplayBuffer.addition (:133-137)"""
        acm = self._pending_acm
        self._pending_acm = None
        self.add_timestep_batch([obs_idx], [next_obs_idx], torch.as_tensor(action).reshape(1, -1), [float(rew)],
                                [bool(done)], [bool(end)], acm)

    # ------------------------------------------------------------------ reads
    def _idx_dev(self, idx):
        """Host indices (sample_batch's numpy draw) -> device int64, through pinned memory and an async copy:
        a pageable upload synchronises the stream (the device would drain before every grad step of the
        reference schedule).  torch's pinned-block cache keeps the block until the copy has completed."""
        if isinstance(idx, torch.Tensor) and idx.device.type == self.device.type and (
                self.device.index is None or idx.device.index == self.device.index):
            return idx.to(torch.int64).contiguous()  # (device="cuda" has no index: any cuda tensor is already there)
        h = torch.as_tensor(np.asarray(idx) if not isinstance(idx, torch.Tensor) else idx, dtype=torch.int64)
        if self.device.type != "cuda":
            return h.contiguous()
        pin = torch.empty(h.shape, dtype=torch.int64, pin_memory=True)
        pin.copy_(h)
        return pin.to(self.device, non_blocking=True)

    def gather(self, idx):
        """Tuples for given indices, reference layout (sample_batch :385-398)."""
        idx = self._idx_dev(idx)
        B = idx.numel()
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa
        obs, nobs, act, rew, acm = f(B, self.obs_shape), f(B, self.obs_shape), f(B, self.act_shape), f(B), f(
            B, self.acm_act_shape)
        done = torch.empty(B, dtype=torch.int8, device=self.device)
        call("sppReplayGather", self._h, ptr(idx), B, ptr(obs), ptr(nobs), ptr(act), ptr(rew), ptr(done), ptr(acm),
             stream_handle())
        if self.obs_norm:
            obs, nobs = self.normalize(obs), self.normalize(nobs)
        return [obs, nobs, act, rew, done, acm]

    def last_rollout(self):
        """BufferAcMOffPolicy.last_rollout (:335-383): the last complete episode (device search for
        the end flags, one gather of its transitions)."""
        first, length = ctypes.c_int64(), ctypes.c_int64()
        call("sppReplayLastRollout", self._h, ctypes.byref(first), ctypes.byref(length), stream_handle())
        T, n = length.value, len(self)
        idx = (first.value + torch.arange(T, dtype=torch.int64)) % n
        norm, self.obs_norm = self.obs_norm, False  # raw observations (make_obs_memory_tensor)
        try:
            obs, nobs, act, rew, _, acm = BufferAcMOffPolicy.gather(self, idx)
        finally:
            self.obs_norm = norm
        end = torch.zeros(T, dtype=torch.bool, device=self.device)
        end[-1] = True
        return Memory(torch.cat([obs, nobs[-1:]]), act, rew, end, acm if self.HAS_ACM else None, self)

    def sample_batch(self, batch_size=64, device=None):
        """idx = np.random.randint(0, len, B) from numpy's global stream (replay_buffer.py:234)."""
        idx = np.random.randint(0, len(self), batch_size)
        return self.gather(idx)

    def sample_acm_batch(self, batch_size=64):
        idx = np.random.randint(0, len(self), batch_size)
        o, no, _, _, _, acm = self.gather(idx)
        return [o, no, acm]

    # ------------------------------------------------------------------ normaliser
    def update_obs_mean_std(self):
        """MetaReplayBuffer.update_obs_mean_std (:83-96), on device."""
        if len(self) <= 10:
            return
        call("sppReplayObsStats", self._h, ptr(self.obs_mean), ptr(self.obs_std), ptr(self.max_obs),
             ptr(self.min_obs), 0 if self._have_minmax else 1, stream_handle())
        self._have_minmax = True

    def update_obs_mean_std_dp(self, allreduce_sum, n_global=None, host_sum=None, allgather=None):
        """update_obs_mean_std over the union of the data-parallel ranks' shards (SURVEY.md
        §8e): ``allreduce_sum(t)`` sums a device tensor in place across ranks (RCCL).  Exact
        global percentiles (radix select on all-reduced histograms); mean / std from fp64
        sums about the replicated current mean.  ``n_global`` (total live rows) may be given
        when known on the host; otherwise the shard lengths (host bookkeeping) are summed once per
        change of the shards: through ``host_sum`` (a gloo exchange of host integers, no device
        synchronisation, spprl.dp.make_host_allreduce_sum) when given, else as a device tensor
        through ``allreduce_sum`` (one host sync).  The ranks write timesteps in lockstep, so the
        count of timestep writes is the same on every rank and all of them reuse the cached total
        between writes (the bench's reference-rate stats run several passes per vector step on
        unchanged shards).

        With ``allgather`` (spprl.dp.make_allgather / NativeComm.allgather: rank-major all-gather with
        ``world`` / ``rank`` attributes) the call reads the local rows ONCE (sppReplayObsStatsDP1: union
        sample all-gathered, one bracketed pass, one all-reduce of moments and counts, four all-reduces of
        candidate histograms); without it, the stepwise radix protocol (4-5 passes over the rows)."""
        if n_global is None:
            gen = getattr(self, "_gen", 0)
            if getattr(self, "_ng_gen", None) != gen:
                # (len, gen, gen^2, 1) summed together: the ranks must be in lockstep (every rank writes
                # timesteps the same number of times, so every rank reaches this exchange).  All gens are equal
                # iff world * sum(gen^2) == sum(gen)^2 (Cauchy-Schwarz), so EVERY rank sees a mismatch and
                # raises.  The check covers ranks that all wrote since the last exchange; a rank that did not
                # write at all skips this exchange and the mismatch then shows as a hang of the collective
                # below (the trainer writes every rank's timesteps in the same vector step, so it cannot).
                if host_sum is not None:
                    ng, sgen, sgen2, world = host_sum([len(self), gen, gen * gen, 1])
                else:
                    n = torch.tensor([len(self), gen, gen * gen, 1], dtype=torch.int64, device=self.device)
                    allreduce_sum(n)
                    ng, sgen, sgen2, world = (int(v) for v in n.tolist())
                if sgen * sgen != sgen2 * world:
                    raise RuntimeError("data-parallel replay shards out of lockstep: timestep-write counts "
                                       "differ across ranks (this rank %d, sum %d over %d ranks)" % (gen, sgen, world))
                self._ng, self._ng_gen = ng, gen
            n_global = self._ng
        if n_global <= 10:  # replay_buffer.py:84, on the global buffer
            return
        if allgather is not None:
            return self._obs_stats_dp1(allreduce_sum, allgather, n_global)
        if getattr(self, "_dp_hist", None) is None:
            hs = _lib.load().sppReplayObsStatsDPHistSize(self._h)
            self._dp_hist = torch.zeros(hs, dtype=torch.int32, device=self.device)
            self._dp_sums = torch.zeros(self.obs_shape, 2, dtype=torch.float64, device=self.device)
            self._dp_pivot = torch.zeros(self.obs_shape, device=self.device)
        ob = self.obs_shape
        top = ob * 256  # step 0's histogram: the top byte of every column ([ob][256]; the rest is zero)
        for step in self.obs_stats_dp_steps(n_global):
            if step == 0:
                # one collective for the fp64 moment sums and the top-byte counts (exact in fp64)
                buf = torch.cat([self._dp_sums.reshape(-1), self._dp_hist[:top].to(torch.float64)])
                allreduce_sum(buf)
                self._dp_sums.copy_(buf[:2 * ob].view(ob, 2))
                # counts reach 2^32 - 1 (n_global < 2^32): through int64 and the low 32 bits, the uint32
                # pattern k_stats_sel reads (a direct fp64 -> int32 cast is undefined past 2^31)
                self._dp_hist[:top].copy_((buf[2 * ob:].to(torch.int64) & 0xFFFFFFFF).to(torch.int32))
            else:
                allreduce_sum(self._dp_hist)

    def _obs_stats_dp1(self, allreduce_sum, allgather, n_global):
        """The one-pass protocol (sppReplayObsStatsDP1 phases 0..6 with the collectives between)."""
        W, R, ob = allgather.world, allgather.rank, self.obs_shape
        Sl = _lib.load().sppReplayObsStatsDP1SampleRows(self._h, W, n_global)
        key = (W, Sl)
        if getattr(self, "_dp1_key", None) != key:
            self._dp1_samp = torch.zeros(W * ob * Sl, dtype=torch.int32, device=self.device)
            self._dp1_exch = torch.zeros(12 * ob, dtype=torch.float64, device=self.device)
            self._dp1_hist = torch.zeros(ob * 1024, dtype=torch.int32, device=self.device)
            self._dp1_key = key
        first = 0 if self._have_minmax else 1
        mine = self._dp1_samp[R * ob * Sl:(R + 1) * ob * Sl]
        # Shards unchanged since the last call (timestep-write count, checked in lockstep across ranks, and
        # the same global row count): every rank skips the sample and its all-gather and keeps the union
        # bracket.  Rows changed by add_obs alone keep a stale bracket, which is still exact.
        gen = getattr(self, "_gen", 0)
        bkey = (gen, n_global, key)
        # only on a write count the lockstep exchange verified (else a rank out of step would skip the
        # all-gather the others run)
        verified = getattr(self, "_ng_gen", None) == gen and getattr(self, "_ng", None) == n_global
        reuse = verified and getattr(self, "_dp1_bkey", None) == bkey
        self._dp1_bkey = bkey
        for phase in range(7):
            if reuse and phase == 0:
                continue
            ph = (1 | _lib.SPP_DP1_REUSE_BRACKET) if (reuse and phase == 1) else phase
            # pivot = the running mean itself (replicated across ranks): phase 6 reads pivot[c] before it
            # writes mean[c], in the same thread
            call("sppReplayObsStatsDP1", self._h, ph, W, R, ptr(self.obs_mean), ptr(self._dp1_samp),
                 ptr(self._dp1_exch), ptr(self._dp1_hist), n_global, ptr(self.obs_mean), ptr(self.obs_std),
                 ptr(self.max_obs), ptr(self.min_obs), first, stream_handle())
            if phase == 0:
                allgather(self._dp1_samp, mine)
            elif phase == 1:
                allreduce_sum(self._dp1_exch)
            elif phase <= 5:
                allreduce_sum(self._dp1_hist)
        self._have_minmax = True

    def obs_stats_dp_steps(self, n_global):
        """Generator over the stepwise protocol: yields after each step whose outputs
        (sums after step 0, hist after every step) must be all-reduced before the next."""
        self._dp_pivot.copy_(self.obs_mean)  # replicated across ranks
        done = ctypes.c_int(0)
        step = 0
        first = 0 if self._have_minmax else 1
        while True:
            call("sppReplayObsStatsDP", self._h, step, ptr(self._dp_pivot), ptr(self._dp_sums), ptr(self._dp_hist),
                 n_global, ptr(self.obs_mean), ptr(self.obs_std), ptr(self.max_obs), ptr(self.min_obs), first,
                 ctypes.byref(done), stream_handle())
            if done.value:
                break
            yield step
            step += 1
        self._have_minmax = True

    def normalize(self, obs, force=False):
        """BufferAcMOffPolicy.normalize (replay_buffer.py:77-81) -> MemoryMeta.normalize (memory.py:76-88)."""
        if not (self.obs_norm or force):
            return obs
        if self.min_max_denormalize and not self._have_minmax:
            return obs
        return self._norm(obs, 0)

    def denormalize(self, obs):
        """MemoryMeta.denormalize (memory.py:90-127)."""
        return self._norm(obs, 1)

    def _norm(self, obs, inverse):
        x = self._dev(obs)
        out = torch.empty_like(x)
        call("sppObsNormalize", ptr(x), x.numel() // self.obs_shape, self.obs_shape, ptr(self.min_obs),
             ptr(self.max_obs), ptr(self.obs_mean), ptr(self.obs_std), int(self.min_max_denormalize), int(inverse),
             ptr(out), stream_handle())
        return out


class ReplayBuffer(BufferAcMOffPolicy):
    """ReplayBuffer (rltoolkit/buffer/replay_buffer.py:99-261): the same HBM obs-index ring
    without the ACM action; ``sample_batch`` returns (obs, next_obs, action, reward, done)."""
    HAS_ACM = False

    def __init__(self, size, obs_shape, act_shape, device="cuda", **kw):
        super().__init__(size, obs_shape, act_shape, act_shape, device=device, **kw)

    def gather(self, idx):
        return super().gather(idx)[:5]

    def sample_acm_batch(self, batch_size=64):
        raise AttributeError("ReplayBuffer has no ACM actions")
