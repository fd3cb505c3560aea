"""The vectorized training loop (spprl/trainer.py): reference cadence, fused schedule,
pre-train, test, host envs with side-stream copies.

CPU tests drive the loop's host logic with a stand-in agent (no device calls);
GPU tests run the real loop through libspprl.so on SynthVecEnv / HostVecEnv."""
import numpy as np
import pytest
import torch

from spprl import trainer
from spprl.trainer import OffPolicyLoop, StatsLogger


class _FakeEnv:
    is_host = False

    def __init__(self, n):
        self.n = n


class _FakeRB:
    def __init__(self):
        self.n = 0
        self.sampled = []

    def __len__(self):
        return self.n

    def sample_batch(self, B, device=None):
        self.sampled.append(B)
        return [None] * 6


class _FakeAgent(OffPolicyLoop):
    """Hopper SPP-SAC cadence (train/spp_sac_hopper.py): B=100, 50 grad steps every 50
    frames, ACM 100 batches of 100 every 1000 frames after iteration 0."""

    def __init__(self, n_envs=1, **kw):
        self.env_name, self.ob_dim, self.ac_dim, self.actor_output_dim = "Hopper-v2", 11, 3, 11
        self.device = torch.device("cpu")
        self.update_batch_size, self.acm_lr = 100, 1e-3
        self.replay_buffer = _FakeRB()
        self.updates, self.acm_batches = 0, 0
        args = dict(update_freq=50, grad_steps=50, acm_update_freq=1000, acm_update_batches=100, acm_batch_size=100,
                    acm_epochs=1, random_frames=1000, batch_size=1000)
        args.update(kw)
        self._init_loop(env=_FakeEnv(n_envs), **args)

    def update(self, *batch):
        self.updates += 1

    def update_acm_batches(self, n):
        self.acm_batches += n


def test_reference_cadence_counts():
    ag = _FakeAgent()
    assert ag.schedule == "reference"
    for it in range(3):
        ag.iteration = it
        for _ in range(1000):
            ag.stats_logger.frames += 1
            ag.replay_buffer.n += 1
            ag.make_update()
    # updates start once len > 100; frame 100 has len 100 (not >), first update at frame 150
    n_upd_frames = sum(1 for f in range(1, 3001) if f > 100 and f % 50 == 0)
    assert ag.updates == 50 * n_upd_frames
    assert set(ag.replay_buffer.sampled) == {100}
    # ACM: iteration > 0 and frames % 1000 == 0 -> frames 2000 and 3000
    assert ag.acm_batches == 200


def test_fused_schedule_preserves_replay_ratio():
    ag = _FakeAgent(n_envs=4096)
    assert ag.schedule == "fused"
    assert ag.rho == 100 and ag.sigma == 10
    assert ag.fused_batch_sizes() == (409600, 40960)
    ag2 = _FakeAgent(n_envs=8192, update_freq=500, grad_steps=1, update_batch_size=100, acm_update_freq=500,
                     acm_update_batches=200, acm_batch_size=128)
    assert ag2.fused_batch_sizes() == (int(round(8192 * 100 / 500)), int(round(8192 * 51.2)))


def test_stats_logger_running_return():
    s = StatsLogger()
    assert s.calc_running_return(None) is None
    assert s.calc_running_return(10.0) == 10.0
    assert abs(s.calc_running_return(20.0) - 11.0) < 1e-12  # 0.9 * 10 + 0.1 * 20


def test_max_frames_assertion():
    with pytest.raises(AssertionError):
        _FakeAgent(iterations=2, batch_size=10, max_frames=100)


def test_acm_step_lr_schedule():
    assert trainer.acm_lr_at(1e-3, 0.5, 25, 0) == 1e-3
    assert trainer.acm_lr_at(1e-3, 0.5, 25, 24) == 1e-3
    assert trainer.acm_lr_at(1e-3, 0.5, 25, 25) == 5e-4
    assert trainer.acm_lr_at(1e-3, 0.5, 25, 50) == 2.5e-4


# ------------------------------------------------------------------ GPU


def _sac(**kw):
    import spprl

    args = dict(env_name="Hopper-v2", gamma=0.99, acm_critic=True, custom_loss=0.2, norm_closs=False,
                min_max_denormalize=True, denormalize_actor_out=True, buffer_size=200_000, device="cuda:0", seed=0,
                update_freq=50, grad_steps=50, acm_update_freq=1000, acm_update_batches=100, acm_batch_size=100,
                acm_pre_train_samples=2000, acm_pre_train_epochs=2, random_frames=1000, loop_seed=3)
    args.update(kw)
    return spprl.SAC_AcM(**args)


@pytest.mark.gpu
def test_fused_sac_training_loop_runs():
    E = 256
    ag = _sac(n_envs=E, max_batch=100 * E, batch_size=4 * E, iterations=3, test_episodes=2)
    ag.pre_train()
    n0 = len(ag.replay_buffer)
    assert n0 >= 2000
    assert np.isfinite(ag.acm_loss)
    ag.train()
    torch.cuda.synchronize()
    assert ag.stats_logger.frames == 3 * 4 * E
    assert len(ag.replay_buffer) == n0 + 3 * 4 * E  # timesteps (replay_buffer.py:53-54)
    for k, v in ag.loss.items():
        assert np.isfinite(v), (k, v)
    assert np.isfinite(ag.acm_loss)
    assert np.isfinite(ag.stats_logger.test_return)


@pytest.mark.gpu
def test_reference_schedule_single_env():
    # 1 env, short synthetic episodes: every frame follows the reference cadence
    ag = _sac(n_envs=1, env_spec=(11, 3, 1.0, 120), batch_size=100, iterations=2, random_frames=50,
              update_freq=20, grad_steps=2, acm_update_freq=100, acm_update_batches=3)
    calls = []
    orig = ag.update

    def counting(*b, **k):
        calls.append(b[0].shape[0])
        return orig(*b, **k)

    ag.update = counting
    ag.train()
    torch.cuda.synchronize()
    # one 120-step episode per iteration (episodes run to their end, ddpg.py:192-223)
    assert ag.stats_logger.frames == 240
    assert len(ag.replay_buffer) == 240
    n_upd = sum(1 for f in range(1, 241) if f > 100 and f % 20 == 0)  # len == frames
    assert len(calls) == 2 * n_upd and set(calls) == {100}
    assert ag.stats_logger.running_return is not None
    for v in ag.loss.values():
        assert np.isfinite(v)


@pytest.mark.gpu
def test_fused_ddpg_training_loop_runs():
    import spprl

    E = 128
    ag = spprl.DDPG_AcM(env_name="HalfCheetah-v2", gamma=0.99, acm_critic=True, custom_loss=1.0, norm_closs=True,
                        min_max_denormalize=True, denormalize_actor_out=True, buffer_size=100_000, device="cuda:0",
                        seed=0, n_envs=E, batch_size=2 * E, iterations=2, update_freq=50, grad_steps=50,
                        acm_update_freq=500, acm_update_batches=200, acm_batch_size=128, random_frames=0,
                        max_batch=100 * E, acm_pre_train_samples=1000, acm_pre_train_epochs=1)
    ag.pre_train()
    ag.train()
    torch.cuda.synchronize()
    assert ag.stats_logger.frames == 4 * E
    for v in ag.loss.values():
        assert np.isfinite(v)


class _NpSynthEnv:
    """Host (numpy) SynthEnv, SURVEY.md Appendix A."""

    def __init__(self, ob=11, ac=3, T=50, seed=0):
        from types import SimpleNamespace

        self.observation_space = SimpleNamespace(shape=(ob,))
        rng = np.random.RandomState(seed)
        self.action_space = SimpleNamespace(shape=(ac,), sample=lambda: rng.uniform(-1, 1, ac).astype(np.float32))
        self._max_episode_steps, self._rng, self._t = T, rng, 0
        self._A = (rng.randn(ob, ob) * 0.05).astype(np.float32)

    def reset(self):
        self._t = 0
        self._s = self._rng.randn(self._A.shape[0]).astype(np.float32)
        return self._s.copy()

    def step(self, a):
        a = np.asarray(a, np.float32).reshape(-1)
        self._t += 1
        self._s = (np.tanh(self._A @ self._s) + 0.1 * np.resize(a, self._s.shape)).astype(np.float32)
        return self._s.copy(), float(-np.square(a).sum() + self._s[0]), self._t >= self._max_episode_steps, {}


@pytest.mark.gpu
def test_host_env_pool_pipelined_loop():
    from spprl.trainer import HostVecEnv

    envs = [_NpSynthEnv(T=30 + 7 * i, seed=i) for i in range(6)]  # ragged episode ends
    env = HostVecEnv(envs, device="cuda:0", env_fn=lambda: _NpSynthEnv(T=30))
    ag = _sac(env=env, max_batch=600, batch_size=60, iterations=4, random_frames=60, test_episodes=2)
    ag.train()
    torch.cuda.synchronize()
    assert ag.schedule == "fused" and ag.stats_logger.frames == 4 * 60
    ends = sum((40 // (30 + 7 * i)) for i in range(6))  # 240 frames = 40 steps of each env
    assert ag.stats_logger.rollouts == 6 + ends
    assert len(ag.replay_buffer) == 240
    for v in ag.loss.values():
        assert np.isfinite(v)
    assert np.isfinite(ag.stats_logger.test_return)


@pytest.mark.gpu
def test_ppo_acm_vectorized_loop_runs():
    import spprl

    ag = spprl.PPO_AcM(env_name="HalfCheetah-v2", n_envs=64, batch_size=1024, iterations=3, ppo_batch_size=256,
                       acm_pre_train_samples=2000, acm_pre_train_epochs=1, acm_update_freq=2, acm_epochs=1,
                       acm_batch_size=64, custom_loss=0.1, device="cuda:0", seed=0, test_episodes=2,
                       env_spec=(17, 6, 1.0, 40))
    ag.pre_train()
    ag.train()
    torch.cuda.synchronize()
    assert ag.T == 16 and ag.stats_logger.frames == 3 * 1024
    assert np.isfinite(ag.loss["critic"]) and np.isfinite(ag.loss["actor"]) and np.isfinite(ag.loss["kl"])
    assert ag.stats_logger.running_return is not None
    assert np.isfinite(ag.stats_logger.test_return)


@pytest.mark.gpu
def test_ppo_acm_single_env_collects_whole_episodes():
    import spprl

    ag = spprl.PPO_AcM(env_name="HalfCheetah-v2", n_envs=1, batch_size=100, iterations=1, ppo_batch_size=64,
                       acm_pre_train_samples=300, acm_pre_train_epochs=1, acm_update_freq=1, acm_epochs=1,
                       device="cuda:0", seed=0, env_spec=(17, 6, 1.0, 60))
    ag.pre_train()
    mem = ag.collect_batch()
    assert mem["T"] == 120  # two 60-step episodes (a2c.py:155-184 finishes the episode in progress)
    assert int(mem["end"].sum()) == 2 and int(mem["done"].sum()) == 0  # time-limit ends are not terminal
    ag.update(mem)
    torch.cuda.synchronize()
    assert np.isfinite(ag.loss["critic"])


@pytest.mark.gpu
def test_acm_act_given_action_matches_oracle():
    """sppPolicyAct mode 3 (on-policy process_action): env action = AcM(cat(obs, denorm(a)))."""
    import spprl
    from oracle import nets as onets

    ag = spprl.SAC_AcM(env_name="HalfCheetah-v2", min_max_denormalize=True, denormalize_actor_out=True,
                       max_batch=256, buffer_size=64, device="cuda:0", seed=3)
    rb = ag.replay_buffer
    rng = np.random.RandomState(0)
    lo, hi = -rng.uniform(0.5, 2, 17).astype(np.float32), rng.uniform(0.5, 2, 17).astype(np.float32)
    rb.min_obs.copy_(torch.from_numpy(lo))
    rb.max_obs.copy_(torch.from_numpy(hi))
    rb._have_minmax = True
    E = 77
    obs = torch.from_numpy(rng.randn(E, 17).astype(np.float32))
    a = torch.from_numpy(rng.uniform(-1.2, 1.2, (E, 17)).astype(np.float32))
    tgt, env = ag.act(obs.cuda(), eps=a.cuda(), mode=3)
    P = {n: torch.as_tensor(v) for n, v in ag.net_state(5).items()}
    ad = torch.from_numpy(lo + (hi - lo) / 2) * 0 + (torch.from_numpy((hi + lo) / 2) + a * torch.from_numpy((hi - lo) / 2))
    ref = onets.acm(P, torch.cat([obs, ad], 1), ag.ac_lim)
    np.testing.assert_allclose(tgt.cpu().numpy(), ad.numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(env.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)


# ------------------------------------------------------------------ advisor round-1 regressions
def test_default_max_batch_covers_fused_schedule():
    """SAC_AcM(n_envs=E) without max_batch must size its scratch for rho*E (and sigma*E)."""
    from spprl import config

    kw = dict(n_envs=4096, grad_steps=50, update_freq=50, acm_update_batches=100, acm_batch_size=100,
              acm_update_freq=1000)
    assert config.default_max_batch(100, kw) == 409_600
    kw = dict(n_envs=8192, acm_update_batches=200, acm_batch_size=128, acm_update_freq=500)
    assert config.default_max_batch(100, kw) == max(819_200, 419_430)
    assert config.default_max_batch(100, dict(n_envs=1)) == 128  # reference cadence: B and acm batch
    assert config.default_max_batch(100, dict(env=_FakeEnv(64), schedule="reference")) == 128


def test_dp_obs_stats_count_is_all_reduced_not_assumed():
    """Under DP the obs-stats call must not assume equal shard lengths (resets advance the
    obs rings unevenly): the trainer passes no n_global, so the buffer all-reduces it."""
    calls = []

    class RB(_FakeRB):
        def update_obs_mean_std_dp(self, allreduce_sum, n_global=None, host_sum=None, allgather=None):
            calls.append((n_global, host_sum))

    def host_sum(x):  # the shard lengths are summed on the host (spprl.dp.make_host_allreduce_sum)
        return x

    ag = _FakeAgent(n_envs=4)
    ag.replay_buffer = RB()
    ag.allreduce_sum = lambda t: t
    ag.host_sum = host_sum
    ag.update_obs_stats()
    assert calls == [(None, host_sum)]


def test_stream_keys_are_distinct_per_consumer():
    from spprl.dp import stream_key

    tags = ("policy", "index", "update_eps", "env", "env_action")
    keys = [stream_key(s, t) for s in (0, 1, 1000, 2000) for t in tags]
    assert len(set(keys)) == len(keys)
    assert all(0 <= k < (1 << 63) for k in keys)


class _RecordingEnv(_NpSynthEnv):
    """Records every terminal observation it returns (episode end)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.terminal = []

    def step(self, a):
        o, r, d, info = super().step(a)
        if d:
            self.terminal.append(o.copy())
        return o, r, d, info


@pytest.mark.gpu
def test_host_env_terminal_next_obs_survives_reset():
    """A terminal transition's next_obs must be the env's terminal observation even though
    the reset observation is written to the pinned staging right after (the
    queued H2D copy used to pick up the reset row)."""
    from spprl.trainer import HostVecEnv

    envs = [_RecordingEnv(T=5 + 3 * i, seed=i) for i in range(6)]
    env = HostVecEnv(envs, device="cuda:0")
    ag = _sac(env=env, max_batch=600, batch_size=60, iterations=3, random_frames=30, buffer_size=10_000)
    ag.train()
    torch.cuda.synchronize()
    rb = ag.replay_buffer
    n = len(rb)
    obs, nobs, act, rew, done, acm = rb.gather(torch.arange(n))
    got = nobs[done.bool()].cpu().numpy()
    want = np.concatenate([np.stack(e.terminal) for e in envs if e.terminal])
    assert got.shape == want.shape
    key = lambda a: a[np.lexsort(a.T[::-1])]  # noqa: E731  (compare as multisets of rows)
    np.testing.assert_array_equal(key(got), key(want))


@pytest.mark.gpu
def test_agent_with_many_envs_needs_no_max_batch():
    E = 64
    ag = _sac(n_envs=E, batch_size=2 * E, iterations=1, random_frames=0)
    assert ag.max_batch >= 100 * E
    ag.train()
    torch.cuda.synchronize()
    assert all(np.isfinite(v) for v in ag.loss.values())
