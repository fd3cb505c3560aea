"""ORACLE (test infrastructure only): the off-policy SPP replay ring.

Restates rltoolkit/buffer/replay_buffer.py (reference @ v0):
  MetaReplayBuffer.add_obs            :56-60   obs ring, slot = obs_idx, advance mod size
  MetaReplayBuffer.add_timestep       :65-75   index pair + payload at ts_idx; wrap rule (Q6)
  ReplayBuffer.addition               :133-137 action / reward / done / end payload
  BufferAcMOffPolicy.add_acm_action   :332-333 env action stored at ts_idx before add_timestep
  ReplayBuffer._sample_batch          :233-261 idx = randint(0, len, B); gather; fp32 / int8 casts
  BufferAcMOffPolicy.sample_batch     :385-398 + acm actions
  rbuffer_sample_acm                  :404-430
  MetaReplayBuffer.update_obs_mean_std :83-96  fp64 mean, std (ddof=0), percentile 99/1, running max/min
Storage is float64 as in the reference (Q5); every stored value comes from a
float32 tensor so fp32 round-trips are exact.
"""
import numpy as np


class OracleReplay:
    def __init__(self, size, ob, aout, ac):
        self.size, self.ob, self.aout, self.ac = size, ob, aout, ac
        self.obs_idx = 0
        self.ts_idx = 0
        self.current_len = 0
        self._obs = np.zeros((size, ob))
        self._obs_idx = np.zeros(size, np.int64)
        self._next_obs_idx = np.zeros(size, np.int64)
        self._actions = np.zeros((size, aout))
        self._actions_acm = np.zeros((size, ac))
        self._rewards = np.zeros(size, np.float32)
        self._done = np.zeros(size, np.bool_)
        self._end = np.zeros(size, np.bool_)
        # ReplayBuffer.__init__ :113-115 — identity normalizer until the first stats update
        self.obs_mean = np.zeros(ob, np.float32)
        self.obs_std = np.ones(ob, np.float32)
        self.max_obs = self.min_obs = None

    def __len__(self):
        return self.current_len

    def add_obs(self, obs):
        self._obs[self.obs_idx] = np.asarray(obs, np.float32).reshape(-1)
        i = self.obs_idx
        self.obs_idx = (self.obs_idx + 1) % self.size
        return i

    def add_acm_action(self, acm):
        self._actions_acm[self.ts_idx] = np.asarray(acm, np.float32).reshape(-1)

    def add_timestep(self, obs_idx, next_obs_idx, action, rew, done, end):
        t = self.ts_idx
        self._obs_idx[t] = obs_idx
        self._next_obs_idx[t] = next_obs_idx
        self._actions[t] = np.asarray(action, np.float32).reshape(-1)
        self._rewards[t] = rew
        self._done[t] = done
        self._end[t] = end
        if next_obs_idx < self.ts_idx:
            self.current_len = self.ts_idx + 1
            self.ts_idx = 0
        else:
            self.ts_idx += 1
        self.current_len = max(self.ts_idx, self.current_len)

    def gather(self, idx):
        o = self._obs[self._obs_idx[idx]].astype(np.float32)
        no = self._obs[self._next_obs_idx[idx]].astype(np.float32)
        return (o, no, self._actions[idx].astype(np.float32), self._rewards[idx].astype(np.float32),
                self._done[idx].astype(np.int8), self._actions_acm[idx].astype(np.float32))

    def sample_batch(self, B, mt):
        """mt: object with randint(high, n) (numpy-legacy compatible stream)."""
        idx = mt.randint(len(self), B)
        return self.gather(idx), idx

    def sample_acm_batch(self, B, mt):
        idx = mt.randint(len(self), B)
        o, no, _, _, _, acm = self.gather(idx)
        return (o, no, acm), idx

    def live_obs(self):
        return self._obs[self._obs_idx[: self.current_len]]

    def update_obs_mean_std(self):
        obs = self.live_obs()
        if len(obs) <= 10:
            return
        self.obs_mean = obs.mean(axis=0).astype(np.float32)
        self.obs_std = obs.std(axis=0).astype(np.float32)
        cur_max = np.percentile(obs, 99, axis=0).astype(np.float32)
        cur_min = np.percentile(obs, 1, axis=0).astype(np.float32)
        if self.max_obs is None or self.min_obs is None:
            self.max_obs, self.min_obs = cur_max, cur_min
        else:
            self.max_obs = np.maximum(cur_max, self.max_obs)
            self.min_obs = np.minimum(cur_min, self.min_obs)


def percentile_linear(col_sorted, q):
    """numpy 'linear' percentile on an ascending fp64 column (restated for the
    device radix-select check): virtual index v = q/100*(n-1), lerp between
    floor/ceil order statistics with numpy's _lerp form."""
    n = len(col_sorted)
    v = q / 100.0 * (n - 1)
    lo = int(np.floor(v))
    hi = min(lo + 1, n - 1)
    g = v - lo
    a, b = col_sorted[lo], col_sorted[hi]
    diff = b - a
    return (b - diff * (1 - g)) if g >= 0.5 else (a + diff * g)
