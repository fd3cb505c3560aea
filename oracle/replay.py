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
  last_end / last_rollout             :170-218, :335-383  the last complete episode, walked backwards
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

    def last_end(self, idx):  # :170-177 (python indexing: -1 is the array's last element)
        end = self._end[idx]
        while not end:
            idx -= 1
            if idx < 0:
                idx = self.current_len - 1
            end = self._end[idx]
        return idx

    def last_rollout(self):  # :335-383 -> (obs [T+1], actions, rewards, dones, actions_acm, ts indices)
        i = self.last_end(self.ts_idx - 1)  # -1 stays python's last element, as in the reference
        obs, actions, rewards, dones, acms, ts = [], [], [], [], [], []
        last_obs = self._obs[self._next_obs_idx[i]].astype(np.float32)
        next_end = False
        while not next_end:
            obs.insert(0, self._obs[self._obs_idx[i]].astype(np.float32))
            actions.insert(0, self._actions[i].astype(np.float32))
            rewards.insert(0, self._rewards[i])
            dones.insert(0, self._end[i])
            acms.insert(0, self._actions_acm[i].astype(np.float32))
            ts.insert(0, i % self.size)
            i -= 1
            if i < 0:
                i = self.current_len - 1
            next_end = self._end[i]
        obs.append(last_obs)
        return (np.stack(obs), np.stack(actions), np.array(rewards, np.float32), np.array(dones), np.stack(acms),
                np.array(ts))

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


def _fkey(x):
    """float32 -> order-preserving uint32 key (the device kernels' fkey)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)


def _funkey(k):
    k = np.uint64(k)
    u = (k & np.uint64(0x7FFFFFFF)) if (k & np.uint64(0x80000000)) else ((~k) & np.uint64(0xFFFFFFFF))
    return np.array([u], np.uint32).view(np.float32)[0]


def dp_obs_stats(shard, allreduce_sum, pivot):
    """Data-parallel update_obs_mean_std (replay_buffer.py:83-96) over the union of the
    ranks' shards, the protocol of sppReplayObsStatsDP restated: fp64 sums about a
    replicated pivot and 8-bit radix selects of numpy's 'linear' percentile neighbours
    (ranks floor((n-1)q) and +1) over histograms all-reduced across ranks.
    shard: (n_r, ob) float32.  allreduce_sum(np array) -> summed array.  Returns
    (mean, std, p99, p1) as float32."""
    x = np.asarray(shard, np.float32)
    ob = x.shape[1]
    d = x.astype(np.float64) - np.asarray(pivot, np.float32).astype(np.float64)
    sums = allreduce_sum(np.concatenate([d.sum(0), (d * d).sum(0)]))
    n = int(allreduce_sum(np.array([x.shape[0]], np.int64))[0])
    m1 = sums[:ob] / n
    mean = (np.asarray(pivot, np.float64) + m1).astype(np.float32)
    std = np.sqrt(np.maximum(sums[ob:] / n - m1 * m1, 0.0)).astype(np.float32)
    keys = _fkey(x)
    out = []
    for q in (0.99, 0.01):
        vi = (n - 1) * q
        lo = int(np.floor(vi))
        vals = []
        for rank in (lo, min(lo + 1, n - 1)):
            col = []
            for c in range(ob):
                prefix, mask, r = 0, 0, rank
                for shift in (24, 16, 8, 0):
                    sel = (keys[:, c] & np.uint64(mask)) == np.uint64(prefix)
                    h = np.bincount(((keys[sel, c] >> np.uint64(shift)) & np.uint64(255)).astype(np.int64),
                                    minlength=256).astype(np.int64)
                    h = allreduce_sum(h)
                    cum = np.cumsum(h)
                    b = int(np.searchsorted(cum, r, side="right"))
                    r -= int(cum[b - 1]) if b > 0 else 0
                    prefix |= b << shift
                    mask |= 255 << shift
                col.append(_funkey(prefix))
            vals.append(np.array(col, np.float64))
        g = vi - lo
        a, b = vals
        diff = b - a
        out.append(np.where(g >= 0.5, b - diff * (1.0 - g), a + diff * g).astype(np.float32))  # numpy _lerp
    return mean, std, out[0], out[1]
