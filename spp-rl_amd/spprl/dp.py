"""Data-parallel plumbing for the SPP-SAC hot path.

One process per GPU.  Each rank steps its own E envs into a local replay shard,
samples rho*E transitions from it and computes gradients locally; the flat
gradient buckets of ``SAC_AcM`` ([critic_1|critic_2], [actor|alpha operand],
[acm]) are averaged across ranks between the ``*Grads`` and ``*Apply`` halves
of the update, so every rank applies the identical Adam step and the replicas
stay bit-identical.  With equal shard batches the average of per-rank mean-loss
gradients equals the full-batch mean-loss gradient (all losses of the path are
batch means: sac_acm.py:97-131, :60-87, sac.py:201-216, acm.py:356-372).
"""
import os

import torch.distributed as dist


def _single_rank_exchange():
    """SPP_DP_FORCE=1 keeps the exchange on with a one-rank group: the RCCL path (bucket
    all-reduce, the stepwise global obs statistics) then runs on a single GPU, which is how it
    is rehearsed on a one-GPU box (tests/test_gpu_dp_rccl.py).  Results equal the N = 1 path."""
    return os.environ.get("SPP_DP_FORCE", "0") == "1"


def make_allreduce(group=None):
    """Returns ``allreduce(bucket)`` (in-place average over the group) or None
    when the group has a single rank.  On ROCm the "nccl" backend is RCCL."""
    if not dist.is_available() or not dist.is_initialized():
        return None
    world = dist.get_world_size(group)
    if world == 1 and not _single_rank_exchange():
        return None
    inv = 1.0 / world

    def allreduce(bucket):
        dist.all_reduce(bucket, group=group)
        bucket.mul_(inv)

    return allreduce


def make_allreduce_sum(group=None):
    """Returns ``allreduce_sum(t)`` (in-place sum over the group; exact for integer
    histograms, fp64 for moment sums) or None with a single rank."""
    if not dist.is_available() or not dist.is_initialized():
        return None
    if dist.get_world_size(group) == 1 and not _single_rank_exchange():
        return None

    def allreduce_sum(t):
        dist.all_reduce(t, group=group)

    return allreduce_sum


class _AllGather:
    """Rank-major all-gather over a torch.distributed group: ``ag(out, inp)`` with out = world x inp
    (inp may be this rank's slice of out); ``world`` / ``rank`` of the group."""

    def __init__(self, group):
        self.group, self.world, self.rank = group, dist.get_world_size(group), dist.get_rank(group)

    def __call__(self, out, inp):
        dist.all_gather_into_tensor(out, inp, group=self.group)


def make_allgather(group=None):
    """The one-pass obs-statistics sample exchange (spprl.replay.update_obs_mean_std_dp) or None with a
    single rank."""
    if not dist.is_available() or not dist.is_initialized():
        return None
    if dist.get_world_size(group) == 1 and not _single_rank_exchange():
        return None
    if os.environ.get("SPP_DP_STATS", "onepass") == "stepwise":  # A/B: the stepwise radix protocol
        return None
    return _AllGather(group)


_HOST_GROUPS = {}


def make_host_allreduce_sum(group=None):
    """Returns ``host_sum(x) -> int`` (sum of a host integer over the group; a list of integers gives the
    list of sums) or None with a single rank.  Host-known counts (the shards' live row counts) are
    exchanged as CPU tensors over gloo: no device tensor, so no device synchronisation on the way.  For a
    group on another backend a gloo group over the SAME ranks is created once per distinct rank set (and
    per default group: it is rebuilt after the default group is destroyed and re-initialised); every
    rank OF THE DEFAULT GROUP must call this in the same order, also for a subgroup it is not in
    (``dist.new_group`` is collective over the default group; the agents' constructors do)."""
    if not dist.is_available() or not dist.is_initialized():
        return None
    if dist.get_world_size(group) == 1 and not _single_rank_exchange():
        return None
    import torch

    g = group
    if dist.get_backend(group) != "gloo":
        ranks = tuple(dist.get_process_group_ranks(group if group is not None else dist.group.WORLD))
        world = dist.group.WORLD
        ent = _HOST_GROUPS.get(ranks)
        # keyed by rank set, validated by the identity of the default group it was made under (an id() of a
        # destroyed default group may be reused by its successor; the object itself is held here)
        if ent is None or ent[0] is not world:
            # new_group is collective over the DEFAULT group: every rank of it must reach this line, also
            # for a subgroup it is not a member of
            ent = (world, dist.new_group(ranks=list(ranks), backend="gloo"))
            _HOST_GROUPS[ranks] = ent
        g = ent[1]

    def host_sum(x):
        many = isinstance(x, (list, tuple))
        t = torch.tensor([int(v) for v in x] if many else [int(x)], dtype=torch.int64)
        dist.all_reduce(t, group=g)
        return [int(v) for v in t.tolist()] if many else int(t.item())

    return host_sum


def stream_key(seed, tag):
    """Philox key of one random-stream consumer (policy eps, replay indices, update eps, env
    resets, env actions): splitmix64 of (seed, tag), so consumers sharing a seed never share
    a (key, counter) pair."""
    import zlib

    m = (1 << 64) - 1
    z = (int(seed) * 0x9E3779B97F4A7C15 + zlib.crc32(tag.encode()) * 0xD1B54A32D192ED03) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return (z ^ (z >> 31)) & ((1 << 63) - 1)


def shard_seed(base, rank):
    """Per-rank seed of the env / sampling / eps streams (ranks must differ)."""
    return int(base) + 1000 * int(rank)


def shard_batch(B, world):
    """Per-rank minibatch of a global batch B (equal shards keep the mean exact)."""
    if B % world:
        raise ValueError("global batch %d not divisible by world size %d" % (B, world))
    return B // world


class NativeComm:
    """An RCCL communicator owned by libspprl (sppCommGetUniqueId / sppCommInitRank), for hosts
    that run the §8e exchange through the C-ABI (sppAllReduceGrads) rather than
    torch.distributed.  ``share_uid(buf)`` ships rank 0's 128-byte id to every rank (any channel,
    e.g. a gloo broadcast) and returns it."""

    def __init__(self, rank, world, device, share_uid):
        import ctypes

        from . import _lib

        self.rank, self.world = int(rank), int(world)
        uid = ctypes.create_string_buffer(_lib.SPP_COMM_ID_BYTES)
        if self.rank == 0:
            _lib.call("sppCommGetUniqueId", uid)
        raw = share_uid(bytes(uid.raw))
        uid = ctypes.create_string_buffer(bytes(raw), _lib.SPP_COMM_ID_BYTES)
        self.comm = ctypes.c_void_p()
        _lib.call("sppCommInitRank", ctypes.byref(self.comm), self.world, uid, self.rank, int(device))

    def allreduce_sum(self, t):
        """In-place sum of a device tensor over the communicator (fp32 / fp64 / int32 / int64 / uint32:
        the obs-statistics exchange), on the current stream (sppCommAllReduceSum)."""
        from . import _lib

        import torch

        code = {torch.float32: 0, torch.float64: 1, torch.int32: 2, torch.int64: 3}[t.dtype]
        _lib.call("sppCommAllReduceSum", self.comm, _lib.ptr(t), t.numel(), code, _lib.stream_handle())

    def host_sum(self, x):
        """Sum of host integers over the communicator (one small device all-reduce + a host read)."""
        import torch

        many = isinstance(x, (list, tuple))
        t = torch.tensor([int(v) for v in x] if many else [int(x)], dtype=torch.int64, device="cuda")
        self.allreduce_sum(t)
        return [int(v) for v in t.tolist()] if many else int(t.item())

    def allgather(self, out, inp):
        """Rank-major all-gather of device tensors over the communicator (sppCommAllGather)."""
        from . import _lib

        _lib.call("sppCommAllGather", self.comm, _lib.ptr(inp), _lib.ptr(out), inp.numel() * inp.element_size(),
                  _lib.stream_handle())

    def attach(self, agent):
        """Run ``agent``'s data-parallel exchange over this communicator: gradient buckets, the
        obs-statistics sums and the row counts (all three are needed: with the gradients averaged but the
        statistics per rank, the replicas' normalisers would drift apart)."""
        agent.allreduce = self.allreduce_for(agent)
        agent.allreduce_sum = self.allreduce_sum
        agent.host_sum = self.host_sum
        agent.allgather = self  # world / rank / __call__ (one-pass obs statistics)
        return agent

    def __call__(self, out, inp):
        self.allgather(out, inp)

    def allreduce_for(self, agent):
        """``allreduce(bucket)`` over the agent's exchange buckets (bucket_critic / _actor / _acm),
        averaged in place on the current stream by sppAllReduceGrads."""
        from . import _lib

        ids = {id(agent.bucket_critic): _lib.SPP_BUCKET_CRITIC, id(agent.bucket_actor): _lib.SPP_BUCKET_ACTOR,
               id(agent.bucket_acm): _lib.SPP_BUCKET_ACM}

        def allreduce(bucket):
            _lib.call("sppAllReduceGrads", agent._h, ids[id(bucket)], self.world, self.comm, _lib.stream_handle())

        return allreduce

    def close(self):
        from . import _lib

        if self.comm:
            _lib.call("sppCommDestroy", self.comm)
            self.comm = None
