"""Data-parallel SAC_AcM update through the HIP kernels against one process on the union batch (SURVEY.md §8e;
acm/off_policy/sac_acm.py:89-162): 2 processes on one GPU over gloo, each running the split update
(sppSacAcmCriticGrads -> bucket all-reduce -> CriticApply -> ActorGrads -> bucket all-reduce -> ActorApply, the
exchange points bench.py's N > 1 runs use) on its half of the reference-fixture batch (sac_hopper_paper, B = 100,
2 steps).  Checks: both replicas bit-identical; the averaged gradient buckets equal the single-process HIP update's
gradients on the whole batch (the mean of equal-size shard means is the batch mean: relative error < 1e-5, fp32
summation order only); the post-step parameters equal the single process's within Adam's first-step allowance
(and the reference fixture's)."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from golden_cases import sac_case
from rank_results import collect

pytestmark = pytest.mark.gpu
CASE, WORLD = "sac_hopper_paper", 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _build(cfg, fx, params, norm, B):
    import spprl
    from spprl import _lib

    ob, aout, ac = (int(v) for v in fx["dims"][:3])
    ag = spprl.SAC_AcM(env_name="custom", env_spec=(ob, ac, 1.0, 1000), gamma=float(fx["gamma"]),
                       acm_critic=cfg["acm_critic"], custom_loss=cfg["custom_loss"], norm_closs=cfg["norm_closs"],
                       min_max_denormalize=cfg["min_max"], denormalize_actor_out=cfg["min_max"],
                       alpha=float(fx["alpha0"]), max_batch=B, buffer_size=64, device="cuda:0")
    names = {"actor": _lib.SPP_NET_ACTOR, "critic_1": _lib.SPP_NET_CRITIC1, "critic_2": _lib.SPP_NET_CRITIC2,
             "critic_1_targ": _lib.SPP_NET_CRITIC1_TARG, "critic_2_targ": _lib.SPP_NET_CRITIC2_TARG,
             "acm": _lib.SPP_NET_ACM}
    for k, net in names.items():
        ag.load_net(net, params[k])
    rb = ag.replay_buffer
    for dst, src in ((rb.min_obs, norm.lo), (rb.max_obs, norm.hi), (rb.obs_mean, norm.mean), (rb.obs_std, norm.std)):
        dst.copy_(src)
    rb._have_minmax = True
    return ag, names


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from spprl import _lib
        from spprl.dp import make_allreduce

        torch.cuda.set_device(0)
        cfg, fx, params, layouts, norm, steps = sac_case(CASE)
        B = int(fx["dims"][3])
        b = B // WORLD
        sl = slice(rank * b, (rank + 1) * b)
        ag, names = _build(cfg, fx, params, norm, b)
        allreduce = make_allreduce()
        assert allreduce is not None
        st = _lib.stream_handle()
        buckets = []
        for batch, e1, e2 in steps:
            bt, keep = ag._batch(*(x[sl] for x in batch))
            d1 = torch.from_numpy(np.ascontiguousarray(e1[sl])).cuda()
            d2 = torch.from_numpy(np.ascontiguousarray(e2[sl])).cuda()
            _lib.call("sppSacAcmCriticGrads", ag._h, ctypes.byref(bt), _lib.ptr(d1), _lib.ptr(ag._losses), st)
            allreduce(ag.bucket_critic)
            _lib.call("sppSacAcmCriticApply", ag._h, st)
            _lib.call("sppSacAcmActorGrads", ag._h, _lib.ptr(d2), _lib.ptr(ag._losses), st)
            allreduce(ag.bucket_actor)
            _lib.call("sppSacAcmActorApply", ag._h, _lib.ptr(ag._losses), st)
            torch.cuda.synchronize()
            buckets.append((ag.bucket_critic.cpu().numpy().copy(), ag.bucket_actor.cpu().numpy().copy()))
        q.put((rank, buckets, {k: ag.params[n].cpu().numpy() for k, n in names.items()}, ag.current_alpha()))
    finally:
        dist.destroy_process_group()


def test_dp_sac_kernels_equal_one_process_on_the_union_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = collect(q, procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (bk0, p0, al0), (bk1, p1, al1) = res[0], res[1]
    for k in p0:
        np.testing.assert_array_equal(p0[k], p1[k], err_msg=k)  # replicas bit-identical
    assert al0 == al1
    cfg, fx, params, layouts, norm, steps = sac_case(CASE)
    B = int(fx["dims"][3])
    one, names = _build(cfg, fx, params, norm, B)
    for i, (batch, e1, e2) in enumerate(steps):
        one.update(*batch, eps_next=e1, eps_cur=e2)
        torch.cuda.synchronize()
        for got, want in ((bk0[i][0], one.bucket_critic.cpu().numpy()), (bk0[i][1], one.bucket_actor.cpu().numpy())):
            err = np.linalg.norm(got.astype(np.float64) - want) / np.linalg.norm(want.astype(np.float64))
            assert err < 1e-5, (i, err)
    lr = 1e-3
    for k in ("actor", "critic_1", "critic_2", "critic_1_targ", "critic_2_targ"):
        for want in (one.params[names[k]].cpu().numpy(), fx["post_" + k]):
            d = np.abs(p0[k] - want)
            assert d.max() <= 2 * len(steps) * lr * 1.01, (k, d.max())
            assert np.mean(d > 1e-5) < 2e-3, (k, np.mean(d > 1e-5))
    assert al0 == pytest.approx(one.current_alpha(), rel=1e-5)
