"""GPU parity of the PPO advantage / loss kernels.

Checked against the reference-generated fixture (tests/golden/ppo_gae_clip.npz),
the reference's own KATs (rltoolkit/algorithms/ppo/test/test_ppo.py:34-76,
79-134) and the oracle (oracle/ppo.py) on large random streams.
"""
import numpy as np
import pytest
import torch

from golden_cases import load
from oracle.ppo import clip_loss as o_clip_loss
from oracle.ppo import gae_loop, q_val

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def ppo():
    from spprl import ppo
    return ppo


def _t(x, dt=torch.float32):
    return torch.as_tensor(np.asarray(x)).to(DEV, dt)


@pytest.mark.parametrize("mode", [0, 1])
def test_gae_fixture(ppo, mode):
    fx = load("ppo_gae_clip")
    w = fx["w"]
    v_next = (fx["next_obs"] @ w).astype(np.float32)
    v = (fx["obs"] @ w).astype(np.float32)
    q, adv = ppo.calculate_gae(_t(fx["rew"]), _t(v), _t(v_next), _t(fx["done"]), _t(fx["end"]),
                               float(fx["gamma"]), float(fx["lam"]), mode=mode)
    np.testing.assert_allclose(q.cpu().numpy(), fx["q"], rtol=1e-6, atol=1e-6)
    tol = 1e-5 if mode == 0 else 2e-5
    np.testing.assert_allclose(adv.cpu().numpy(), fx["adv"], rtol=tol, atol=tol)


@pytest.mark.parametrize("mode", [0, 1])
def test_gae_reference_kat(ppo, mode):
    """rltoolkit/algorithms/ppo/test/test_ppo.py:79-134 (gamma = lambda = 0.5, V = 10)."""
    rew = np.array(list(range(10)) + [1, 2], np.float32)
    done = np.zeros(12, np.float32)
    done[[3, 6, 11]] = 1
    end = done.copy()
    end[9] = 1
    v = np.full(12, 10.0, np.float32)
    q, adv = ppo.calculate_gae(_t(rew), _t(v), _t(v), _t(done), _t(end), 0.5, 0.5, mode=mode)
    np.testing.assert_array_equal(q.cpu().numpy(), [5, 6, 7, 3, 9, 10, 6, 12, 13, 14, 6, 2])
    np.testing.assert_almost_equal(adv.cpu().numpy(),
                                   [-6.2969, -5.1875, -4.75, -7, -1.25, -1, -4, 3.1562, 4.625, 6.5, -6, -8], decimal=4)


def _random_streams(T, E, seed):
    rng = np.random.RandomState(seed)
    rew = rng.randn(T, E).astype(np.float32)
    v = rng.randn(T, E).astype(np.float32)
    vn = rng.randn(T, E).astype(np.float32)
    done = (rng.rand(T, E) < 0.01).astype(np.float32)
    end = ((rng.rand(T, E) < 0.005) | (np.arange(T)[:, None] == T - 1)).astype(np.float32)
    return rew, v, vn, done, end


def test_gae_sequential_bit_exact_vs_oracle(ppo):
    """mode 0 follows the reference's float32 operation order: bit-exact per stream."""
    T, E = 300, 257
    rew, v, vn, done, end = _random_streams(T, E, 3)
    q, adv = ppo.calculate_gae(_t(rew), _t(v), _t(vn), _t(done), _t(end), 0.99, 0.95, mode=0)
    q, adv = q.cpu().numpy(), adv.cpu().numpy()
    for e in range(0, E, 16):
        qe = q_val(rew[:, e], done[:, e], vn[:, e], 0.99)
        np.testing.assert_array_equal(q[:, e], qe)
        ae = gae_loop(qe - v[:, e], done[:, e], end[:, e], vn[:, e], 0.99, 0.95)
        np.testing.assert_array_equal(adv[:, e], ae)


def test_gae_scan_long_stream(ppo):
    """mode 1 (wavefront-shuffle scan) on streams longer than one 1024-step chunk."""
    T, E = 5000, 3
    rew, v, vn, done, end = _random_streams(T, E, 4)
    _, adv = ppo.calculate_gae(_t(rew), _t(v), _t(vn), _t(done), _t(end), 0.99, 0.95, mode=1)
    adv = adv.cpu().numpy()
    for e in range(E):
        qe = q_val(rew[:, e], done[:, e], vn[:, e], 0.99)
        ae = gae_loop((qe - v[:, e]).astype(np.float64), done[:, e], end[:, e], vn[:, e].astype(np.float64),
                      0.99, 0.95)
        np.testing.assert_allclose(adv[:, e], ae, rtol=1e-4, atol=1e-4)


def test_gae_empty_and_single(ppo):
    z = torch.zeros(0, device=DEV)
    q, adv = ppo.calculate_gae(z, z, z, z, z, 0.9, 0.9)
    assert adv.numel() == 0
    one = _t([1.0])
    q, adv = ppo.calculate_gae(one, one * 0.5, one * 2, _t([0.0]), _t([1.0]), 0.5, 0.5, mode=0)
    # q = 1 + 0.5*2 = 2; delta = 1.5; end bootstrap: 2*0.25 + 1.5 = 2.0
    assert q.item() == 2.0 and adv.item() == 2.0


@pytest.mark.parametrize("case", [
    ([-2.3, -5, -1.4, -1.5], [-2.3, -5, -1.4, -1.5], [1, 2.0, 3.0, 4.0], -2.5),
    ([-1.0], [-1.0], [-1.0], 1),
    ([-1.0], [-2.0], [-1.0], 0.8),
    ([-2.0], [-1.0], [1.0], -1.2),
    ([-1.0], [-2.0], [1.0], -0.3679),
])
def test_clip_loss_reference_kat(ppo, case):
    """rltoolkit/algorithms/ppo/test/test_ppo.py:34-76."""
    old, new, adv, want = case
    loss, kl, _ = ppo.clip_loss(_t(old), _t(new), _t(adv))
    assert loss.item() == pytest.approx(want, rel=1e-4)
    assert kl.item() == pytest.approx(float(np.mean(np.float32(old) - np.float32(new))), rel=1e-6, abs=1e-7)


def test_clip_loss_fixture_and_grad(ppo):
    fx = load("ppo_gae_clip")
    loss, kl, grad = ppo.clip_loss(_t(fx["clip_lp_old"]), _t(fx["clip_lp_new"]), _t(fx["clip_adv"]))
    assert loss.item() == pytest.approx(float(fx["clip_loss"]), rel=1e-6)
    # gradient vs torch autograd of the reference expression (ppo.py:199-203)
    old = torch.as_tensor(fx["clip_lp_old"])
    new = torch.as_tensor(fx["clip_lp_new"]).clone().requires_grad_(True)
    adv = torch.as_tensor(fx["clip_adv"])
    ratio = torch.exp(new - old)
    ref = -(torch.min(ratio * adv, torch.clamp(ratio, 0.8, 1.2) * adv)).mean()
    ref.backward()
    np.testing.assert_allclose(grad.cpu().numpy(), new.grad.numpy(), rtol=1e-5, atol=1e-7)


def test_clip_loss_large_batch(ppo):
    rng = np.random.RandomState(9)
    B = 100_003
    old = rng.randn(B).astype(np.float32) * 0.3 - 1
    new = old + rng.randn(B).astype(np.float32) * 0.2
    adv = rng.randn(B).astype(np.float32)
    loss, kl, grad = ppo.clip_loss(_t(old), _t(new), _t(adv))
    assert loss.item() == pytest.approx(o_clip_loss(old, new, adv), rel=1e-5)
    assert kl.item() == pytest.approx(float(np.mean(old.astype(np.float64) - new)), rel=1e-5)
    assert torch.isfinite(grad).all()


def test_normalize_advantages(ppo):
    rng = np.random.RandomState(2)
    a = (rng.randn(70_001) * 3 + 1.5).astype(np.float32)
    got = ppo.normalize_advantages(_t(a)).cpu().numpy()
    t = torch.as_tensor(a)
    want = ((t - t.mean()) / (t.std() + 1.2e-7)).numpy()
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)
