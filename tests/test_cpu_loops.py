"""The CPU-baseline loops bench.py times (oracle/cpu_loop.py, oracle/cpu_loop_ppo.py), at toy sizes:
they run the reference cadence (frames, replay growth, ACM cycle) and stay finite."""
import numpy as np
import torch

from oracle.cpu_loop import CpuLoop
from oracle.cpu_loop_ppo import PpoCpuLoop


def test_off_policy_cpu_loop_cadence():
    L = CpuLoop("sac_acm", 11, 3, update_batch_size=16, update_freq=10, grad_steps=2, acm_update_freq=20,
                acm_update_batches=2, acm_batch_size=16, batch_size=25, buffer_size=5000, prefill=200)
    fps, n, el = L.run(0.2)
    assert fps > 0 and n == L.frames and L.frames % 10 == 0
    assert len(L.rb) == 200 + n


def test_ppo_cpu_loop_iteration_cycle():
    L = PpoCpuLoop(batch_size=120, ring=2000, prefill=1000, acm_epochs=1, acm_batch_size=64, ep_len=40,
                   critic_target_updates=2, critic_updates_per_target=2, max_ppo_epochs=2, ppo_batch_size=64)
    w0 = [t.detach().clone() for t in L.acm.values()]
    fps, n, el = L.run()  # one ACM cycle: 3 iterations, the ACM epochs on the third
    assert fps > 0 and n >= 3 * 120 and L.iteration == 4
    assert len(L.rb) == 1000 + n
    assert any(not torch.equal(a, b) for a, b in zip(w0, L.acm.values()))
    assert np.all(np.isfinite(L.mean)) and np.all(L.std > 0)
