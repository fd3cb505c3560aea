"""CPU-baseline calibration, build container only (needs /root/reference): time the
reference's own SAC_AcM.update (rltoolkit/acm/off_policy/sac_acm.py:89-162, B = 100, Hopper paper flags,
torch.set_num_threads(1)) next to the port's (oracle/sac_acm.py) on the same batches, and split both by phase.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_calibrate.py [steps]
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

_orig_normal = torch.distributions.normal._standard_normal
import make_golden as mg  # noqa: E402  (the reference behind the Appendix-A dependency stand-ins)

torch.distributions.normal._standard_normal = _orig_normal  # make_golden injects eps queues: undo
from golden_cases import make_batch  # noqa: E402
from oracle import nets as onets  # noqa: E402
from oracle.nets import Norm  # noqa: E402
from oracle.sac_acm import OracleSacAcm  # noqa: E402

torch.set_num_threads(1)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
B, ob, ac = 100, 11, 3
flags = dict(acm_critic=True, custom_loss=0.2, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True)
torch.manual_seed(0)
ref = mg.SAC_AcM(env_name="Hopper-v2", gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2,
                 buffer_size=1000, acm_pre_train_samples=10, acm_val_buffer_size=None, update_batch_size=B,
                 use_gpu=False, **flags)
rng = np.random.RandomState(0)
lo = -rng.uniform(0.5, 2.0, ob).astype(np.float32)
hi = rng.uniform(0.5, 2.0, ob).astype(np.float32)
ref.replay_buffer.min_obs, ref.replay_buffer.max_obs = torch.from_numpy(lo), torch.from_numpy(hi)
batches = [make_batch(rng, B, ob, ob, ac) for _ in range(8)]
tb = [[torch.from_numpy(x) for x in b] for b in batches]


def timeit(fn, n):
    for i in range(5):
        fn(i)
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    return (time.perf_counter() - t0) / n * 1e3


ref_ms = timeit(lambda i: ref.update(*tb[i % 8]), steps)
params = {k: {n: v.detach().numpy().copy() for n, v in m.state_dict().items()}
          for k, m in (("actor", ref._actor), ("critic_1", ref._critic_1), ("critic_2", ref._critic_2),
                       ("critic_1_targ", ref.critic_1_targ), ("critic_2_targ", ref.critic_2_targ), ("acm", ref.acm))}
norm = Norm(True, torch.from_numpy(lo), torch.from_numpy(hi))
port = OracleSacAcm(ob, ob, ac, acm_critic=True, custom_loss=0.2, norm_closs=False, norm=norm,
                    actor_lim=ref.actor_ac_lim.numpy(), acm_lim=np.asarray(ref.acm.ac_lim, np.float32), gamma=0.99,
                    params=params)
eps = [(rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32)) for _ in range(8)]
port_ms = timeit(lambda i: port.update(*batches[i % 8], *eps[i % 8]), steps)
print("SAC_AcM.update, B = %d, 1 thread, %d steps: reference %.3f ms, port %.3f ms (ref / port %.2f)"
      % (B, steps, ref_ms, port_ms, ref_ms / port_ms))
# where the reference spends it: torch's own profiler over 50 updates, top operators by self CPU time
from torch.profiler import ProfilerActivity, profile  # noqa: E402

for name, fn in (("reference", lambda i: ref.update(*tb[i % 8])),
                 ("port", lambda i: port.update(*batches[i % 8], *eps[i % 8]))):
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for i in range(50):
            fn(i)
    print("==", name)
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=14))

# the port with the reference's optimizer object: torch.optim.Adam (the single-tensor CPU path the reference's
# Adam takes, rl.py:62 / sac.py:107-110) stepping .grad, instead of the restated OracleAdam
class TorchAdam:
    def __init__(self, params, lr):
        self.params = list(params)
        self.o = torch.optim.Adam(self.params, lr=lr)

    def step(self, grads):
        for p, g in zip(self.params, grads):
            p.grad = g
        self.o.step()
        self.o.zero_grad(set_to_none=True)


port2 = OracleSacAcm(ob, ob, ac, acm_critic=True, custom_loss=0.2, norm_closs=False, norm=norm,
                     actor_lim=ref.actor_ac_lim.numpy(), acm_lim=np.asarray(ref.acm.ac_lim, np.float32), gamma=0.99,
                     params=params)
for k in ("actor", "critic_1", "critic_2"):
    port2.opt[k] = TorchAdam(port2.p[k].values(), 1e-3)
port2.opt_alpha = TorchAdam([port2.log_alpha], 1e-3)
p2_ms = timeit(lambda i: port2.update(*batches[i % 8], *eps[i % 8]), steps)
ref2_ms = timeit(lambda i: ref.update(*tb[i % 8]), steps)
port_again = timeit(lambda i: port.update(*batches[i % 8], *eps[i % 8]), steps)
print("again: reference %.3f ms, port %.3f ms, port with torch.optim.Adam %.3f ms (ref / port-torch-adam %.2f)"
      % (ref2_ms, port_again, p2_ms, ref2_ms / p2_ms))
