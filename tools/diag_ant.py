import sys
import numpy as np
import torch
sys.path[:0] = ["spp-rl_amd", "tests", "tests/golden", "."]
import test_gpu_parity as T  # noqa: E402
from spprl import _lib  # noqa: E402

DEV = T.DEV
ob, ac, B = 111, 8, 613
outs = []
for trial in range(3):
    a2 = T._filled_agent("Ant-v2", ob, ac, 3000)
    idx = torch.from_numpy(np.random.RandomState(5).randint(0, 3000, B)).to(DEV)
    rng = np.random.RandomState(9)
    e1 = torch.from_numpy(rng.randn(B, ob).astype(np.float32)).to(DEV)
    e2 = torch.from_numpy(rng.randn(B, ob).astype(np.float32)).to(DEV)
    a2.update(*a2.replay_buffer.gather(idx), eps_next=e1, eps_cur=e2)
    torch.cuda.synchronize()
    outs.append({k: a2.params[k].cpu().numpy().copy() for k in (_lib.SPP_NET_ACTOR, _lib.SPP_NET_CRITIC1)})
    print("trial", trial, a2.loss, flush=True)
for k in outs[0]:
    for t in (1, 2):
        d = np.abs(outs[0][k] - outs[t][k])
        print("net", k, "trial", t, "max diff", d.max(), "n diff", int((d > 0).sum()), flush=True)
