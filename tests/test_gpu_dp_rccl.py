"""RCCL data-parallel path rehearsed on one GPU.

bench.py's N > 1 path (torch.distributed "nccl" = RCCL process group, the gradient-bucket
all-reduce between the *Grads and *Apply halves of every update, the stepwise global obs
statistics with all-reduced moment sums and radix histograms, the max-over-ranks timing)
normally runs only on a multi-GPU node.  With SPP_DP_FORCE=1 the same code runs as a
one-rank RCCL job under torch.distributed.run, so it executes on a one-GPU box.  With one rank
every all-reduce is the identity (average over 1), so the losses must equal the plain N = 1
run's: gradient buckets bit-exact, obs statistics exact percentiles either way and fp64
moments (the stepwise and the sample-bracket methods sum in different orders), hence rtol 1e-5 (abs 2e-5: the bench prints losses to 5 decimals).
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(config, extra_env, launcher):
    args = ["bench.py", "--config", config, "--steps", "3", "--warmup", "1", "--envs", "1024",
            "--buffer", "200000", "--no-cpu-baseline", "--no-pmc"]
    if launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", "29561"] + args + ["--gpus", "1"]
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, **extra_env)
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["sac_hopper", "ddpg_hcheetah"])
def test_rccl_one_rank_exchange_matches_single_gpu(config):
    plain = _bench(config, {}, launcher=False)
    dp = _bench(config, {"SPP_DP_FORCE": "1", "SPP_DIST_BACKEND": "nccl"}, launcher=True)
    assert dp["n_gpus"] == 1 and plain["n_gpus"] == 1
    assert set(dp["losses"]) == set(plain["losses"])
    for k, v in plain["losses"].items():
        assert dp["losses"][k] == pytest.approx(v, rel=1e-5, abs=2e-5), k
