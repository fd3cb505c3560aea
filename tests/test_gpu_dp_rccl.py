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


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["sac_hopper", "ddpg_hcheetah"])
def test_rccl_exchange_overlap_changes_no_result(config):
    """The actor bucket's all-reduce runs on the exchange stream beside the ACM step's gradients
    (spprl.trainer._exchange, SPP_DP_OVERLAP=1); with SPP_DP_OVERLAP=0 (the default) the same operations run in the
    serial order.  The parameters after the run (a checksum of per-tensor sums) and the losses must be identical."""
    env = {"SPP_DP_FORCE": "1", "SPP_DIST_BACKEND": "nccl"}
    serial = _bench(config, dict(env, SPP_DP_OVERLAP="0"), launcher=True)
    over = _bench(config, dict(env, SPP_DP_OVERLAP="1"), launcher=True)
    assert over["param_checksum"] == serial["param_checksum"]
    assert over["losses"] == serial["losses"]


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["sac_hopper", "ppo_hcheetah"])
def test_bench_gpus_two_launches_two_ranks(config):
    """``bench.py --gpus 2`` with no external launcher starts one rank per GPU itself (torch.distributed.run
    as a child process) and relays rank 0's JSON line.  Rehearsed on one GPU with the gloo backend (both
    ranks share cuda:0): two ranks really run (n_gpus 2) and the data-parallel replicas stay bit-identical."""
    args = ["bench.py", "--config", config, "--gpus", "2", "--steps", "2", "--warmup", "1", "--envs", "512",
            "--no-cpu-baseline", "--no-pmc", "--no-rocprof"] + (["--buffer", "100000"] if config != "ppo_hcheetah"
                                                                 else [])
    env = dict(os.environ, SPP_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable] + args, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = lines[0]
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2"
    if config != "ppo_hcheetah":
        assert r["replicas_identical"] is True
