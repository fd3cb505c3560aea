#!/usr/bin/env python3
"""bench.py — env-steps/sec (rollout+update) of the SPP off-policy loop on N MI355X.

One "step" = one vector step of E lockstep envs per GPU through the product training
loop (spprl.trainer.OffPolicyLoop, fused schedule), all on device:
  rollout   policy act (actor sample + act_noise + clip + denorm + ACM)     ddpg_acm.py:40-50, off_policy.py:89-106
            synthetic fixed-shape env step (SURVEY Appendix A SynthEnv)      (MuJoCo is not in this image)
            replay writes: obs ring + timestep ring (Q6 rule)                replay_buffer.py:56-75,133-137,332-333
  update    B = rho*E uniform samples, one grad step on them                 sac_acm.py:89-162 / ddpg_acm.py:147-201
            rho = update_batch_size*grad_steps/update_freq = 100 (train/spp_*.py)
  ACM       sigma*E samples, one AcMTrainer regression step                  acm.py:246-258, 356-372
            sigma = acm_update_batches*acm_batch_size/acm_update_freq (10 SAC, 51.2 DDPG)
  stats     update_obs_mean_std over the live replay rows                    replay_buffer.py:83-96
FLOPs per env-step equal the reference cadence (one grad step of 100 samples per env step).

--config sac_hopper (default; BASELINE.json configs[1]: SPP-SAC Hopper-v2, 4096 envs, fp32)
         ddpg_hcheetah (configs[2]: SPP-DDPG HalfCheetah-v2, 8192 envs, 10M-transition HBM replay)
         sac_ant (configs[4] per-GPU shape: SPP-SAC Ant, 32768 envs / 8 GPUs = 4096 per GPU, fp32 MLP)
N > 1: one process per GPU (torchrun), each with E envs and a local replay shard; gradient
buckets are averaged with RCCL all-reduce at the update's exchange points (critic grads,
actor grads, ACM grads); value = all ranks' env-steps / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "spp-rl_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA peak
PEAK_BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA peak (no sparsity)
PEAK_HBM_GBS = 8000.0

CONFIGS = {
    "sac_hopper": dict(
        algo="sac", env="Hopper-v2", ob=11, ac=3, envs=4096, buffer=1_000_000, baseline_idx=1,
        workload="SPP-SAC Hopper-v2, %d vectorized envs per GPU, fp32 (BASELINE.json configs[1])",
        agent=dict(gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2, acm_lr=1e-3, acm_critic=True,
                   custom_loss=0.2, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                   update_batch_size=100, update_freq=50, grad_steps=50, acm_update_freq=1000,
                   acm_update_batches=100, acm_batch_size=100)),
    "ddpg_hcheetah": dict(
        algo="ddpg", env="HalfCheetah-v2", ob=17, ac=6, envs=8192, buffer=10_000_000, baseline_idx=2,
        workload="SPP-DDPG HalfCheetah-v2, %d vectorized envs per GPU, 10M-transition HBM replay, fp32 "
                 "(BASELINE.json configs[2])",
        agent=dict(gamma=0.95, actor_lr=5e-4, critic_lr=5e-4, acm_lr=0.005, act_noise=0.05, acm_critic=True,
                   custom_loss=1.0, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                   update_batch_size=100, update_freq=50, grad_steps=50, acm_update_freq=500,
                   acm_update_batches=200, acm_batch_size=128)),
    "sac_ant_bf16": dict(
        algo="sac", env="Ant-v2", ob=111, ac=8, envs=4096, buffer=1_000_000, baseline_idx=4, bf16=True,
        workload="SPP-SAC Ant (111-dim obs), %d vectorized envs per GPU, bf16 MFMA MLP + fp32 targets "
                 "(BASELINE.json configs[4] per-GPU shape)",
        agent=dict(gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2, acm_lr=1e-3, acm_critic=True,
                   custom_loss=0.2, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                   update_batch_size=100, update_freq=50, grad_steps=50, acm_update_freq=1000,
                   acm_update_batches=100, acm_batch_size=100, mlp_bf16=True)),
    "sac_ant": dict(
        algo="sac", env="Ant-v2", ob=111, ac=8, envs=4096, buffer=1_000_000, baseline_idx=4,
        workload="SPP-SAC Ant (111-dim obs), %d vectorized envs per GPU, fp32 MLP (BASELINE.json configs[4] "
                 "per-GPU shape)",
        agent=dict(gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2, acm_lr=1e-3, acm_critic=True,
                   custom_loss=0.2, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                   update_batch_size=100, update_freq=50, grad_steps=50, acm_update_freq=1000,
                   acm_update_batches=100, acm_batch_size=100)),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="sac_hopper", choices=sorted(CONFIGS) + ["ppo_hcheetah"])
    ap.add_argument("--envs", type=int, default=None)
    ap.add_argument("--buffer", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=min(8, os.cpu_count() or 1),
                    help="concurrent 1-thread oracle processes for the CPU baseline (reference N_CORES)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(cfg, seconds):
    """The oracle (CPU restatement of the reference update path, torch 1 thread) run at
    the reference cadence: per env step one policy act and one grad step of B=100; the
    ACM regression at its reference rate (sigma/100 batches of 100 per env step); one
    obs-stats pass over a 1e6-row buffer amortised over an iteration of 1000 frames."""
    import oracle.nets as onets
    from oracle.nets import Norm
    from tests.golden.weights import fill_params

    torch.set_num_threads(1)
    rng = np.random.RandomState(0)
    ob, ac = cfg["ob"], cfg["ac"]
    sac = cfg["algo"] == "sac"
    norm = Norm(True, torch.full((ob,), -2.0), torch.full((ob,), 2.0))
    if sac:
        from oracle.acm import OracleAcmTrainer
        from oracle.sac_acm import OracleSacAcm

        lay = {"actor": onets.sac_actor_layout(ob, ob), "critic_1": onets.critic_layout(ob + ac),
               "critic_2": onets.critic_layout(ob + ac), "critic_1_targ": onets.critic_layout(ob + ac),
               "critic_2_targ": onets.critic_layout(ob + ac), "acm": onets.acm_layout(2 * ob, ac)}
        params = {k: fill_params(v, i) for i, (k, v) in enumerate(lay.items())}
        o = OracleSacAcm(ob, ob, ac, acm_critic=True, custom_loss=0.2, norm_closs=False, norm=norm,
                         acm_lim=np.ones(ac, np.float32), gamma=0.99, params=params)
        acm = OracleAcmTrainer(2 * ob, ac, lr=1e-3, params=params["acm"])
        P = {k: {n: torch.as_tensor(v) for n, v in params[k].items()} for k in ("actor", "acm")}

        def act(obs):
            with torch.no_grad():
                a, _, _ = onets.sac_actor(P["actor"], obs, torch.tensor(1.0), torch.randn(1, ob))
                return onets.acm(P["acm"], torch.cat([obs, norm.denormalize(a)], 1), torch.ones(ac))

        def upd(batch):
            o.update(*batch, rng.randn(100, ob).astype(np.float32), rng.randn(100, ob).astype(np.float32))

        acm_step = acm.batch_update
        acm_every = 100.0 / (cfg["agent"]["acm_update_batches"] * cfg["agent"]["acm_batch_size"] /
                             cfg["agent"]["acm_update_freq"])
    else:
        from oracle.ddpg_acm import OracleDdpgAcm

        lay = {"actor": onets.ddpg_actor_layout(ob, ob), "critic": onets.critic_layout(ob + ac),
               "actor_targ": onets.ddpg_actor_layout(ob, ob), "critic_targ": onets.critic_layout(ob + ac),
               "acm": onets.basic_acm_layout(2 * ob, ac)}
        params = {k: fill_params(v, i) for i, (k, v) in enumerate(lay.items())}
        o = OracleDdpgAcm(ob, ob, ac, acm_critic=True, custom_loss=1.0, norm_closs=False, norm=norm, gamma=0.95,
                          params=params)
        Pa = {n: torch.as_tensor(v) for n, v in params["actor"].items()}
        Pm = {n: torch.as_tensor(v).clone().requires_grad_(True) for n, v in params["acm"].items()}
        opt = torch.optim.Adam(Pm.values(), lr=0.005)

        def act(obs):
            with torch.no_grad():
                a = onets.ddpg_actor(Pa, obs, torch.tensor(1.0)) + 0.05 * torch.randn(1, ob)
                return onets.basic_acm(Pm, torch.cat([obs, norm.denormalize(a.clamp(-1.1, 1.1))], 1))

        def upd(batch):
            o.update(*batch)

        def acm_step(x, y):
            loss = torch.nn.functional.mse_loss(onets.basic_acm(Pm, torch.as_tensor(x)), torch.as_tensor(y))
            opt.zero_grad()
            loss.backward()
            opt.step()

        acm_every = 128.0 / (cfg["agent"]["acm_update_batches"] * cfg["agent"]["acm_batch_size"] /
                             cfg["agent"]["acm_update_freq"])

    t_stats0 = time.perf_counter()
    big = rng.randn(1_000_000, ob)
    big.mean(0), big.std(0), np.percentile(big, 99, axis=0), np.percentile(big, 1, axis=0)
    t_stats = time.perf_counter() - t_stats0
    n, acc, t_loop = 0, 0.0, 0.0
    B = 100
    start = time.perf_counter()
    while time.perf_counter() - start < seconds:
        obs = torch.from_numpy(rng.randn(1, ob).astype(np.float32))
        batch = (rng.randn(B, ob).astype(np.float32), rng.randn(B, ob).astype(np.float32),
                 rng.randn(B, ob).astype(np.float32), rng.randn(B).astype(np.float32),
                 (rng.rand(B) < 0.01).astype(np.int8), rng.uniform(-1, 1, (B, ac)).astype(np.float32))
        xa = rng.randn(100 if sac else 128, 2 * ob).astype(np.float32)
        ya = rng.uniform(-1, 1, (xa.shape[0], ac)).astype(np.float32)
        t0 = time.perf_counter()
        act(obs)
        upd(batch)
        acc += 1.0
        while acc >= acm_every:
            acm_step(xa, ya)
            acc -= acm_every
        t_loop += time.perf_counter() - t0
        n += 1
    per_step = t_loop / n + t_stats / 1000.0
    return {"value": round(1.0 / per_step, 2), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": "%d env steps of the %s reference cadence (1 act + 1 grad step B=100 per env step, ACM "
                      "regression at its reference rate, obs stats of a 1e6-row buffer amortised /1000); oracle = "
                      "torch-CPU restatement, 1 thread; %.1f s" % (n, cfg["env"], time.perf_counter() - start)}


def bench_ppo(args, world, rank, dev):
    """configs[3]: SPP-PPO HalfCheetah-v2, 16384 envs over 8 GPUs = 2048 per GPU (train/spp_ppo_hcheetah.py
    hyper-parameters).  One step = one PPO_AcM iteration: T = 16 vector steps of rollout (actor sample,
    AcM, env, ACM ring writes), 10 x 10 full-batch critic steps, GAE over [T][E], <= 10 clip-loss epochs of
    512-sample minibatches with the KL stop, the ACM regression (5 epochs of 64-sample batches over the
    1.1e5 ring every 3 iterations), ring obs statistics."""
    import spprl
    from spprl.dp import shard_seed

    E = args.envs or 2048
    T = 16
    seed = shard_seed(1000, rank)
    ag = spprl.PPO_AcM(env_name="HalfCheetah-v2", gamma=0.99, actor_lr=3e-4, critic_lr=3e-4, batch_size=T * E,
                       ppo_batch_size=512, kl_div_threshold=0.1, max_ppo_epochs=10, entropy_coef=0.0,
                       custom_loss=0.1, norm_closs=True, min_max_denormalize=True, denormalize_actor_out=True,
                       acm_epochs=5, acm_batch_size=64, acm_update_freq=3, acm_lr=3e-4,
                       acm_pre_train_samples=100_000, n_envs=E, device=dev, seed=0, loop_seed=seed)
    rb = ag.replay_buffer
    ob, ac = ag.ob_dim, ag.ac_dim
    torch.manual_seed(seed)
    fill = rb.size - 2 * E  # the ACM ring after pre-training (random env actions)
    prev = rb.add_obs_batch(torch.randn(1, ob, device=dev))
    slots = rb.add_obs_batch(torch.randn(fill, ob, device=dev))
    prevs = np.concatenate([prev[-1:], slots[:-1]])
    z = torch.zeros(fill, dtype=torch.uint8, device=dev)
    rb.add_timestep_batch(prevs, slots, torch.randn(fill, ob, device=dev), torch.randn(fill, device=dev), z, z,
                          torch.rand(fill, ac, device=dev) * 2 - 1)
    ag.acm.update_obs_stats()
    ag.iteration = 1

    def iteration():
        ag.perform_iteration(sync=False)
        ag.iteration += 1  # ACM update every acm_update_freq iterations (on_policy.py:66-70)

    for _ in range(args.warmup):
        iteration()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        iteration()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    elapsed = float(tmax.item())
    value = world * T * E * args.steps / elapsed
    res = {"metric": "env-steps/sec (rollout+update) SPP-PPO HalfCheetah-v2", "value": round(value, 1),
           "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic: SynthEnv linear-tanh dynamics (HalfCheetah-v2 shapes ob=17, ac=6), random-init "
                   "networks, ACM ring pre-filled with N(0,1) transitions",
           "config": {"workload": "SPP-PPO HalfCheetah-v2, %d vectorized envs per GPU x %d steps per iteration "
                                  "(BASELINE.json configs[3] per-GPU shape)" % (E, T), "envs_per_gpu": E,
                      "steps_per_iteration": T, "acm_ring": rb.size, "parallelism": "dp%d" % world},
           "losses": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in ag.loss.items()}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _cpu_worker(args):
    name, seconds = args
    return cpu_baseline(CONFIGS[name], seconds)


def cpu_baseline_pool(name, seconds, procs):
    """The reference's N_CORES layout (train/spp_*.py: a multiprocessing pool of independent
    1-thread runs, evals.py:22-26): `procs` concurrent oracle runs on the host cores; the
    aggregate is the sum of the per-process env-steps/s."""
    import multiprocessing as mp

    if procs <= 1:
        return cpu_baseline(CONFIGS[name], seconds)
    # the workers are CPU-only: hide the GPUs from them (a process that loads the HIP runtime
    # may count as a GPU user; the box allows 16 per job)
    saved = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    for k in saved:
        os.environ[k] = "-1"
    try:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker, [(name, seconds)] * procs)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    vals = [r["value"] for r in res]
    out = dict(res[0])
    out.update(value=round(sum(vals), 2), cores=procs, per_core=round(sum(vals) / procs, 2),
               sample="%d concurrent 1-thread processes, each: %s" % (procs, res[0]["sample"]))
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SPP_DIST_BACKEND=gloo (testing only): ranks may share one GPU; the default is RCCL ("nccl")
    backend = os.environ.get("SPP_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.config == "ppo_hcheetah":
        return bench_ppo(args, world, rank, dev)
    import spprl
    from spprl import flops
    from spprl.dp import shard_seed

    cfg = CONFIGS[args.config]
    ob, ac = cfg["ob"], cfg["ac"]
    E = args.envs or cfg["envs"]
    cap = args.buffer or cfg["buffer"]
    a = cfg["agent"]
    rho = a["update_batch_size"] * a["grad_steps"] / a["update_freq"]
    sigma = a["acm_update_batches"] * a["acm_batch_size"] / a["acm_update_freq"]
    B, BA = int(round(rho * E)), int(round(sigma * E))
    seed = shard_seed(1000, rank)
    Agent = spprl.SAC_AcM if cfg["algo"] == "sac" else spprl.DDPG_AcM
    ag = Agent(env_name=cfg["env"], buffer_size=cap, max_batch=max(B, BA), device=dev, seed=0, n_envs=E,
               schedule="fused", random_frames=0, batch_size=E, iterations=10 ** 9, loop_seed=seed,
               acm_epochs=1, **a)
    rb = ag.replay_buffer
    assert ag.fused_batch_sizes() == (B, BA)

    # ---- pre-fill the replay shard with N(0,1) transitions
    torch.manual_seed(seed)
    fill = cap - 2 * E
    chunk = 1 << 18
    prev = rb.add_obs_batch(torch.randn(1, ob, device=dev))
    done_fill = 0
    while done_fill < fill:
        n = min(chunk, fill - done_fill)
        slots = rb.add_obs_batch(torch.randn(n, ob, device=dev))
        prevs = np.concatenate([prev[-1:], slots[:-1]])
        z = torch.zeros(n, dtype=torch.uint8, device=dev)
        rb.add_timestep_batch(prevs, slots, torch.randn(n, ob, device=dev), torch.randn(n, device=dev), z, z,
                              torch.rand(n, ac, device=dev) * 2 - 1)
        prev = slots
        done_fill += n
    ag.update_obs_stats()
    ag.iteration = 1  # past the first iteration: ACM regression is on (ddpg_acm.py:52-57)
    ag.stats_logger.frames = fill

    def vector_step():
        ag.collect_batch_and_train(E)  # act -> env -> replay -> rho*E grad step -> sigma*E ACM step
        ag.update_obs_stats()  # global across ranks (RCCL) when N > 1

    for _ in range(args.warmup):
        vector_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ag.set_timing(True)
    ag.get_timing()  # clear
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        vector_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms, cnt = ag.get_timing()
    ag.set_timing(False)
    losses = ag.loss
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    elapsed = float(tmax.item())

    mac = flops.sac_macs(ob, ac) if cfg["algo"] == "sac" else flops.ddpg_macs(ob, ac)
    value = world * E * args.steps / elapsed
    k_ms = {name: ms[i] / max(cnt[i], 1) for i, name in enumerate(["critic_phase", "actor_phase", "dw_gemm",
                                                                      "adam", "acm_regress"])}
    tf = lambda m, t: 2.0 * m * B / (t * 1e-3) / 1e12  # noqa: E731
    crit_tf, act_tf = tf(mac["critic_phase"], k_ms["critic_phase"]), tf(mac["actor_phase"], k_ms["actor_phase"])
    dw_tf = tf(mac["dw"] / 2, k_ms["dw_gemm"])  # two dW launches per grad step
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            key = "critic_phase_bytes_per_launch" if cfg["algo"] == "sac" else "ddpg_critic_phase_bytes_per_launch"
            t = json.load(open(pmc))
            if t.get("config", "sac_hopper") == args.config:
                traffic = t.get(key)
        except Exception:
            traffic = None
    flop_step = 2.0 * (mac["update"] * B + mac["acm_reg"] * BA + mac["act"] * E)
    bf16 = cfg.get("bf16", False)
    peak = PEAK_BF16_MFMA_TFLOPS if bf16 else PEAK_FP32_MFMA_TFLOPS
    kname = "k_sac_critic_phase" if cfg["algo"] == "sac" else "k_ddpg_critic_phase"
    result = {
        "metric": "env-steps/sec (rollout+update) %s" % ("SPP-SAC " + cfg["env"] if cfg["algo"] == "sac"
                                                         else "SPP-DDPG " + cfg["env"]),
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 MFMA MLP, fp32 accumulate / targets / optimizer" if bf16 else "fp32",
        "data": "synthetic: SynthEnv linear-tanh dynamics (%s shapes ob=%d, ac=%d), random-init networks, replay "
                "pre-filled with N(0,1) transitions" % (cfg["env"], ob, ac),
        "config": {"workload": cfg["workload"] % E, "envs_per_gpu": E, "update_batch": B, "acm_batch": BA,
                   "rho": rho, "sigma": sigma, "replay_rows_per_gpu": cap, "parallelism": "dp%d" % world},
        "roofline": {"bound": "mfma", "kernel": "%s (critic targets + critic fwd/bwd)" % kname,
                     "achieved": round(crit_tf, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(crit_tf / peak, 4), "traffic": traffic,
                     "flop_per_launch": 2.0 * mac["critic_phase"] * B, "avg_launch_ms": round(k_ms["critic_phase"], 3)},
        "kernels_ms_per_launch": {k: round(v, 3) for k, v in k_ms.items()},
        "kernels_tflops": {"critic_phase": round(crit_tf, 2), "actor_phase": round(act_tf, 2),
                           "dw_gemm": round(dw_tf, 2)},
        "step_tflops": round(flop_step * args.steps / elapsed / 1e12, 2),
        "losses": {k: round(v, 5) for k, v in losses.items()},
    }
    if world > 1:  # data-parallel replicas must stay bit-identical (same averaged grads, same Adam)
        chk = torch.stack([p.double().sum() for p in ag.params.values()] +
                          [p.double().abs().sum() for p in ag.params.values()])
        allc = [torch.empty_like(chk) for _ in range(world)]
        dist.all_gather(allc, chk)
        result["replicas_identical"] = bool(all(torch.equal(allc[0], c) for c in allc))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_pool(args.config, args.cpu_seconds, args.cpu_procs)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
