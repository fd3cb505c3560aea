#!/usr/bin/env python3
"""bench.py — env-steps/sec (rollout+update), SPP-SAC Hopper-v2, on N MI355X.

One "step" = one vector step of E lockstep envs per GPU through the whole
SPP-SAC loop, all on device (SURVEY.md §8d batched schedule):
  rollout   policy act (actor rsample + act_noise + clip + denorm + ACM)    ddpg_acm.py:40-50, off_policy.py:89-106
            synthetic fixed-shape env step (SURVEY Appendix A SynthEnv)     (MuJoCo is not in this image)
            replay writes: obs ring + timestep ring (Q6 rule)               replay_buffer.py:56-75,133-137,332-333
  update    B = rho*E uniform samples (rho = 100 = 100*50/50, train/spp_sac_hopper.py:19-22),
            one SAC_AcM grad step on them                                   sac_acm.py:89-162
  ACM       sigma*E samples (sigma = 10 = 100*100/1000, train/spp_sac_hopper.py:31-36),
            one AcMTrainer regression step                                  acm.py:246-258, 356-372
  stats     update_obs_mean_std over the live replay rows                   replay_buffer.py:83-96
FLOPs per env-step match the reference cadence (1 grad step of 100 samples per env step).
N > 1: one process per GPU (torchrun), each with E envs and a local 1e6-row replay
shard; gradient buckets are averaged with RCCL all-reduce at the update's two exchange
points (critic grads, actor grads) and at the ACM step; value = all ranks' env-steps / max time.
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

# Hopper SPP-SAC (train/spp_sac_hopper.py)
OB, AC = 11, 3
EP_LEN = 1000
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32 MFMA = f32 vector peak
PEAK_HBM_GBS = 8000.0

# algorithmic MACs per replayed sample, Hopper dims, H = 256
A_MAC = OB * 256 + 256 * 256 + 256 * 2 * OB            # actor forward
M_MAC = 2 * OB * 64 + 64 * 32 + 32 * AC                # ACM forward
C_MAC = (OB + AC) * 256 + 256 * 256 + 256              # critic forward
CRITIC_PHASE_MAC = A_MAC + M_MAC + 2 * C_MAC + 2 * C_MAC + 2 * (256 + 256 * 256)
ACTOR_PHASE_MAC = A_MAC + M_MAC + 2 * C_MAC + 2 * (256 + 256 * 256 + AC * 256) + (AC * 32 + 32 * 64 + 64 * OB) + (
    2 * OB * 256 + 256 * 256)
DW_MAC = 2 * C_MAC + A_MAC                               # weight gradients of both critics + actor
ACM_REG_MAC = M_MAC + M_MAC + (AC * 32 + 32 * 64)        # ACM fwd + dW + dX (regression step)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--rho", type=int, default=100)
    ap.add_argument("--sigma", type=int, default=10)
    ap.add_argument("--buffer", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(seconds):
    """The oracle (CPU restatement of SAC_AcM.update etc., torch 1 thread) run at the
    reference cadence: per env step one policy act, one grad step of B=100, 1/10 of an
    ACM batch step of 100, 1/1000 of an obs-stats pass over a 1e6-row buffer."""
    import oracle.nets as onets
    from oracle.acm import OracleAcmTrainer
    from oracle.nets import Norm
    from oracle.sac_acm import OracleSacAcm
    from tests.golden.weights import fill_params

    torch.set_num_threads(1)
    rng = np.random.RandomState(0)
    lay = {"actor": onets.sac_actor_layout(OB, OB), "critic_1": onets.critic_layout(OB + AC),
           "critic_2": onets.critic_layout(OB + AC), "critic_1_targ": onets.critic_layout(OB + AC),
           "critic_2_targ": onets.critic_layout(OB + AC), "acm": onets.acm_layout(2 * OB, AC)}
    params = {k: fill_params(v, i) for i, (k, v) in enumerate(lay.items())}
    norm = Norm(True, torch.full((OB,), -2.0), torch.full((OB,), 2.0))
    o = OracleSacAcm(OB, OB, AC, acm_critic=True, custom_loss=0.2, norm_closs=False, norm=norm,
                     acm_lim=np.ones(AC, np.float32), gamma=0.99, params=params)
    acm = OracleAcmTrainer(2 * OB, AC, lr=1e-3, params=params["acm"])
    B = 100
    P = {k: {n: torch.as_tensor(v) for n, v in params[k].items()} for k in ("actor", "acm")}

    def act(obs, eps):
        with torch.no_grad():
            a, _, _ = onets.sac_actor(P["actor"], obs, torch.tensor(1.0), eps)
            ad = norm.denormalize(a)
            return onets.acm(P["acm"], torch.cat([obs, ad], 1), torch.ones(AC))

    t_stats0 = time.perf_counter()
    big = rng.randn(1_000_000, OB)
    big.mean(0), big.std(0), np.percentile(big, 99, axis=0), np.percentile(big, 1, axis=0)
    t_stats = time.perf_counter() - t_stats0
    n = 0
    t_upd = t_act = t_acm = 0.0
    start = time.perf_counter()
    while time.perf_counter() - start < seconds:
        obs = torch.from_numpy(rng.randn(1, OB).astype(np.float32))
        t0 = time.perf_counter()
        act(obs, torch.from_numpy(rng.randn(1, OB).astype(np.float32)))
        t1 = time.perf_counter()
        batch = (rng.randn(B, OB).astype(np.float32), rng.randn(B, OB).astype(np.float32),
                 rng.randn(B, OB).astype(np.float32), rng.randn(B).astype(np.float32),
                 (rng.rand(B) < 0.01).astype(np.int8), rng.uniform(-1, 1, (B, AC)).astype(np.float32))
        o.update(*batch, rng.randn(B, OB).astype(np.float32), rng.randn(B, OB).astype(np.float32))
        t2 = time.perf_counter()
        if n % 10 == 0:
            acm.batch_update(rng.randn(B, 2 * OB).astype(np.float32), rng.uniform(-1, 1, (B, AC)).astype(np.float32))
        t3 = time.perf_counter()
        t_act += t1 - t0
        t_upd += t2 - t1
        t_acm += t3 - t2
        n += 1
    per_step = (t_act + t_upd + t_acm) / n + t_stats / 1000.0
    return {"value": round(1.0 / per_step, 2), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": "%d env steps of the SPP-SAC Hopper reference cadence (1 act + 1 grad step B=100 per env step, "
                      "ACM batch 100 every 10 steps, obs stats of a 1e6-row buffer amortised /1000); oracle = "
                      "torch-CPU restatement, 1 thread; %.1f s" % (n, time.perf_counter() - start)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import spprl
    from spprl import _lib
    from spprl._lib import call, ptr, stream_handle
    from spprl.dp import make_allreduce, shard_seed

    E, rho, sigma = args.envs, args.rho, args.sigma
    B, BA = rho * E, sigma * E
    ag = spprl.SAC_AcM(env_name="Hopper-v2", gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2,
                       acm_lr=1e-3, acm_critic=True, custom_loss=0.2, norm_closs=False, min_max_denormalize=True,
                       denormalize_actor_out=True, max_batch=max(B, BA), buffer_size=args.buffer, device=dev, seed=0)
    rb = ag.replay_buffer
    allreduce = make_allreduce()  # RCCL over xGMI; None at N=1

    g = torch.Generator(device="cpu").manual_seed(1234)  # SynthEnv dynamics: shared across ranks
    A = (torch.randn(OB, OB, generator=g) * 0.05).to(dev)
    seed = shard_seed(1000, rank)
    st = stream_handle()

    # ---- pre-fill the replay shard (min(capacity, 1e6) rows of N(0,1) obs)
    torch.manual_seed(seed)
    fill = min(args.buffer - 2 * E, 1_000_000 - 2 * E)
    chunk = 65536
    prev = rb.add_obs_batch(torch.randn(1, OB, device=dev))
    done_fill = 0
    while done_fill < fill:
        n = min(chunk, fill - done_fill)
        slots = rb.add_obs_batch(torch.randn(n, OB, device=dev))
        prevs = np.concatenate([prev[-1:], slots[:-1]])
        rb.add_timestep_batch(prevs, slots, torch.randn(n, OB, device=dev), torch.randn(n, device=dev),
                              torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros(n, dtype=torch.uint8,
                                                                                           device=dev),
                              torch.rand(n, AC, device=dev) * 2 - 1)
        prev = slots
        done_fill += n
    rb.update_obs_mean_std()

    # ---- rollout state
    obs = torch.randn(E, OB, device=dev)
    prev_slots = rb.add_obs_batch(obs)
    ep_t = 0
    eps = torch.empty(E, OB, device=dev)
    noise = torch.empty(E, OB, device=dev)
    nobs = torch.empty(E, OB, device=dev)
    rew = torch.empty(E, device=dev)
    zeros_u8 = torch.zeros(E, dtype=torch.uint8, device=dev)
    ones_u8 = torch.ones(E, dtype=torch.uint8, device=dev)
    idx = torch.empty(B, dtype=torch.int64, device=dev)
    idx_acm = torch.empty(BA, dtype=torch.int64, device=dev)
    xa = torch.empty(BA, 2 * OB, device=dev)
    ya = torch.empty(BA, AC, device=dev)
    acm_loss = torch.zeros(1, device=dev)
    counter = [0]

    def vector_step():
        nonlocal obs, prev_slots, ep_t, nobs
        c = counter[0]
        counter[0] += 1
        # rollout: noisy actor action -> ACM env action (mode 1), then the env
        call("sppRandNormal", ptr(eps), E * OB, seed, 4 * c, st)
        call("sppRandNormal", ptr(noise), E * OB, seed, 4 * c + 1, st)
        tgt, env_act = ag.act(obs, eps=eps, noise=noise, mode=1)
        call("sppSynthEnvStep", ptr(A), ptr(obs), ptr(env_act), E, OB, AC, ptr(nobs), ptr(rew), st)
        ep_t += 1
        end = ep_t >= EP_LEN
        flag = ones_u8 if end else zeros_u8  # Q3: SPP keeps time-limit done (max_ep_len None)
        slots = rb.add_obs_batch(nobs)
        rb.add_timestep_batch(prev_slots, slots, tgt, rew, flag, flag, env_act)
        obs, nobs = nobs, obs
        prev_slots = slots
        if end:
            obs = torch.randn(E, OB, device=dev)
            prev_slots = rb.add_obs_batch(obs)
            ep_t = 0
        n_live = len(rb)
        # update: one SAC_AcM grad step on rho*E uniform samples
        call("sppRandIndex", ptr(idx), B, n_live, seed, 4 * c + 2, st)
        ag.update_from_replay_dp(idx, seed, c, allreduce)
        # ACM regression on sigma*E samples
        call("sppRandIndex", ptr(idx_acm), BA, n_live, seed, 4 * c + 3, st)
        ag.acm_update_from_replay(idx_acm, xa, ya, acm_loss, allreduce)
        # obs statistics (replay_buffer.py:83-96)
        rb.update_obs_mean_std()

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

    env_steps = world * E * args.steps
    value = env_steps / elapsed
    k_ms = {name: ms[i] / max(cnt[i], 1) for i, name in enumerate(["critic_phase", "actor_phase", "dw_gemm",
                                                                      "adam", "acm_regress"])}
    crit_tf = 2.0 * CRITIC_PHASE_MAC * B / (k_ms["critic_phase"] * 1e-3) / 1e12
    act_tf = 2.0 * ACTOR_PHASE_MAC * B / (k_ms["actor_phase"] * 1e-3) / 1e12
    dw_tf = 2.0 * DW_MAC * B / 2 / (k_ms["dw_gemm"] * 1e-3) / 1e12  # two dW launches per step
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("critic_phase_bytes_per_launch")
        except Exception:
            traffic = None
    flop_step = 2.0 * ((CRITIC_PHASE_MAC + ACTOR_PHASE_MAC + DW_MAC) * B + ACM_REG_MAC * BA + (A_MAC + M_MAC) * E)
    result = {
        "metric": "env-steps/sec (rollout+update) SPP-SAC Hopper-v2",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: SynthEnv linear-tanh dynamics (Hopper shapes ob=11, ac=3), random-init networks",
        "config": {"workload": "SPP-SAC Hopper-v2, %d vectorized envs per GPU, fp32 (BASELINE.json configs[1])" % E,
                   "envs_per_gpu": E, "update_batch": B, "acm_batch": BA, "rho": rho, "sigma": sigma,
                   "replay_rows_per_gpu": args.buffer, "parallelism": "dp%d" % world},
        "roofline": {"bound": "mfma", "kernel": "k_sac_critic_phase (critic targets + both critics fwd/bwd)",
                     "achieved": round(crit_tf, 2), "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(crit_tf / PEAK_FP32_MFMA_TFLOPS, 4), "traffic": traffic,
                     "flop_per_launch": 2.0 * CRITIC_PHASE_MAC * B, "avg_launch_ms": round(k_ms["critic_phase"], 3)},
        "kernels_ms_per_launch": {k: round(v, 3) for k, v in k_ms.items()},
        "kernels_tflops": {"critic_phase": round(crit_tf, 2), "actor_phase": round(act_tf, 2),
                           "dw_gemm": round(dw_tf, 2)},
        "step_tflops": round(flop_step * args.steps / elapsed / 1e12, 2),
        "losses": {k: round(v, 5) for k, v in losses.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
