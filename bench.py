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
  stats     update_obs_mean_std over the live replay rows at the reference's rate: one pass per
            batch_size = 1000 frames (ddpg.py:159-170), i.e. floor(frames / 1000) passes so far
FLOPs per env-step equal the reference cadence (one grad step of 100 samples per env step).

--config sac_hopper (default; BASELINE.json configs[1]: SPP-SAC Hopper-v2, 4096 envs, fp32)
         ddpg_hcheetah (configs[2]: SPP-DDPG HalfCheetah-v2, 8192 envs, 10M-transition HBM replay)
         sac_ant / sac_ant_bf16 (configs[4] per-GPU shape: 32768 envs / 8 GPUs = 4096, fp32 / bf16 MLP)
         ppo_hcheetah (configs[3] per-GPU shape: 16384 envs / 8 GPUs = 2048, one PPO_AcM iteration per step)
         vanilla_sac_hcheetah (configs[0]: vanilla SAC, 1 env, the reference cadence frame by frame;
                               one step = one frame)
N > 1: one process per GPU (torchrun; `bench.py --gpus N` started without one launches it as a child
process and relays rank 0's JSON line), each with E envs and a local replay shard; gradient
buckets are averaged with RCCL all-reduce at the update's exchange points (critic grads,
actor grads, ACM grads); value = all ranks' env-steps / max-over-ranks time.

Roofline: the dominant kernel's algorithmic FLOPs per launch / its average HIP-event launch
time inside the timed region.  traffic: HBM bytes per launch of that kernel from two
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short child run of this same
script, config, E and library (N = 1 only; null when rocprofv3 is absent or --no-pmc).
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "spp-rl_amd"))
sys.path.insert(0, REPO)

# HIP hardware queues per process (read once, when the runtime initialises: before torch touches the GPU).  The
# PPO_AcM iteration runs its ACM epochs on a second stream beside the update; with a process group's RCCL
# streams there are more streams than HIP's default 4 queues, and the runtime then maps the update's stream and
# the ACM's onto one queue, serialising them (DP-forced PPO 452 K vs 496 K env-steps/s at 4 queues, equal to the
# plain line at 8: profiles/r05/ab_acm_wv.txt).  8 <= the pool's limit of 32.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense fp32 MFMA peak
PEAK_BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA peak (no sparsity)
PEAK_HBM_GBS = 8000.0
LIB = os.path.join(REPO, "spp-rl_amd", "spprl", "libspprl.so")

SAC_AGENT = dict(gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2, acm_lr=1e-3, acm_critic=True,
                 custom_loss=0.2, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                 update_batch_size=100, update_freq=50, grad_steps=50, acm_update_freq=1000,
                 acm_update_batches=100, acm_batch_size=100, batch_size=1000)
CONFIGS = {
    "sac_hopper": dict(
        algo="sac", env="Hopper-v2", ob=11, ac=3, envs=4096, buffer=1_000_000, baseline_idx=1,
        workload="SPP-SAC Hopper-v2, %d vectorized envs per GPU, fp32 (BASELINE.json configs[1])", agent=SAC_AGENT),
    "ddpg_hcheetah": dict(
        algo="ddpg", env="HalfCheetah-v2", ob=17, ac=6, envs=8192, buffer=10_000_000, baseline_idx=2,
        workload="SPP-DDPG HalfCheetah-v2, %d vectorized envs per GPU, 10M-transition HBM replay, fp32 "
                 "(BASELINE.json configs[2])",
        agent=dict(gamma=0.95, actor_lr=5e-4, critic_lr=5e-4, acm_lr=0.005, act_noise=0.05, acm_critic=True,
                   custom_loss=1.0, norm_closs=False, min_max_denormalize=True, denormalize_actor_out=True,
                   update_batch_size=100, update_freq=50, grad_steps=50, acm_update_freq=500,
                   acm_update_batches=200, acm_batch_size=128, batch_size=1000)),
    "sac_ant_bf16": dict(
        algo="sac", env="Ant-v2", ob=111, ac=8, envs=4096, buffer=1_000_000, baseline_idx=4, bf16=True,
        workload="SPP-SAC Ant (111-dim obs), %d vectorized envs per GPU, bf16 MFMA MLP + fp32 targets "
                 "(BASELINE.json configs[4] per-GPU shape)", agent=dict(SAC_AGENT, mlp_bf16=True)),
    "sac_ant": dict(
        algo="sac", env="Ant-v2", ob=111, ac=8, envs=4096, buffer=1_000_000, baseline_idx=4,
        workload="SPP-SAC Ant (111-dim obs), %d vectorized envs per GPU, fp32 MLP (BASELINE.json configs[4] "
                 "per-GPU shape)", agent=SAC_AGENT),
    "vanilla_sac_hcheetah": dict(
        algo="vanilla", env="HalfCheetah-v2", ob=17, ac=6, envs=1, buffer=1_000_000, baseline_idx=0,
        workload="vanilla SAC HalfCheetah-v2, 1 env, reference cadence (B=100, 50 grad steps every 50 frames) "
                 "(BASELINE.json configs[0], train/vanilla_sac_hcheetah.py)",
        agent=dict(gamma=0.99, actor_lr=1e-3, critic_lr=1e-3, alpha_lr=1e-3, alpha=0.2, update_batch_size=100,
                   update_freq=50, grad_steps=50, batch_size=1000)),
}
DEFAULT_STEPS = {"vanilla_sac_hcheetah": (2000, 100), "ppo_hcheetah": (30, 3)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 200; vanilla: 2000 frames)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 10)")
    ap.add_argument("--config", default="sac_hopper", choices=sorted(CONFIGS) + ["ppo_hcheetah"])
    ap.add_argument("--envs", type=int, default=None)
    ap.add_argument("--buffer", type=int, default=None)
    ap.add_argument("--stats-rate", choices=["reference", "per-step"], default="reference",
                    help="obs-stats passes: one per 1000 frames (reference) or one per vector step")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=None,
                    help="concurrent 1-thread reference-loop processes (default: the host's CPU share, max 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc child passes (traffic null)")
    ap.add_argument("--no-rocprof", action="store_true",
                    help="skip the rocprofv3 --kernel-trace child run (roofline.frac_rocprof null)")
    ap.add_argument("--trace-dir", default=os.path.join(REPO, "gpurun_out"),
                    help="where the rocprof child run's steady-state kernel summary is written")
    ap.add_argument("--dp-comm", choices=["native", "torch"], default="native",
                    help="N > 1 exchange: libspprl's own RCCL communicator on the compute stream (gradient buckets, "
                         "obs-statistics collectives) or torch.distributed's (its own stream + event waits)")
    ap.add_argument("--rehearse-world", type=int, default=None,
                    help="ppo_hcheetah on one GPU: the per-rank work of a W-rank job (ACM cadence scaled for W ranks, "
                         "update on a W-rank union's shape); value = W x this rank's env-steps/s (projection)")
    ap.add_argument("--ppo-minibatch", type=int, default=None,
                    help="ppo_hcheetah: the clip-loss minibatch (default 512 x s, the cadence rule of every sample "
                         "count; 512 = the reference's absolute minibatch, round 5's line)")
    ap.add_argument("--ppo-dp", choices=["shard", "union"], default="shard",
                    help="ppo_hcheetah data parallel update: each rank on its own rollout with one gradient all-reduce "
                         "per critic / actor step (shard), or one all-gather of the rollouts and the whole update on "
                         "the union on every rank (union, round 5)")
    ap.add_argument("--acm-passes", type=int, default=None,
                    help="ppo_hcheetah: 64-row passes per workgroup and step of the persistent ACM SGD "
                         "(sppSetAcmSgdPasses; default: the library's)")
    ap.add_argument("--replicas", type=int, default=1,
                    help="vanilla_sac_hcheetah: R independent single-env runs (separate processes, seeds i) sharing "
                         "the GPU, timed together -- the layout of the reference's own configs[0] script (a pool of "
                         "independent runs) and of this line's cpu_baseline; value = R x steps / the slowest "
                         "replica's timed span")
    ap.add_argument("--replica-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--host-env", action="store_true",
                    help="step the envs on the host CPU (HostSynthEnv: vectorised numpy SynthEnv behind pinned "
                         "staging + side-stream copies, the update overlapping the host step): the PCIe-inclusive "
                         "host-simulator rate, not the metric")
    a = ap.parse_args()
    st, wu = DEFAULT_STEPS.get(a.config, (200, 10))
    a.steps = st if a.steps is None else a.steps
    a.warmup = wu if a.warmup is None else a.warmup
    return a


# ------------------------------------------------------------------ CPU baseline (the reference's N_CORES path)
def _cpu_worker(args):
    name, seconds = args
    return cpu_baseline(name, seconds)


def cpu_baseline(name, seconds):
    """One 1-thread process of the reference's CPU training loop (oracle/cpu_loop.py: the
    per-frame DDPG.collect_batch_and_train loop with act, env step, fp64 replay ring,
    sample_batch, the update, the ACM batches and the per-iteration obs statistics)."""
    from oracle.cpu_loop import CpuLoop

    torch.set_num_threads(1)
    cfg = CONFIGS[name]
    a = cfg["agent"]
    algo = {"sac": "sac_acm", "ddpg": "ddpg_acm", "vanilla": "sac"}[cfg["algo"]]
    L = CpuLoop(algo, cfg["ob"], cfg["ac"], update_batch_size=a["update_batch_size"], update_freq=a["update_freq"],
                grad_steps=a["grad_steps"], acm_update_freq=a.get("acm_update_freq", 1),
                acm_update_batches=a.get("acm_update_batches", 0), acm_batch_size=a.get("acm_batch_size", 100),
                batch_size=10 ** 12, buffer_size=1_000_000, prefill=990_000)
    t0 = time.perf_counter()
    L._obs_stats()  # one update_obs_mean_std over the 990K-row buffer, amortised over batch_size frames
    t_stats = time.perf_counter() - t0
    fps, n, el = L.run(seconds)
    per = 1.0 / fps + t_stats / a["batch_size"]
    return {"value": round(1.0 / per, 2), "frames": n, "seconds": round(el, 2), "stats_s": round(t_stats, 3)}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_report(name, seconds, procs):
    """The reference's N_CORES layout (train/spp_*.py: a multiprocessing pool of independent
    1-thread runs, evals.py:22-26), on the GPU box's host cores, plus a 1-core run alone."""
    import multiprocessing as mp

    one = cpu_baseline(name, seconds)
    # the workers are CPU-only: hide the GPUs from them (the box counts GPU-using processes)
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
    ref_per_core = {"sac": 103.4, "vanilla": 113.3}.get(CONFIGS[name]["algo"])
    out = {"value": round(sum(vals), 2), "unit": "env-steps/s", "cores": procs, "kind": "port",
           "per_core": round(sum(vals) / procs, 2), "one_core": one["value"], "cpu_model": _cpu_model(),
           "cores_note": "the box's CPU share is 16 and at most 16 processes may hold the GPU runtime (this "
                         "process included), so the pool is 15 single-thread workers",
           "sample": "%d concurrent 1-thread processes of the reference's per-frame training loop restated on the "
                     "CPU (oracle/cpu_loop.py: act, SynthEnv step, fp64 replay ring, sample_batch, B=100 grad steps "
                     "at the reference cadence, ACM batches, obs stats of a 990K-row buffer per 1000 frames), "
                     "%.0f s each (%d frames per process); one_core = the same loop alone"
                     % (procs, seconds, res[0]["frames"])}
    if ref_per_core:
        out["reference_per_core_measured_in_survey"] = ref_per_core
        out["port_vs_reference_per_core"] = round(one["value"] / ref_per_core, 3)
        out["calibration"] = (
            "port_vs_reference_per_core divides this host's port rate by the reference's rate measured on the build "
            "container's CPU (SURVEY Appendix B): two different CPUs.  Same host, same moment "
            "(tools/cpu_calibrate.py, profiles/r05/cpu_calibrate.txt): the reference's SAC_AcM.update (B = 100, one "
            "thread) takes 1.03-1.08x the port's over two runs (12.96 vs 12.55 ms, 8.77 vs 8.11 ms) since the port "
            "steps the reference's own optimizer class, torch.optim.Adam; with round 4's restated Adam the port's "
            "update was 1.31-1.38x faster, and the rest of round 4's 2.27x is the faster host CPU")
    return out


def _ppo_cpu_worker(_):
    """One 1-thread process of the reference's PPO_AcM iteration restated (oracle/cpu_loop_ppo.py), over
    one ACM update cycle (acm_update_freq = 3 iterations of 2000 frames)."""
    from oracle.cpu_loop_ppo import PpoCpuLoop

    torch.set_num_threads(1)
    fps, n, el = PpoCpuLoop().run()
    return {"value": round(fps, 2), "frames": n, "seconds": round(el, 2)}


def ppo_cpu_baseline_report(procs):
    """train/spp_ppo_hcheetah.py's layout: a multiprocessing pool of independent 1-thread runs."""
    import multiprocessing as mp

    one = _ppo_cpu_worker(0)
    saved = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")}
    for k in saved:
        os.environ[k] = "-1"
    try:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_ppo_cpu_worker, range(procs))
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    vals = [r["value"] for r in res]
    return {"value": round(sum(vals), 2), "unit": "env-steps/s", "cores": procs, "kind": "port",
            "per_core": round(sum(vals) / procs, 2), "one_core": one["value"], "cpu_model": _cpu_model(),
            "cores_note": "the box's CPU share is 16 and at most 16 processes may hold the GPU runtime (this "
                          "process included), so the pool is 15 single-thread workers",
            "sample": "%d concurrent 1-thread processes of the reference's PPO_AcM iteration restated on the CPU "
                      "(oracle/cpu_loop_ppo.py: 2000-frame single-env collection with actor sample + AcM, 10 x 10 "
                      "full-batch critic steps, the GAE loop, <= 10 clip-loss epochs of 512 with the KL stop, the "
                      "ACM ring, 5 ACM epochs of 64-sample batches over the 1e5-row ring every 3 iterations, obs "
                      "stats), one ACM cycle = 3 iterations = %d frames each (%.1f s); one_core = the same alone"
                      % (procs, res[0]["frames"], res[0]["seconds"])}


def default_cpu_procs():
    # The GPU box gives one job a 16-CPU share (os.cpu_count() reports the whole machine there)
    # and counts every process that imports the ROCm torch runtime as a GPU user (at most 16,
    # the bench's own process included): 15 workers.
    n = os.cpu_count() or 1
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    return max(1, min(15, n - 1))


# ------------------------------------------------------------------ PMC traffic (child passes)
def lib_digest():
    h = hashlib.sha1()
    with open(LIB, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:12]


def pmc_traffic(args, E, cap, kernels, steps=2):
    """HBM bytes per launch of ``kernels`` (name prefixes) from two rocprofv3 --pmc passes
    (FETCH_SIZE, WRITE_SIZE; counters cannot share a pass) over a short child run of this
    script at the same config / E / buffer.  FETCH_SIZE is doubled: gfx950 counts half the
    bytes of wide streaming reads (MI355X_MICROARCH.md "HBM"); both are KB -> x1024."""
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    per = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="spp_pmc_", dir="/tmp")
        cmd = ["timeout", "-s", "KILL", "240", rp, "--pmc", c, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", str(steps), "--warmup",
               "1", "--no-cpu-baseline", "--no-pmc", "--no-rocprof"]
        cmd += (["--envs", str(E)] if E is not None else []) + (["--buffer", str(cap)] if cap is not None else [])
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            return None, "rocprofv3 --pmc %s exit %d: %s" % (c, r.returncode, r.stdout[-300:])
        import csv
        import glob

        files = glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True)
        if not files:
            return None, "no counter csv"
        vals = {}
        for row in csv.DictReader(open(files[0])):
            for k in kernels:
                if k in row["Kernel_Name"]:
                    vals.setdefault(k, []).append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        for k, v in vals.items():
            per.setdefault(k, {})[c] = sum(v) / len(v) * 1024.0
    out = {}
    for k, d in per.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            out[k] = int(2 * d["FETCH_SIZE"] + d["WRITE_SIZE"])
    return out, "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over bench.py --config %s " \
                "--envs %s --steps %d --warmup 1, same library (sha1 %s); bytes = 2*FETCH + WRITE per launch" % (
                    args.config, E, steps, lib_digest())


def rocprof_kernel_ms(args, E, cap, kname, steps=40, warmup=5, timed_launches=None):
    """Average duration (ms) of ``kname`` over the timed launches of a child run of this script under
    ``rocprofv3 --kernel-trace`` (same config, E, buffer and library): the kernel-trace view of the
    roofline's launch time, next to the HIP-event average measured in the main run.  The steady-state
    window (from the first timed launch of ``kname``: its last ``timed_launches`` (default steps) launches) is
    summarised per kernel into ``<trace dir>/steady_kernel_stats_<config>.csv`` (Name, Calls, TotalDurationNs,
    AverageNs), the file the roofline's ``frac_rocprof`` recomputes from (warm-up launches excluded)."""
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    import csv
    import glob

    env = dict(os.environ, TMPDIR="/tmp")
    d = tempfile.mkdtemp(prefix="spp_kt_", dir="/tmp")
    cmd = ["timeout", "-s", "KILL", "300", rp, "--kernel-trace", "-d", d, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", str(steps), "--warmup",
           str(warmup), "--no-cpu-baseline", "--no-pmc", "--no-rocprof"]
    if E is not None:
        cmd += ["--envs", str(E)]
    if cap is not None:
        cmd += ["--buffer", str(cap)]
    r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        return None, "rocprofv3 --kernel-trace exit %d: %s" % (r.returncode, r.stdout[-300:])
    files = glob.glob(os.path.join(d, "**", "run_kernel_trace.csv"), recursive=True)
    if not files:
        return None, "no kernel trace csv"
    rows = list(csv.DictReader(open(files[0])))
    shutil.rmtree(d, ignore_errors=True)
    iv = sorted((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"]) for row in rows)
    mine = [x for x in iv if kname in x[2]]
    nt = timed_launches or steps
    timed = mine[-nt:] if len(mine) >= nt else mine
    if not timed:
        return None, "kernel %s not in the trace" % kname
    t0 = timed[0][0]
    per = {}
    for s0, e0, n in iv:
        if s0 >= t0:
            c = per.setdefault(n, [0, 0])
            c[0] += 1
            c[1] += e0 - s0
    out_dir = args.trace_dir
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "steady_kernel_stats_%s.csv" % args.config)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs"])
        for n, (c, tot) in sorted(per.items(), key=lambda kv: -kv[1][1]):
            w.writerow([n, c, tot, "%.1f" % (tot / c)])
    ms = sum(e0 - s0 for s0, e0, _ in timed) / len(timed) * 1e-6
    return ms, ("rocprofv3 --kernel-trace over bench.py --config %s --steps %d --warmup %d (library sha1 %s): mean "
                "of the last %d of %d launches; steady-state per-kernel summary %s" % (
                    args.config, steps, warmup, lib_digest(), len(timed), len(mine), os.path.relpath(path, REPO)))


# ------------------------------------------------------------------ HBM-bound kernels
def cuda_time(fn, reps=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def hbm_kernels(ag, cfg, B, E):
    """Algorithmic bytes per launch / HIP-event time (torch's current stream, where these ops
    launch) for the HBM-bound kernels of the step, measured right after the timed region."""
    from spprl import _lib

    rb = ag.replay_buffer
    ob, ac = cfg["ob"], cfg["ac"]
    aout = ac if cfg["algo"] == "vanilla" else ob
    n = len(rb)
    out = {}

    def rec(name, ms, nbytes, note):
        gbs = nbytes / (ms * 1e-3) / 1e9
        out[name] = {"ms": round(ms, 4), "bytes": int(nbytes), "GB/s": round(gbs, 1),
                     "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes": note}

    ms = cuda_time(lambda: rb.update_obs_mean_std())
    rec("obs_stats", ms, n * (4 * ob + 8), "one read of the live rows: len x (4 ob + 8 obs_idx)")
    idx = torch.randint(0, n, (B,), device=ag.device)
    acmc = cfg["algo"] != "vanilla"
    per_s = 16 + 8 * ob + 4 * ac + 5 + (0 if acmc else 4 * aout)
    per_w = 4 * (2 * ob + ac + 2 + (0 if acmc else aout))
    ms = cuda_time(lambda: _lib.call("sppAgentStageFromReplay", ag._h, rb._h, _lib.ptr(idx), B, _lib.stream_handle()))
    rec("replay_stage", ms, B * (per_s + per_w), "per sample: 8 idx + 8 (the record's 32-bit obs / next-obs slots) + "
        "gathered values (2 obs rows, ACM action, reward, done) + the same values written feature-major")
    obs = torch.randn(E, ob, device=ag.device)

    def add():
        s = rb.add_obs_batch(obs)
        rb.add_timestep_batch(s, s, torch.zeros(E, aout, device=ag.device), torch.zeros(E, device=ag.device),
                              torch.zeros(E, dtype=torch.uint8, device=ag.device),
                              torch.zeros(E, dtype=torch.uint8, device=ag.device),
                              None if not acmc else torch.zeros(E, ac, device=ag.device))
    ms = cuda_time(add)
    rec("replay_add", ms, E * (8 * ob + 4 * aout + 4 * ac + 4 + 2 + 24 + 8), "per env: obs row read + written, "
        "action / acm / reward / done / end written, (prev, next, ts) metadata; includes the metadata upload")
    return out


# ------------------------------------------------------------------ PPO_AcM (configs[3])
def bench_ppo(args, world, rank, dev, comm=None):
    """configs[3]: SPP-PPO HalfCheetah-v2, 16384 envs over 8 GPUs = 2048 per GPU (train/spp_ppo_hcheetah.py
    hyper-parameters).  One step = one PPO_AcM iteration: T = 16 vector steps of rollout (actor sample,
    AcM, env, ACM ring writes), 10 x 10 full-batch critic steps, GAE over [T][E], <= 10 clip-loss epochs of
    512-sample minibatches with the KL stop, the ACM regression, ring obs statistics.

    ACM cadence (acm/on_policy.py:78-82, acm/acm.py:126-141, 266-303): the reference runs update_acm(5 epochs)
    every 3 iterations of batch_size = 2000 frames over a ring of 1.1 * acm_pre_train_samples = 1.1e5 rows in
    batches of 64: sigma = 5 * 1.1e5 / (3 * 2000) = 91.67 ACM samples per env-step.  An iteration here is
    N = T * E frames per rank, so every sample count of that cadence is scaled by s = world * N / 2000 (as the
    critic's full batch already is): ring 1.1e5 * s rows, ACM batch 64 * s, still 5 epochs every 3 iterations --
    the same sigma, the same number of sequential ACM steps per cycle as the reference (5 * 1719), one
    sppAcmSgd launch per epoch spread over ~s workgroups.  N > 1: the ring is replicated (every rank writes
    every rank's rows, spprl/ppo_acm.py) and the epochs run on every rank with no per-batch collective."""
    import spprl
    from spprl import flops
    from spprl.dp import shard_seed

    if args.acm_passes is not None:
        from spprl import _lib

        _lib.call("sppSetAcmSgdPasses", int(args.acm_passes))
    E = args.envs or 2048
    T = 16
    N = T * E
    ref_batch, ref_ring, ref_acm_bs, ref_ppo_mb, acm_epochs, acm_freq = 2000, 110_000, 64, 512, 5, 3
    # N > 1: the ACM ring is replicated (every rank holds every rank's rows, spprl/ppo_acm.py), so the ACM
    # cadence is scaled by the frames of all ranks
    rw = args.rehearse_world or 0  # (one-GPU rehearsal of a rw-rank job's per-rank work)
    wj = max(world, rw)  # ranks of the job whose cadence is run
    scale = wj * N / ref_batch
    acm_bs = int(round(ref_acm_bs * scale))
    # the actor's minibatch follows the same rule (ppo.py:158-188: ppo_batch_size = 512 against 2000 frames, ~4
    # sequential clip-loss steps per epoch): 512 * s, so every sample count of the iteration scales by s alike
    ppo_mb = args.ppo_minibatch or int(round(ref_ppo_mb * scale))
    seed = shard_seed(1000, rank)
    ag = spprl.PPO_AcM(env_name="HalfCheetah-v2", gamma=0.99, actor_lr=3e-4, critic_lr=3e-4, batch_size=N,
                       ppo_batch_size=ppo_mb, kl_div_threshold=0.1, max_ppo_epochs=10, entropy_coef=0.0,
                       custom_loss=0.1, norm_closs=True, min_max_denormalize=True, denormalize_actor_out=True,
                       acm_epochs=acm_epochs, acm_batch_size=acm_bs, acm_update_freq=acm_freq, acm_lr=3e-4,
                       acm_ring_size=int(round(ref_ring * scale)), n_envs=E, device=dev, seed=0, loop_seed=seed,
                       rehearse_world=rw or None, dp_update=args.ppo_dp, comm=comm)
    rb = ag.replay_buffer
    ob, ac = ag.ob_dim, ag.ac_dim
    sigma = acm_epochs * rb.size / (acm_freq * N * wj)
    torch.manual_seed(1000)  # the same pre-filled ring on every rank (replicated)
    fill = rb.size - 2 * E  # the ACM ring after pre-training (random env actions)
    prev = rb.add_obs_batch(torch.randn(1, ob, device=dev))
    slots = rb.add_obs_batch(torch.randn(fill, ob, device=dev))
    prevs = np.concatenate([prev[-1:], slots[:-1]])
    z = torch.zeros(fill, dtype=torch.uint8, device=dev)
    rb.add_timestep_batch(prevs, slots, torch.randn(fill, ob, device=dev), torch.randn(fill, device=dev), z, z,
                          torch.rand(fill, ac, device=dev) * 2 - 1)
    ag.acm.update_obs_stats()
    ag.iteration = 1
    epochs = {"ppo": 0, "acm_updates": 0}

    def iteration():
        acm_now = ag.acm_update_freq and ag.iteration % ag.acm_update_freq == 0
        ag.perform_iteration(sync=False)
        epochs["ppo"] += ag.nets.last_epochs
        epochs["acm_updates"] += int(bool(acm_now))
        ag.iteration += 1  # ACM update every acm_update_freq iterations (on_policy.py:66-70)

    for _ in range(args.warmup):
        iteration()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    epochs["ppo"], epochs["acm_updates"] = 0, 0
    ag.acm.sgd_events = []  # HIP events around every ACM epoch launch (the dominant kernel), torch's stream
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
    value = wj * N * args.steps / elapsed
    mac = flops.onpolicy_macs(ob, ob, ac)
    # algorithmic work of the timed iterations: 100 full-batch critic steps on N samples, the PPO
    # epochs actually run (KL stop) over N samples, acm_epochs epochs over the ring per ACM update, the rollout
    # (the ACM epochs run replicated on every rank: their algorithmic share per rank is 1/world of them)
    acm_samples = epochs["acm_updates"] * acm_epochs * rb.size / wj
    flop = 2.0 * (args.steps * (mac["critic_step"] * N * 100 + (mac["A"] + mac["M"]) * N)
                  + mac["actor_step"] * N * epochs["ppo"] + mac["acm_step"] * acm_samples)
    per_env_step = flop / (args.steps * N)
    res = {"metric": "env-steps/sec (rollout+update) SPP-PPO HalfCheetah-v2", "value": round(value, 1),
           "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic: SynthEnv linear-tanh dynamics (HalfCheetah-v2 shapes ob=17, ac=6), random-init "
                   "networks, ACM ring pre-filled with N(0,1) transitions",
           "config": {"workload": "SPP-PPO HalfCheetah-v2, %d vectorized envs per GPU x %d steps per iteration "
                                  "(BASELINE.json configs[3] per-GPU shape)" % (E, T), "envs_per_gpu": E,
                      "steps_per_iteration": T, "frames_per_iteration": N, "cadence_scale": round(scale, 4),
                      "acm_ring": rb.size, "acm_batch": acm_bs, "acm_epochs_every_3_iterations": acm_epochs,
                      "acm_sigma": round(sigma, 3), "acm_updates_timed": epochs["acm_updates"],
                      "ppo_epochs_timed": epochs["ppo"], "ppo_minibatch": ppo_mb,
                      "flop_per_env_step": round(per_env_step), "parallelism": "dp%d" % world,
                      "cadence": "reference train/spp_ppo_hcheetah.py per iteration with every sample count x "
                                 "s = world*N/2000 (critic full batch N, PPO minibatch 512*s, ACM ring 1.1e5*s, "
                                 "ACM batch 64*s): the reference's sequential step counts per iteration (~4 clip-loss "
                                 "steps per epoch, 1719 ACM steps per epoch); sigma = ACM samples per env-step "
                                 "(reference 91.67)"},
           "roofline": {"bound": "mfma", "kernel": "whole iteration (64-wide MLPs, latency-bound chain of "
                                                    "dependent optimizer steps)",
                        "achieved": round(flop / elapsed / 1e12, 4), "peak": PEAK_FP32_MFMA_TFLOPS,
                        "unit": "TFLOP/s", "frac": None, "traffic": None,
                        "note": "achieved = the timed iterations' algorithmic FLOPs (critic, actor epochs run, ACM, "
                                "rollout: SURVEY §8d) / elapsed; 5 x 1719 sequential ACM steps every 3 iterations "
                                "bound the iteration by latency"},
           "losses": {k: (round(v, 5) if isinstance(v, float) else v) for k, v in ag.loss.items()}}
    res["roofline"]["frac"] = round(res["roofline"]["achieved"] / PEAK_FP32_MFMA_TFLOPS, 5)
    if ag.dp and ag.dp_update == "union":
        res["config"]["update_batch"] = ("union of %d ranks' rollouts, %d rows, replicated on every rank (one "
                                         "all-gather per iteration; no per-step gradient exchange)" % (wj, wj * N))
    elif ag.dp:
        res["config"]["update_batch"] = ("sharded: each rank's own %d rows, one gradient all-reduce per critic step "
                                         "and per clip-loss step (minibatch %d per rank = %d / %d), %s" % (
                                             N, ppo_mb // wj, ppo_mb, wj,
                                             "libspprl RCCL on the compute stream" if comm else "torch.distributed"))
    if rw:
        res["config"]["rehearsal"] = (
            "one GPU running the per-rank work of a %d-rank job: ACM ring / batch scaled for %d ranks and the "
            "replicated ring written with %d ranks' rows per iteration; %s; value = %d x this GPU's env-steps/s (a "
            "projection, not a multi-GPU measurement: the per-step all-reduces run on a one-rank communicator, so "
            "their 8-GPU latency is not in it)" % (
                rw, rw, rw, "update(mem) on the local rollout tiled to the %d-rank union shape" % rw
                if ag.dp_update == "union" else "update(mem) on the local rollout with the per-step exchange", rw))
    if world > 1:  # the replicas must stay bit-identical (identical union batch, ring and permutation streams)
        chk = torch.stack([t.double().sum() for t in (ag.nets.params[0], ag.nets.params[1], ag.acm.params[5])] +
                          [t.double().abs().sum() for t in (ag.nets.params[0], ag.nets.params[1],
                                                            ag.acm.params[5])])
        allc = [torch.empty_like(chk) for _ in range(world)]
        dist.all_gather(allc, chk)
        res["replicas_identical"] = bool(all(torch.equal(allc[0], c) for c in allc))
    # the dominant kernel: the ACM epoch (k_mlp_sgd<2 ob, 32, ac, 0>, sequential 64 x s-row Adam steps over the
    # ring), timed by HIP events around each launch on the stream it runs on
    ev = ag.acm.sgd_events
    ag.acm.sgd_events = None
    if ev:
        # one launch per epoch (sppAcmSgdEpoch: the ragged last batch inside it); rows = the ring's live rows
        ms_l = [a.elapsed_time(b) for a, b, _ in ev]
        rows = sum(n for _, _, n in ev) / len(ev)
        kflop = 2.0 * mac["acm_step"] * rows
        k_ms = sum(ms_l) / len(ms_l)
        kname = "k_mlp_sgd<%d, 32, %d, 0" % (2 * ob, ac)
        res["roofline"] = {
            "bound": "mfma", "kernel": "%s, true> (one ACM epoch: %d sequential Adam steps of %d rows, workgroups "
                                      "%d)" % (kname, -(-rows // acm_bs), acm_bs, ag.acm.acm_sgd_workgroups()),
            "achieved": round(kflop / (k_ms * 1e-3) / 1e12, 4), "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
            "frac": round(kflop / (k_ms * 1e-3) / 1e12 / PEAK_FP32_MFMA_TFLOPS, 5), "traffic": None,
            "flop_per_launch": kflop, "algorithmic": "2 x 3 x %d MAC (AcM forward + both backward GEMMs) per row x %d "
                                                     "rows per epoch" % (mac["M"], round(rows)),
            "avg_launch_ms": round(k_ms, 4), "launches": len(ms_l),
            "us_per_sgd_step": round(k_ms * 1e3 / -(-rows // acm_bs), 2),
            "whole_iteration": {"achieved": res["roofline"]["achieved"], "frac": res["roofline"]["frac"],
                                "note": res["roofline"]["note"]},
            "scope": "achieved / frac / traffic are the dominant kernel's (one ACM-epoch launch), as in every bench "
                     "line since round 4; the iteration's algorithmic rate is whole_iteration"}
        if rank == 0 and world == 1 and not args.no_rocprof:
            kt_ms, kt_src = rocprof_kernel_ms(args, args.envs, None, kname, steps=6, warmup=3, timed_launches=10)
            rl = res["roofline"]
            rl["avg_launch_ms_rocprof"] = round(kt_ms, 4) if kt_ms else None
            rl["frac_rocprof"] = round(kflop / (kt_ms * 1e-3) / 1e12 / PEAK_FP32_MFMA_TFLOPS, 5) if kt_ms else None
            rl["rocprof_source"] = kt_src
        if rank == 0 and world == 1 and not args.no_pmc:
            traffic, src = pmc_traffic(args, args.envs, None, [kname], steps=3)
            res["roofline"]["traffic"] = traffic.get(kname) if traffic else None
            res["roofline"]["traffic_source"] = src
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = ppo_cpu_baseline_report(args.cpu_procs or default_cpu_procs())
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ------------------------------------------------------------------ off-policy configs
def prefill(ag, rb, cap, E, ob, ac, aout, seed, dev, acm=True):
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
        rb.add_timestep_batch(prevs, slots, torch.randn(n, aout, device=dev).clamp(-1, 1) if not acm else
                              torch.randn(n, aout, device=dev), torch.randn(n, device=dev), z, z,
                              torch.rand(n, ac, device=dev) * 2 - 1 if acm else None)
        prev = slots
        done_fill += n
    return fill


def native_comm(world, rank, local):
    """libspprl's RCCL communicator (spprl.dp.NativeComm): its collectives run on the caller's stream,
    so the exchange needs no cross-stream event waits; rank 0's id travels by a process-group broadcast."""
    from spprl.dp import NativeComm

    def share(uid):
        box = [uid if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    return NativeComm(rank, world, local, share)


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n):
    """``bench.py --gpus N`` (N > 1) started without a launcher: run it as one process per GPU under
    ``torch.distributed.run`` (a CHILD process; this parent never touches the GPU, so no exec after GPU
    init), forward every output line to stderr except the JSON result line(s), which rank 0 prints and
    this process relays on stdout, and exit with the child's code."""
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC (the only mode the host supports)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in p.stdout:
        t = line.strip()
        if t.startswith("{") and '"metric"' in t:
            print(t, flush=True)
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    return p.wait()


def run_replicas(args):
    """--replicas R: R worker processes of this script (one vanilla-SAC run each, seed = replica index), started
    before this process touches the GPU; each reports READY after its warm-up and starts its timed steps on GO,
    which this process sends to all of them at once."""
    import subprocess

    argv, skip = [], False
    for a in sys.argv[1:]:
        if skip:
            skip = False
            continue
        if a == "--replicas":
            skip = True
            continue
        if a.startswith("--replicas="):
            continue
        argv.append(a)
    cmd = [sys.executable, os.path.abspath(__file__)] + argv + ["--replica-worker", "--no-cpu-baseline", "--no-pmc",
                                                                 "--no-rocprof"]
    procs = []
    for i in range(args.replicas):
        env = dict(os.environ, SPP_REPLICA_INDEX=str(i))
        procs.append(subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env))
    try:
        for p in procs:
            while True:
                line = p.stdout.readline()
                if not line:
                    raise RuntimeError("replica worker exited before READY (status %s)" % p.wait())
                if line.strip() == "READY":
                    break
        t0 = time.perf_counter()
        for p in procs:
            p.stdin.write("GO\n")
            p.stdin.flush()
        outs = []
        for p in procs:
            out, _ = p.communicate(timeout=1200)
            lines = [ln for ln in out.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not lines:
                raise RuntimeError("replica worker failed (status %s)" % p.returncode)
            outs.append(json.loads(lines[-1]))
        wall = time.perf_counter() - t0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    spans = [o["ms_per_step"] * o["steps"] / 1e3 for o in outs]
    res = dict(outs[0])
    res["value"] = round(args.replicas * args.steps / max(spans), 1)
    res["ms_per_step"] = round(max(spans) / args.steps * 1e3, 4)
    res["config"] = dict(res["config"], workload=res["config"]["workload"] + "; %d independent replicas sharing one "
                         "GPU" % args.replicas, parallelism="%d replicas, 1 GPU" % args.replicas)
    res["replicas"] = {"n": args.replicas, "per_replica_value": [o["value"] for o in outs],
                       "per_replica_ms_per_step": [o["ms_per_step"] for o in outs],
                       "param_checksums": [o.get("param_checksum") for o in outs],
                       "wall_s_incl_teardown": round(wall, 3),
                       "note": "value = replicas x steps / the slowest replica's timed span (each replica times its "
                               "own steps from the common GO); the same layout as cpu_baseline (concurrent "
                               "independent single-thread runs) and the reference's train/vanilla_sac_hcheetah.py "
                               "(a multiprocessing pool of independent runs)"}
    for k in ("roofline", "kernels_ms_per_launch", "kernels_tflops", "step_tflops"):
        res.pop(k, None)
    res["roofline"] = outs[0].get("roofline")
    if res["roofline"] is not None:
        res["roofline"] = dict(res["roofline"], scope="replica 0's critic-phase launches, measured while all "
                                                      "replicas ran")
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_report(args.config, args.cpu_seconds, args.cpu_procs or default_cpu_procs())
    print(json.dumps(res), flush=True)


def main():
    args = parse()
    if args.replicas > 1 and not args.replica_worker:
        if args.config != "vanilla_sac_hcheetah" or args.gpus != 1:
            sys.stderr.write("bench.py: --replicas is for --config vanilla_sac_hcheetah on one GPU\n")
            sys.exit(2)
        return run_replicas(args)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.stderr.write("bench.py: WORLD_SIZE=%s but --gpus %d: launch one rank per GPU with --gpus equal to the "
                         "rank count\n" % (env_world, args.gpus))
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SPP_DIST_BACKEND=gloo (testing only): ranks may share one GPU; the default is RCCL ("nccl")
    backend = os.environ.get("SPP_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if args.config == "ppo_hcheetah" and (args.rehearse_world or 0) > 1 and args.ppo_dp == "shard":
        # a sharded update's per-rank work includes its per-step exchange: rehearsed on a one-rank communicator
        os.environ["SPP_DP_FORCE"] = "1"
    # SPP_DP_FORCE=1 (rehearsal): the process group and the exchange also run with one rank
    distributed = world > 1 or os.environ.get("SPP_DP_FORCE", "0") == "1"
    if distributed and "RANK" not in os.environ:  # a one-rank group started without a launcher (rehearsal)
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(_free_port()))
    if distributed:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.config == "ppo_hcheetah":
        comm = None
        if distributed and backend == "nccl" and args.dp_comm == "native":
            comm = native_comm(world, rank, local)
        return bench_ppo(args, world, rank, dev, comm)
    import spprl
    from spprl import flops
    from spprl.dp import shard_seed

    cfg = CONFIGS[args.config]
    ob, ac = cfg["ob"], cfg["ac"]
    vanilla = cfg["algo"] == "vanilla"
    aout = ac if vanilla else ob
    E = args.envs or cfg["envs"]
    cap = args.buffer or cfg["buffer"]
    a = dict(cfg["agent"])
    batch_size = a.pop("batch_size")
    rho = a["update_batch_size"] * a["grad_steps"] / a["update_freq"]
    sigma = a["acm_update_batches"] * a["acm_batch_size"] / a["acm_update_freq"] if not vanilla else 0.0
    seed = shard_seed(1000, rank + int(os.environ.get("SPP_REPLICA_INDEX", "0")))
    if vanilla:
        Agent = spprl.SAC
        B, BA = a["update_batch_size"], 0
        sched = "reference" if E == 1 else "fused"
    else:
        Agent = spprl.SAC_AcM if cfg["algo"] == "sac" else spprl.DDPG_AcM
        B, BA = int(round(rho * E)), int(round(sigma * E))
        sched = "fused"
    if sched == "fused" and vanilla:
        B = int(round(rho * E))
    env = None
    if args.host_env:
        env = spprl.HostSynthEnv(E, ob, ac, max_episode_steps=1000, seed=seed, device=dev)
    ag = Agent(env_name=cfg["env"], buffer_size=cap, max_batch=max(B, BA, 128), device=dev, seed=0, n_envs=E,
               schedule=sched, random_frames=0, batch_size=batch_size, iterations=10 ** 9, loop_seed=seed, env=env,
               **({} if vanilla else dict(acm_epochs=1)), **a)
    rb = ag.replay_buffer
    if sched == "fused":
        assert ag.fused_batch_sizes()[0] == B
    comm = None
    if distributed and backend == "nccl" and args.dp_comm == "native":
        comm = native_comm(world, rank, local)
        host_sum = ag.host_sum  # the live-row counts stay on gloo (host integers: no device read)
        comm.attach(ag)
        ag.host_sum = host_sum

    fill = prefill(ag, rb, cap, E, ob, ac, aout, seed, dev, acm=not vanilla)
    ag.update_obs_stats()
    ag.iteration = 1  # past the first iteration: ACM regression is on (ddpg_acm.py:52-57)
    ag.stats_logger.frames = fill
    stats = {"passes": 0, "frames": 0}

    def obs_stats(frames):
        """update_obs_mean_std at the reference's per-frame rate (one pass per batch_size frames)."""
        if args.stats_rate == "per-step":
            ag.update_obs_stats()
            stats["passes"] += 1
            return
        f0 = stats["frames"]
        stats["frames"] += frames
        for _ in range(stats["frames"] // batch_size - f0 // batch_size):
            ag.update_obs_stats()  # global across ranks (RCCL) when N > 1
            stats["passes"] += 1

    if sched == "fused":
        def step():
            ag.collect_batch_and_train(E)  # act -> env -> replay -> rho*E grad step -> sigma*E ACM step
            obs_stats(E)
    else:
        ag._start_episodes()

        def step():  # one frame of DDPG.collect_batch_and_train (ddpg.py:192-223) with make_update
            end = ag._vector_step()
            ag.make_update()
            if bool(end[0]):
                ag._start_episodes()
            obs_stats(1)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ag.set_timing(True)
    ag.get_timing()  # clear
    stats["passes"] = 0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if args.replica_worker:  # run_replicas: start the timed steps together
        print("READY", flush=True)
        sys.stdin.readline()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
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

    if cfg["algo"] == "ddpg":
        mac = flops.ddpg_macs(ob, ac)
    else:
        mac = flops.sac_macs(ob, ac, aout=aout, acm_critic=not vanilla, with_acm=not vanilla)
    value = world * E * args.steps / elapsed
    names = ["critic_phase", "actor_phase", "dw_gemm", "adam", "acm_regress"]
    k_ms = {name: ms[i] / max(cnt[i], 1) for i, name in enumerate(names)}
    k_cnt = {name: int(cnt[i]) for i, name in enumerate(names)}
    tf = lambda m, t: 2.0 * m * B / (t * 1e-3) / 1e12 if t > 0 else 0.0  # noqa: E731
    crit_tf, act_tf = tf(mac["critic_phase"], k_ms["critic_phase"]), tf(mac["actor_phase"], k_ms["actor_phase"])
    dw_tf = tf(mac["dw"] / 2, k_ms["dw_gemm"])  # two dW launches per grad step
    bf16 = cfg.get("bf16", False)
    peak = PEAK_BF16_MFMA_TFLOPS if bf16 else PEAK_FP32_MFMA_TFLOPS
    kname = "k_ddpg_critic_phase" if cfg["algo"] == "ddpg" else "k_sac_critic_phase"
    if vanilla and os.environ.get("SPP_SAC_TEAM", "1") != "0" and \
            -(-B // 32) <= torch.cuda.get_device_properties(dev).multi_processor_count:
        kname = "k_sac_critic_team"  # small batches: the team form (csrc/sac_team.h, api.hip sac_team)
    grad_steps_per_step = k_cnt["critic_phase"] / args.steps
    flop_step = 2.0 * (mac["update"] * B * grad_steps_per_step + mac["acm_reg"] * BA + mac["act"] * E)
    metric = {"sac": "SPP-SAC ", "ddpg": "SPP-DDPG ", "vanilla": "vanilla SAC "}[cfg["algo"]] + cfg["env"]
    result = {
        "metric": "env-steps/sec (rollout+update) %s" % metric,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 MFMA MLP, fp32 accumulate / targets / optimizer" if bf16 else "fp32",
        "data": "synthetic: SynthEnv linear-tanh dynamics (%s shapes ob=%d, ac=%d)%s, random-init networks, replay "
                "pre-filled with N(0,1) transitions" % (cfg["env"], ob, ac, ", stepped on the HOST (HostSynthEnv, "
                                                        "numpy) behind pinned H2D/D2H side-stream copies"
                                                        if args.host_env else ""),
        "config": {"workload": cfg["workload"] % E if "%d" in cfg["workload"] else cfg["workload"],
                   "envs_per_gpu": E, "update_batch": B, "acm_batch": BA, "rho": rho, "sigma": sigma,
                   "schedule": sched, "replay_rows_per_gpu": cap, "parallelism": "dp%d" % world,
                   "env": "host (HostSynthEnv, PCIe-inclusive)" if args.host_env else "device (SynthVecEnv)",
                   "obs_stats": "%s rate: %d passes over %d timed steps (one per %d frames)" % (
                       args.stats_rate, stats["passes"], args.steps, batch_size),
                   "index_rng": ("philox (sppRandIndex, device); the reference's MT19937 stream "
                                 "(np.random.randint, replay_buffer.py:234) is bit-exact through sppMTRandint on "
                                 "the E = 1 reference schedule only") if sched == "fused" else
                                "MT19937 (np.random.randint stream, replay_buffer.py:234), host"},
        "roofline": {"bound": "mfma", "kernel": "%s (critic targets + critic fwd/bwd)" % kname,
                     "achieved": round(crit_tf, 3), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(crit_tf / peak, 5), "traffic": None,
                     "flop_per_launch": 2.0 * mac["critic_phase"] * B,
                     "algorithmic": "2 x %d MAC per replayed sample x B = %d samples per launch" % (
                         mac["critic_phase"], B),
                     "avg_launch_ms": round(k_ms["critic_phase"], 4), "launches": k_cnt["critic_phase"]},
        "kernels_ms_per_launch": {k: round(v, 4) for k, v in k_ms.items()},
        "kernels_tflops": {"critic_phase": round(crit_tf, 2), "actor_phase": round(act_tf, 2),
                           "dw_gemm": round(dw_tf, 2)},
        "step_tflops": round(flop_step * args.steps / elapsed / 1e12, 3),
        "losses": {k: round(v, 5) for k, v in losses.items()},
    }
    chk = torch.stack([p.double().sum() for p in ag.params.values()] +
                      [p.double().abs().sum() for p in ag.params.values()])
    result["param_checksum"] = hashlib.sha1(chk.cpu().numpy().tobytes()).hexdigest()[:16]
    if world > 1:  # data-parallel replicas must stay bit-identical (same averaged grads, same Adam)
        allc = [torch.empty_like(chk) for _ in range(world)]
        dist.all_gather(allc, chk)
        result["replicas_identical"] = bool(all(torch.equal(allc[0], c) for c in allc))
    if world == 1 and not args.replica_worker:
        result["hbm_kernels"] = hbm_kernels(ag, cfg, B, E)
    if rank == 0 and world == 1 and not args.no_rocprof:
        kt_ms, kt_src = rocprof_kernel_ms(args, E, cap, kname)
        rl = result["roofline"]
        rl["avg_launch_ms_rocprof"] = round(kt_ms, 4) if kt_ms else None
        rl["frac_rocprof"] = round(rl["flop_per_launch"] / (kt_ms * 1e-3) / 1e12 / peak, 5) if kt_ms else None
        rl["rocprof_source"] = kt_src
        rl["frac_note"] = ("frac = algorithmic FLOP per launch / HIP-event mean launch time in this run's timed "
                           "region; frac_rocprof = the same FLOP / the rocprofv3 kernel-trace mean of the same "
                           "kernel over a child run's timed launches")
    if rank == 0 and world == 1 and not args.no_pmc:
        traffic, src = pmc_traffic(args, E, cap, [kname, "k_stats_", "k_replay_stage_fm"])
        if traffic:
            result["roofline"]["traffic"] = traffic.get(kname)
            result["roofline"]["traffic_source"] = src
            result["pmc_bytes_per_launch"] = traffic
        else:
            result["roofline"]["traffic_source"] = src
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_report(args.config, args.cpu_seconds,
                                                     args.cpu_procs or default_cpu_procs())
    if distributed:
        result["config"]["dp_comm"] = "native RCCL (libspprl, compute stream)" if comm else "torch.distributed"
    if rank == 0:
        print(json.dumps(result), flush=True)
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
