"""Defaults of the hot path, mirroring rltoolkit/config.py (reference @ v0).

Only the constants that shape the SPP off-policy rollout/update path and its
training loop (rl.py, ddpg.py, acm.py cadence) are kept.
"""
ITERATIONS = 2000
GAMMA = 0.95
BATCH_SIZE = 200
STATS_FREQ = 20
DDPG_LR = 1e-3
TAU = 0.005
UPDATE_BATCH_SIZE = 100
BUFFER_SIZE = int(1e6)
RANDOM_FRAMES = 100
UPDATE_FREQ = 50
GRAD_STEPS = 50
ACT_NOISE = 0.1
ALPHA_LR = 1e-3
ALPHA = 0.2
ACM_LR = 3e-3
ACM_EPOCHS = 1
ACM_PRE_TRAIN_SAMPLES = 1000
ACM_PRE_TRAIN_N_EPOCHS = 10
ACM_SCHEDULER_STEP = 25
ACM_SCHEDULER_GAMMA = 0.5
ACM_UPDATE_BATCHES = False
ACM_KEEP_PRE_TRAIN = True
ACM_BATCH_SIZE = 128
ACM_UPDATE_FREQ = 1
ACM_CRITIC = False
MIN_MAX_DENORMALIZE = False
DENORMALIZE_ACTOR_OUT = False
NORM_CLOSS = True
OBS_NORM = False
MAX_ABS_OBS_VALUE = 10

# gym env shapes the reference trains on (observation dim, action dim, action high,
# episode limit); gym/mujoco themselves are not part of the hot path.
ENV_SPECS = {
    "Hopper-v2": (11, 3, 1.0, 1000),
    "HalfCheetah-v2": (17, 6, 1.0, 1000),
    "Walker2d-v2": (17, 6, 1.0, 1000),
    "Ant-v2": (111, 8, 1.0, 1000),
    "Ant-v3": (111, 8, 1.0, 1000),
    "Pendulum-v0": (3, 1, 2.0, 200),
}


def default_max_batch(update_batch_size, kw):
    """Largest batch the agent's device scratch must hold when the caller gives no
    ``max_batch``: the reference batch, or with E > 1 envs the fused schedule's rho*E
    grad-step batch and sigma*E ACM batch (trainer.OffPolicyLoop.fused_batch_sizes)."""
    env = kw.get("env")
    E = int(env.n) if env is not None else int(kw.get("n_envs", 1))
    rho = update_batch_size * kw.get("grad_steps", GRAD_STEPS) / kw.get("update_freq", UPDATE_FREQ)
    nb = kw.get("acm_update_batches", ACM_UPDATE_BATCHES)
    sigma = nb * kw.get("acm_batch_size", ACM_BATCH_SIZE) / kw.get("acm_update_freq", ACM_UPDATE_FREQ) if nb else 0
    out = max(int(update_batch_size), int(kw.get("acm_batch_size", ACM_BATCH_SIZE)))
    if E > 1 and kw.get("schedule", "fused") == "fused":
        out = max(out, int(round(rho * E)), int(round(sigma * E)))
    return out
