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


# Reference constructor kwargs the device path accepts and that change nothing it computes (the reason for
# each).  Any other keyword an agent does not take explicitly raises TypeError, as the reference's own
# constructor chain does (MetaLearner.__init__, rl.py:17-26, takes no **kwargs).
NO_EFFECT_KWARGS = {
    "use_gpu": "device placement is the `device` argument (rl.py:40)",
    "tensorboard_comment": "event-file name suffix only (rl.py:68-70, 310)",
    "log_dir": "basic text logs / final-model directory (rl.py:177-181, 221, 234, 316)",
    "verbose": "console log level (rl.py:182, 332)",
    "render": "rollout video to TensorBoard (rl.py:81, 183): out of scope (DESIGN §7)",
    "acm_val_buffer_size": "validation buffer for the logged loss['acm_val'] only (acm.py:140-146, 301-303); "
                           "never enters a gradient",
    "pi_update_freq": "stored for hparams only: its use is commented out (sac.py:260, sac_acm.py:139)",
}
ON_POLICY_NO_EFFECT_KWARGS = dict(NO_EFFECT_KWARGS, **{
    "tensorboard_dir": "PPO_AcM logs no TensorBoard panels on this path",
    "debug_mode": "extra TensorBoard panels only (on_policy.py:128-131)",
    "obs_norm_alpha": "redundant in the AcM path: A2C_AcM warns and never updates a running Memory "
                      "normaliser (on_policy.py:138-144, 63-86)",
})


def check_kwargs(owner, kw, allowed=None):
    """Raise TypeError for keywords neither taken explicitly nor listed in ``allowed`` (NO_EFFECT_KWARGS)."""
    allowed = NO_EFFECT_KWARGS if allowed is None else allowed
    bad = sorted(k for k in kw if k not in allowed)
    if bad:
        raise TypeError("%s got unexpected keyword argument(s): %s (accepted with no effect: %s)"
                        % (owner, ", ".join(bad), ", ".join(sorted(allowed))))


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


def acm_columns(acm_ob_idx, ob):
    """AcMTrainer's acm_ob_idx (acm/acm.py:94-99): None for the whole observation vector, else the list of ob
    columns acm_cat takes from obs and next_obs (acm.py:260-264).  The reference builds the AcM with ob +
    len(acm_ob_idx) inputs (acm.py:148) but feeds it 2 * len(acm_ob_idx) (acm_cat), so only lists of length ob
    (a permutation, or repeats) run there; shorter lists fail at the first ACM update in the reference and are
    refused here at construction.  Returns None (identity) or the list."""
    if acm_ob_idx is None:
        return None
    cols = [int(i) for i in acm_ob_idx]
    if any(i < 0 or i >= ob for i in cols):
        raise ValueError("acm_ob_idx out of range for ob_dim %d: %r" % (ob, cols))  # (acm.py:98-99 asserts)
    if len(cols) != ob:
        raise ValueError("acm_ob_idx of length %d with ob_dim %d: the reference's AcM takes ob + %d inputs "
                         "(acm/acm.py:148) but acm_cat gives it 2 x %d (acm.py:260-264), so only length-ob lists "
                         "run in the reference" % (len(cols), ob, len(cols), len(cols)))
    return None if cols == list(range(ob)) else cols
