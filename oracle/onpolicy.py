"""ORACLE (test infrastructure only): A2C / PPO on-policy network steps, restated.

Networks (rltoolkit/basic_model.py:7-76), flat buffers in state_dict order:
  Actor (continuous): log_scale [aout], fc1 ob->64, fc2 64->64, fc3 64->aout;
                      mu = tanh(fc3(tanh(fc2(tanh(fc1 x))))) * lim, Independent(Normal(mu, exp(log_scale)))
  Critic:             fc1 ob->64, fc2 64->64, fc3 64->1 (tanh hidden)
Steps:
  critic_step   A2C.update_critic inner step (rltoolkit/algorithms/a2c/a2c.py:209-219):
                loss = 0.5 * mean((q - V(x))^2); critic_steps: nsteps of them with Adam
  actor_step    PPO.update_actor / PPO_AcM.update_actor_acm minibatch body
                (algorithms/ppo/ppo.py:174-190, acm/on_policy.py:189-205):
                loss = clip_loss(lp_old, lp_new, A) - entropy_coef * entropy
"""
import math

import numpy as np
import torch

H = 64


def actor_layout(ob, aout):
    return [("log_scale", (aout,)), ("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)),
            ("fc2.bias", (H,)), ("fc3.weight", (aout, H)), ("fc3.bias", (aout,))]


def critic_layout(ob):
    return [("fc1.weight", (H, ob)), ("fc1.bias", (H,)), ("fc2.weight", (H, H)), ("fc2.bias", (H,)),
            ("fc3.weight", (1, H)), ("fc3.bias", (1,))]


def _lin(x, p, n):
    return x @ p[n + ".weight"].T + p[n + ".bias"]


def critic(p, x):
    h = torch.tanh(_lin(x, p, "fc1"))
    h = torch.tanh(_lin(h, p, "fc2"))
    return _lin(h, p, "fc3")


def actor_mean(p, x, lim):
    h = torch.tanh(_lin(x, p, "fc1"))
    h = torch.tanh(_lin(h, p, "fc2"))
    return torch.tanh(_lin(h, p, "fc3")) * lim


def actor_dist(p, x, lim):
    normal = torch.distributions.Normal(actor_mean(p, x, lim), torch.exp(p["log_scale"]))
    return torch.distributions.Independent(normal, 1)


def _params(flat, layout, dtype=torch.float32):
    out, o = {}, 0
    flat = torch.as_tensor(np.asarray(flat), dtype=dtype)
    for n, shape in layout:
        k = int(np.prod(shape))
        out[n] = flat[o:o + k].reshape(shape).clone().requires_grad_(True)
        o += k
    return out


def _flat(gs):
    return torch.cat([g.reshape(-1) for g in gs]).numpy()


def critic_step(flat, ob, x, q, dtype=torch.float32):
    """Returns (loss, grad) of 0.5 * mean((q - V(x))^2) (dtype float64: a reference for large batches)."""
    p = _params(flat, critic_layout(ob), dtype)
    v = critic(p, torch.as_tensor(x, dtype=dtype)).squeeze(-1)
    adv = torch.as_tensor(q, dtype=dtype) - v
    loss = 0.5 * adv.pow(2).mean()
    return loss.item(), _flat(torch.autograd.grad(loss, list(p.values())))


def critic_steps(flat, ob, x, q, lr, nsteps, dtype=torch.float32):
    """A2C.update_critic's inner loop for one target (a2c.py:209-219): nsteps full-batch Adam steps on
    0.5 * mean((q - V(x))^2) over the same rows.  Returns (flat, per-step losses)."""
    from oracle.adam import OracleAdam

    p = torch.from_numpy(np.array(flat, np.float64 if dtype == torch.float64 else np.float32, copy=True))
    opt = OracleAdam([p], lr)
    losses = []
    for _ in range(nsteps):
        loss, g = critic_step(p.numpy(), ob, x, q, dtype=dtype)
        opt.step([torch.from_numpy(g)])
        losses.append(loss)
    return p.numpy(), losses


def actor_step(flat, ob, aout, lim, x, act, lp_old, adv, eps_clip=0.2, entropy_coef=0.0, next_obs=None):
    """Returns ({actor, kl, entropy, dist}, grad) of clip_loss - entropy_coef * entropy."""
    p = _params(flat, actor_layout(ob, aout))
    dist = actor_dist(p, torch.as_tensor(x), torch.as_tensor(lim))
    lp_new = dist.log_prob(torch.as_tensor(act))
    ratio = torch.exp(lp_new - torch.as_tensor(lp_old))
    clipped = torch.clamp(ratio, 1 - eps_clip, 1 + eps_clip)
    A = torch.as_tensor(adv)
    actor_loss = -(torch.min(ratio * A, clipped * A)).mean()
    ent = dist.entropy().mean()
    loss = actor_loss - entropy_coef * ent
    g = _flat(torch.autograd.grad(loss, list(p.values())))
    out = {"actor": actor_loss.item(), "kl": (torch.as_tensor(lp_old) - lp_new).mean().item(), "entropy": ent.item()}
    if next_obs is not None:
        out["dist"] = torch.nn.functional.mse_loss(torch.as_tensor(act), torch.as_tensor(next_obs)).item()
    return out, g


def update_actor_epochs(flat, ob, aout, lim, x, act, lp_old, adv, next_obs, lr, max_epochs, kl_threshold,
                        batch_size, eps_clip=0.2, entropy_coef=0.0, custom_loss=0.0, perms=None):
    """PPO_AcM.update_actor_acm (rltoolkit/acm/on_policy.py:164-216; PPO.update_actor ppo.py:152-192):
    epochs of minibatch Adam steps on clip_loss - entropy_coef * entropy, stopped when the KL of the
    previous epoch's LAST minibatch (pre-step log-probs, utils.kl_divergence utils.py:48-59) reached the
    threshold; losses summed over the steps and divided by i + 1 after the loop (one more than the epochs
    run when the check broke it).  ``adv`` are the already normalised advantages; ``perms`` one row
    permutation per epoch (identity by default).  Returns (flat, losses, kls, counter increment)."""
    from oracle.adam import OracleAdam

    flat = torch.from_numpy(np.array(flat, np.float32, copy=True))
    opt = OracleAdam([flat], lr)
    n = len(x)
    tot = {"actor": 0.0, "entropy": 0.0, "policy": 0.0, "dist": 0.0}
    kl, kls, i = 0.0, [], 0
    for i in range(max_epochs):
        if kl >= kl_threshold:
            break
        perm = np.arange(n) if perms is None else np.asarray(perms[i])
        for s in range(0, n, batch_size):
            b = perm[s:s + batch_size]
            out, g = actor_step(flat.numpy(), ob, aout, lim, x[b], act[b], lp_old[b], adv[b], eps_clip=eps_clip,
                                entropy_coef=entropy_coef, next_obs=next_obs[b])
            opt.step([torch.from_numpy(g)])
            tot["actor"] += out["actor"]
            tot["entropy"] += out["entropy"]
            tot["dist"] += out["dist"]
            tot["policy"] += out["actor"] - entropy_coef * out["entropy"] + custom_loss * out["dist"]
            kl = out["kl"]
        kls.append(kl)
    return flat.numpy(), {k: v / (i + 1) for k, v in tot.items()}, kls, i + 1


def act(flat, ob, aout, lim, x, eps=None):
    p = _params(flat, actor_layout(ob, aout))
    with torch.no_grad():
        mu = actor_mean(p, torch.as_tensor(x), torch.as_tensor(lim))
        sc = torch.exp(p["log_scale"])
        a = mu if eps is None else mu + sc * torch.as_tensor(eps)
        lp = torch.distributions.Independent(torch.distributions.Normal(mu, sc), 1).log_prob(a)
    return a.numpy(), lp.numpy()


def init_flat(layout, seed, log_scale=-1.34):
    """nn.Linear-style init; log_scale = -1.34 (basic_model.py:18-20)."""
    rng = np.random.RandomState(seed)
    parts, fan = [], None
    for n, shape in layout:
        if n == "log_scale":
            parts.append(np.full(shape, log_scale, np.float32))
            continue
        if n.endswith("weight"):
            fan = shape[1]
        b = 1.0 / math.sqrt(fan)
        parts.append(rng.uniform(-b, b, shape).astype(np.float32))
    return np.concatenate([x.reshape(-1) for x in parts])
