"""Algorithmic work of the update path, the single source for
bench.py's roofline figures.

MAC counts are per replayed sample and count only the products the reference's
update actually needs (forward passes, the backward passes whose results are used,
weight gradients of the trained nets).  H = 256 hidden units (sac/models.py:17-20,
ddpg/models.py:5-44); AcM 64-32 (basic_model.py:108-132); BasicAcM 100-50 with a
50-wide skip (acm/models/basic_acm.py:11-32).
"""

H = 256


def sac_macs(ob, ac, aout=None, acm_critic=True, with_acm=True):
    """SAC_AcM (sac_acm.py:30-162): per replayed sample MACs of
    critic phase, actor phase and the weight-gradient GEMMs; plus per-sample ACM
    regression and per-env act MACs.  with_acm=False: vanilla SAC (sac.py:138-280)."""
    aout = ob if aout is None else aout
    ca = ac if acm_critic else aout
    A = ob * H + H * H + H * 2 * aout             # actor forward (trunk + mu/log_std heads)
    M = (2 * ob * 64 + 64 * 32 + 32 * ac) if with_acm else 0  # AcM forward
    C = (ob + ca) * H + H * H + H                 # one critic forward
    critic_phase = A + M + 2 * C + 2 * C + 2 * (H + H * H)   # targets (actor', ACM, 2 target critics); 2 critics fwd + bwd
    actor_phase = (A + M + 2 * C + 2 * (H + H * H + ca * H)  # actor fwd, ACM, critics fwd; dQ/da through both critics
                   + ((ac * 32 + 32 * 64 + 64 * aout) if with_acm else 0)  # through the frozen ACM
                   + (2 * aout * H + H * H))                  # heads + layer-2 input gradients of the actor
    dw = 2 * C + A                                            # weight gradients of both critics and the actor
    acm_reg = (M + M + (ac * 32 + 32 * 64)) if with_acm else 0  # ACM fwd, dW, hidden-layer input grads
    act = A + M
    return dict(A=A, M=M, C=C, critic_phase=critic_phase, actor_phase=actor_phase, dw=dw, acm_reg=acm_reg,
                act=act, update=critic_phase + actor_phase + dw)


def ddpg_macs(ob, ac, aout=None, acm_critic=True):
    """DDPG_AcM with BasicAcM (ddpg_acm.py:100-201, train/spp_ddpg_hcheetah.py)."""
    aout = ob if aout is None else aout
    ca = ac if acm_critic else aout
    A = ob * H + H * H + H * aout                 # actor forward
    M = 2 * ob * 100 + 100 * 50 + 2 * ob * 50 + 50 * ac   # BasicAcM forward (fc1, fc2, fc21 skip, fc3)
    C = (ob + ca) * H + H * H + H
    critic_phase = A + M + C + C + (H + H * H)    # target actor, ACM, target critic; critic fwd + bwd
    actor_phase = (A + M + C + (H + H * H + ca * H)          # actor fwd, ACM, critic fwd; dQ/da
                   + (ac * 50 + 50 * 100 + 100 * aout + 50 * aout)  # through BasicAcM to the actor output
                   + (aout * H + H * H))                      # actor head + layer-2 input gradients
    dw = C + A
    acm_reg = M + M + (ac * 50 + 50 * 100)
    act = A + M
    return dict(A=A, M=M, C=C, critic_phase=critic_phase, actor_phase=actor_phase, dw=dw, acm_reg=acm_reg,
                act=act, update=critic_phase + actor_phase + dw)


def onpolicy_macs(ob, aout, ac):
    """PPO_AcM per-sample MACs (basic_model.py:7-76, 108-132): 64-wide tanh Actor / Critic, AcM 64-32."""
    h = 64
    A = ob * h + h * h + h * aout
    V = ob * h + h * h + h
    M = 2 * ob * 64 + 64 * 32 + 32 * ac
    return dict(A=A, V=V, M=M,
                critic_step=3 * V,          # forward, input-gradient and weight-gradient passes
                actor_step=3 * A,
                acm_step=3 * M)
