"""spprl — MI355X-native SPP-RL hot path (rollout -> HBM replay -> SAC_AcM update).

Host side keeps rltoolkit's agent / buffer API; all device work runs in
libspprl.so (hand-written HIP kernels for gfx950) through the C-ABI in
include/spprl.h.
"""
from . import _lib, config, dp, nets, onpolicy, ppo  # noqa: F401
from ._lib import SppError, load  # noqa: F401
from .replay import BufferAcMOffPolicy, ReplayBuffer  # noqa: F401
from .sac_acm import SAC_AcM  # noqa: F401
from .sac import SAC  # noqa: F401
from .ddpg_acm import DDPG_AcM  # noqa: F401
from .ppo_acm import PPO_AcM  # noqa: F401
from .trainer import HostSynthEnv, HostVecEnv, SynthVecEnv  # noqa: F401

__all__ = ["SAC", "SAC_AcM", "DDPG_AcM", "PPO_AcM", "SynthVecEnv", "HostVecEnv", "HostSynthEnv", "BufferAcMOffPolicy", "ReplayBuffer", "SppError", "load"]
