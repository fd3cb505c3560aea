"""ctypes binding of libspprl.so (the C-ABI declared in include/spprl.h).

The library is loaded AFTER torch so both share torch's HIP runtime
(libamdhip64.so.7 is resolved once per process by SONAME).  There is no
fallback: if the library is missing or fails to load, every entry point
raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the HIP library: shared runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPPRL_LIB") or os.path.join(HERE, "libspprl.so")

(SPP_NET_ACTOR, SPP_NET_CRITIC1, SPP_NET_CRITIC2, SPP_NET_CRITIC1_TARG, SPP_NET_CRITIC2_TARG, SPP_NET_ACM,
 SPP_NET_ACTOR_TARG) = range(7)
SPP_ALGO_SAC_ACM, SPP_ALGO_DDPG_ACM, SPP_ALGO_SAC = 1, 2, 3
SPP_BUCKET_CRITIC, SPP_BUCKET_ACTOR, SPP_BUCKET_ACM, SPP_BUCKET_ALL = range(4)
SPP_COMM_ID_BYTES = 128
SPP_DP1_REUSE_BRACKET = 0x100  # sppReplayObsStatsDP1 phase flag (spprl.h)
NUM_LOSSES = 8

c_int, c_int64, c_uint32, c_uint64, c_float, c_void_p = (ctypes.c_int, ctypes.c_int64, ctypes.c_uint32,
                                                         ctypes.c_uint64, ctypes.c_float, ctypes.c_void_p)


class SppError(RuntimeError):
    pass


class AgentConfig(ctypes.Structure):
    _fields_ = [("algo", c_int), ("ob", c_int), ("aout", c_int), ("ac", c_int), ("acm_critic", c_int),
                ("min_max_denormalize", c_int), ("norm_closs", c_int), ("custom_loss", c_float),
                ("gamma", c_float), ("tau", c_float), ("actor_lr", c_float), ("critic_lr", c_float),
                ("alpha_lr", c_float), ("acm_lr", c_float), ("target_entropy", c_float), ("max_batch", c_int),
                ("mlp_bf16", c_int)]


class OnPolicyConfig(ctypes.Structure):
    _fields_ = [("ob", c_int), ("aout", c_int), ("actor_lr", c_float), ("critic_lr", c_float),
                ("ppo_epsilon", c_float), ("entropy_coef", c_float), ("max_batch", c_int)]


class Batch(ctypes.Structure):
    _fields_ = [("B", c_int), ("obs", c_void_p), ("next_obs", c_void_p), ("action", c_void_p),
                ("reward", c_void_p), ("done", c_void_p), ("acm_action", c_void_p)]


class ReplayView(ctypes.Structure):
    _fields_ = [("obs", c_void_p), ("obs_idx", c_void_p), ("rec", c_void_p), ("rec_words", c_int),
                ("rec_acm", c_int), ("rec_act", c_int)]


P = ctypes.POINTER
# name: (restype, argtypes)
_SIGS = {
    "sppGetLastError": (ctypes.c_char_p, []),
    "sppGetVersion": (c_int, []),
    "sppMTCreate": (c_int, [P(c_void_p), c_uint32]),
    "sppMTRandint": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
    "sppMTDestroy": (c_int, [c_void_p]),
    "sppRandNormal": (c_int, [c_void_p, c_int64, c_uint64, c_uint64, c_void_p]),
    "sppRandIndex": (c_int, [c_void_p, c_int64, c_int64, c_uint64, c_uint64, c_void_p]),
    "sppRandPermScratchBytes": (c_int64, [c_int64]),
    "sppRandPerm": (c_int, [c_void_p, c_int64, c_uint64, c_uint64, c_void_p, c_int64, c_void_p]),
    "sppReplayCreate": (c_int, [P(c_void_p), c_int64, c_int, c_int, c_int, c_int]),
    "sppReplayDestroy": (c_int, [c_void_p]),
    "sppReplayAddObs": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "sppReplayAddStep": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p]),
    "sppReplayState": (c_int, [c_void_p, P(c_int64), P(c_int64), P(c_int64)]),
    "sppReplayReset": (c_int, [c_void_p]),
    "sppReplayGather": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p]),
    "sppReplayObsStats": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "sppReplayGetView": (c_int, [c_void_p, P(ReplayView)]),
    "sppReplayCreateEx": (c_int, [P(c_void_p), c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "sppReplayLastRollout": (c_int, [c_void_p, P(c_int64), P(c_int64), c_void_p]),
    "sppCommGetUniqueId": (c_int, [c_void_p]),
    "sppCommInitRank": (c_int, [P(c_void_p), c_int, c_void_p, c_int, c_int]),
    "sppCommDestroy": (c_int, [c_void_p]),
    "sppAllReduceGrads": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sppCommAllReduceSum": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "sppCommAllGather": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "sppAgentCreate": (c_int, [P(c_void_p), P(AgentConfig), c_int]),
    "sppAgentDestroy": (c_int, [c_void_p]),
    "sppAgentNetSize": (c_int, [c_void_p, c_int, P(c_int64)]),
    "sppAgentBindNet": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sppAgentSetLimits": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sppAgentBindNormalizer": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sppAgentBindAlpha": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sppAgentSetSteps": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int64]),
    "sppAgentGetSteps": (c_int, [c_void_p, c_void_p]),
    "sppSacAcmUpdate": (c_int, [c_void_p, P(Batch), c_void_p, c_void_p, c_void_p, c_void_p]),
    "sppSacAcmCriticGrads": (c_int, [c_void_p, P(Batch), c_void_p, c_void_p, c_void_p]),
    "sppSacAcmCriticApply": (c_int, [c_void_p, c_void_p]),
    "sppSacAcmActorGrads": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "sppSacAcmActorApply": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sppAgentStageFromReplay": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "sppAgentStagePost": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "sppSacAcmUpdateStaged": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p, c_void_p]),
    "sppAcmRegressStep": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "sppPolicyAct": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_float, c_int, c_int, c_void_p,
                             c_void_p, c_void_p]),
    "sppAgentBindAlphaGrad": (c_int, [c_void_p, c_void_p]),
    "sppSacAcmDrawEps": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p]),
    "sppAgentReadEps": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "sppAgentImageCount": (c_int, [c_void_p, c_int, c_void_p]),
    "sppAgentUnpackImage": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sppAcmRegressGrads": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "sppAcmRegressApply": (c_int, [c_void_p, c_void_p]),
    "sppReplayGatherAcm": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "sppReplaySetAcmColumns": (c_int, [c_void_p, c_void_p, c_int]),
    "sppAgentSetTiming": (c_int, [c_void_p, c_int]),
    "sppAgentGetTiming": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sppSynthEnvStep": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "sppDdpgAcmUpdate": (c_int, [c_void_p, P(Batch), c_void_p, c_void_p]),
    "sppDdpgAcmCriticGrads": (c_int, [c_void_p, P(Batch), c_void_p, c_void_p]),
    "sppDdpgAcmCriticApply": (c_int, [c_void_p, c_void_p]),
    "sppDdpgAcmActorGrads": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sppDdpgAcmActorApply": (c_int, [c_void_p, c_void_p]),
    "sppOnpCreate": (c_int, [P(c_void_p), P(OnPolicyConfig), c_int]),
    "sppOnpDestroy": (c_int, [c_void_p]),
    "sppOnpNetSize": (c_int, [c_void_p, c_int, P(c_int64)]),
    "sppOnpBindNet": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sppOnpSetLimits": (c_int, [c_void_p, c_void_p]),
    "sppOnpValue": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "sppOnpCriticGrads": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "sppOnpCriticApply": (c_int, [c_void_p, c_void_p]),
    "sppOnpActorGrads": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                 c_void_p]),
    "sppOnpActorApply": (c_int, [c_void_p, c_void_p]),
    "sppOnpAct": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sppGaeScan": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, ctypes.c_double,
                           ctypes.c_double,
                            c_int, c_void_p, c_void_p, c_void_p]),
    "sppPpoClipLoss": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p, c_void_p]),
    "sppAdvNormalize": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "sppRandUniform": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int, c_uint64, c_uint64, c_void_p]),
    "sppEpisodeAccum": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "sppSynthEnvReset": (c_int, [c_void_p, c_void_p, c_int, c_int, c_uint64, c_uint64, c_void_p]),
    "sppAgentSetLr": (c_int, [c_void_p, c_float, c_float, c_float, c_float]),
    "sppReplayObsStatsDPHistSize": (c_int, [c_void_p]),
    "sppReplayObsStatsDP": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_int, P(c_int), c_void_p]),
    "sppReplayObsStatsDP1SampleRows": (c_int, [c_void_p, c_int, c_int64]),
    "sppReplaySetObsStatsCaps": (c_int, [c_void_p, c_int, c_int]),
    "sppReplayObsStatsDP1": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "sppObsNormalize": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                c_void_p, c_void_p]),
    "sppAdvSums": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "sppAdvNormalizeGlobal": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "sppAcmSgd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),  # h, x, y, n, bs
    "sppAcmSgdEpoch": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),  # h, x, y, rows, bs
    "sppAcmSgdStatus": (c_int, [c_void_p, c_void_p]),
    "sppOnpActorEpoch": (c_int, [c_void_p] * 7 + [c_int, c_int, c_void_p, c_void_p]),
    "sppOnpCriticSteps": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "sppOnpCriticStepGrads": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_float, c_void_p]),
    "sppOnpActorStepGrads": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                     c_void_p, c_float, c_void_p]),
    "sppOnpCriticStepsMaxBatch": (c_int, [c_void_p]),
    "sppOnpReserveWorkgroups": (c_int, [c_void_p, c_int]),
    "sppOnpActorEpochMaxBatch": (c_int, [c_void_p]),
    "sppOnpActorEpochStatus": (c_int, [c_void_p, c_void_p]),
    "sppOnpSyncStatusAsync": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sppSetSgdSpinLimit": (c_int, [c_int]),
    "sppSetAcmSgdPasses": (c_int, [c_int]),
    "sppAcmSgdStatusAsync": (c_int, [c_void_p, c_void_p, c_void_p]),
    "sppAcmSgdMaxBatch": (c_int, [c_void_p]),
    "sppAcmSgdWorkgroups": (c_int, [c_void_p, c_int]),
    "sppDebugReadProf": (c_int, [c_void_p, c_int]),
    "sppDebugDense": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
}
EXPORTED = tuple(_SIGS)

_lib = None


def load():
    """Load libspprl.so or raise (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SppError("libspprl.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def check(status):
    if status != 0:
        msg = load().sppGetLastError().decode(errors="replace")
        raise SppError("spprl status %d: %s" % (status, msg))


def call(name, *args):
    check(getattr(load(), name)(*args))


def ptr(t, dtype=None):
    """Device pointer of a contiguous tensor (None -> NULL)."""
    if t is None:
        return None
    if dtype is not None and t.dtype != dtype:
        raise TypeError("expected %s, got %s" % (dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
