/* spprl.h — C-ABI of the MI355X-native SPP-RL hot path (libspprl.so).
 *
 * Replaces the Python-method boundary of rltoolkit (raznem/spp-rl @ v0) for the
 * off-policy SPP rollout -> replay -> update loop.  Each entry
 * point cites the reference interface it stands in for.
 *
 * Conventions
 *   - Every function returns sppStatus (0 = OK); sppGetLastError() gives text.
 *     No C++ exception crosses this boundary.
 *   - Device buffers are CALLER-OWNED (e.g. torch tensors); handles own only
 *     internal scratch.  All device work is stream-ordered on the hipStream_t
 *     passed in (void* here so the header needs no HIP include) and async:
 *     losses are written to device memory, nothing synchronises the host.
 *   - One host thread per handle; one process per GPU.
 *   - Matrices are row-major, float32, nn.Linear layout ([out][in]); each
 *     network's parameters are ONE flat buffer in state_dict order (layouts
 *     in DESIGN.md §Data layout).
 */
#ifndef SPPRL_H
#define SPPRL_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int sppStatus;
enum {
  SPP_OK = 0,
  SPP_E_INVALID_ARG = 1,
  SPP_E_SHAPE = 2,
  SPP_E_OOM = 3,
  SPP_E_HIP = 4,
  SPP_E_STATE = 5,
  SPP_E_RCCL = 6
};

/* Text of the last error raised on this thread ("" if none). */
const char* sppGetLastError(void);
int sppGetVersion(void);

/* ------------------------------------------------------------------ RNG
 * numpy legacy MT19937 stream: np.random.seed(s); np.random.randint(0, high, n)
 * (index draw of rltoolkit/buffer/replay_buffer.py:234, :418).  Host-side,
 * bit-exact.  */
typedef struct sppMT19937* sppMTHandle;
sppStatus sppMTCreate(sppMTHandle* out, uint32_t seed);
sppStatus sppMTRandint(sppMTHandle h, int64_t high, int64_t n, int64_t* out_host);
sppStatus sppMTDestroy(sppMTHandle h);

/* Counter-based (Philox4x32-10) device streams for the vectorised path.
 * Normal draws by Box-Muller; uniform ints by masked rejection. */
sppStatus sppRandNormal(float* out_dev, int64_t n, uint64_t seed, uint64_t offset, void* stream);
sppStatus sppRandIndex(int64_t* out_dev, int64_t n, int64_t high, uint64_t seed, uint64_t offset,
                       void* stream);
/* Random permutation of [0, n) on the device (the shuffle of a DataLoader(shuffle=True) epoch:
 * acm/acm.py:275, acm/on_policy.py:176-190), deterministic for (seed, offset).  n < 2^20: uniform -- 64-bit
 * Philox keys (counters offset + i), stable radix sort of (key, index), out_dev [n] = the sorted indices;
 * n >= 2^20 (round 6): a keyed 6-round Feistel bijection with cycle walking (a pseudo-random permutation, one
 * O(n) launch).  scratch: device bytes >= sppRandPermScratchBytes(n).  Stream-ordered, no host synchronisation
 * (replaces torch.randperm on the device). */
int64_t sppRandPermScratchBytes(int64_t n);
sppStatus sppRandPerm(int64_t* out_dev, int64_t n, uint64_t seed, uint64_t offset, void* scratch_dev,
                      int64_t scratch_bytes, void* stream);

/* ------------------------------------------------------------------ replay ring
 * BufferAcMOffPolicy (rltoolkit/buffer/replay_buffer.py:303-401) with the
 * MetaReplayBuffer obs-index ring (:7-96): obs stored once per slot, each
 * timestep keeps (obs_idx, next_obs_idx); wrap rule Q6 reproduced exactly.
 * Storage lives in HBM, fp32 (exact: every stored value is an fp32 tensor
 * value, the reference's fp64 store round-trips it unchanged — Q5). */
typedef struct sppReplay* sppReplayHandle;
sppStatus sppReplayCreate(sppReplayHandle* out, int64_t capacity, int ob, int aout, int ac, int device);
sppStatus sppReplayDestroy(sppReplayHandle h);
/* MetaReplayBuffer.add_obs (:56-60) for E rows at once; slots returned to host. */
sppStatus sppReplayAddObs(sppReplayHandle h, const float* obs_dev /*[E][ob]*/, int E,
                          int64_t* slots_host_out /*[E]*/, void* stream);
/* add_acm_action (:332-333) + add_timestep (:65-75) + addition (:133-137), E
 * transitions applied in env order (E = 1 is the reference exactly). */
sppStatus sppReplayAddStep(sppReplayHandle h, const int64_t* prev_host, const int64_t* next_host, int E,
                           const float* act_dev /*[E][aout]*/, const float* acm_dev /*[E][ac]*/,
                           const float* rew_dev /*[E]*/, const uint8_t* done_dev /*[E]*/,
                           const uint8_t* end_dev /*[E]*/, void* stream);
/* obs_idx, ts_idx, current_len */
sppStatus sppReplayState(sppReplayHandle h, int64_t* obs_idx, int64_t* ts_idx, int64_t* len);
sppStatus sppReplayReset(sppReplayHandle h); /* reset_idx (:32-35) */
/* _sample_batch / sample_batch gather (:233-261, :385-398) for given indices,
 * reference row-major layout: obs, next_obs [B][ob], act [B][aout], rew [B],
 * done [B] int8, acm [B][ac].  Any output pointer may be NULL. */
sppStatus sppReplayGather(sppReplayHandle h, const int64_t* idx_dev, int B, float* obs, float* next_obs,
                          float* act, float* rew, int8_t* done, float* acm, void* stream);
/* update_obs_mean_std (:83-96): fp64 mean / std(ddof=0) over the live obs,
 * exact np.percentile(.., 99 / 1, linear) by radix select, running max/min.
 * Skipped (returns *updated = 0) when len <= 10.  max/min are read-modify-
 * written (first_update != 0 overwrites them).  A call on rows unchanged since
 * the last call (no AddObs / AddStep / Reset / GetView in between) reuses the
 * stored sample bracket; the result is exact either way. */
sppStatus sppReplayObsStats(sppReplayHandle h, float* mean, float* std, float* max_obs, float* min_obs,
                            int first_update, void* stream);
/* Test hook of the sample-bracketed statistics (sppReplayObsStats, sppReplayObsStatsDP1): lower the per-pass-
 * workgroup candidate-list capacity to list_cap and the per-(column, target) overflow list to ovf_cap keys (0:
 * the full capacities), so the overflow fallbacks run at small sizes.  Results stay exact at any capacity. */
sppStatus sppReplaySetObsStatsCaps(sppReplayHandle h, int list_cap, int ovf_cap);
/* Data-parallel update_obs_mean_std over the union of the ranks' replay shards
 * (SURVEY.md §8e): exact global mean / std (fp64 sums about a replicated pivot,
 * e.g. the current obs_mean) and exact global 99th / 1st percentiles (radix select
 * over all-reduced histograms).  Call with step = 0, 1, 2, ... until *done:
 *   step 0   local pass 1 -> sums[ob][2] (fp64) and hist (top byte)
 *   step k   selection with the global counts (n_global = sum of the ranks' len),
 *            then the next local byte pass -> hist
 * and all-reduce (sum) `sums` after step 0 and `hist` after every step that did
 * not set *done.  hist: sppReplayObsStatsDPHistSize(h) uint32 counters.  n_global < 2^31. */
int sppReplayObsStatsDPHistSize(sppReplayHandle h);
sppStatus sppReplayObsStatsDP(sppReplayHandle h, int step, const float* pivot /*[ob], replicated*/,
                              double* sums /*[ob][2]*/, uint32_t* hist, int64_t n_global, float* mean, float* std,
                              float* max_obs, float* min_obs, int first_update, int* done, void* stream);
/* The same statistics with ONE read of the local rows per call (sample-bracketed, like
 * sppReplayObsStats): call phase = 0 .. 6 in order and run, on the host, between them:
 *   after phase 0   all-gather `samp` across ranks (rank-major [world][ob][Sl] u32, Sl =
 *                   sppReplayObsStatsDP1SampleRows; this rank wrote slot `rank`; in place)
 *   after phase 1   all-reduce (sum) `exch` (fp64, 2*ob + 10*ob: moments, per-target counts)
 *   after 2,3,4,5   all-reduce (sum) `hist` (uint32, ob*2*2*256)
 * Phase 6 writes mean / std / max_obs / min_obs (identical on every rank).  Exact: a sample miss or an
 * overflowed candidate list selects over the raw columns in the same fixed phases.  n_global < 2^31.
 * `pivot` (replicated) may alias `mean`: phase 6 reads pivot[c] before it writes mean[c].
 * Bracket reuse: every rank may skip phase 0 and its all-gather and pass phase 1 as
 * (1 | SPP_DP1_REUSE_BRACKET) when the shards are unchanged since the previous call (the decision
 * must be the same on every rank: the host's lockstep-checked write count).  Phase 1 then keeps the
 * union bracket of that call (or recomputes it from `samp`, which holds the same union sample on every
 * rank, if this handle's bounds were overwritten since).  Any bracket gives the exact result. */
#define SPP_DP1_REUSE_BRACKET 0x100
int sppReplayObsStatsDP1SampleRows(sppReplayHandle h, int world, int64_t n_global);
sppStatus sppReplayObsStatsDP1(sppReplayHandle h, int phase, int world, int rank, const float* pivot /*[ob]*/,
                               uint32_t* samp, double* exch, uint32_t* hist, int64_t n_global, float* mean,
                               float* std, float* max_obs, float* min_obs, int first_update, void* stream);
/* Raw device pointers of the ring.  A timestep is ONE 64-B-aligned record of rec_words 32-bit words:
 *   0 obs slot, 1 next-obs slot (uint32; capacity < 2^31), 2 reward (fp32), 3 done (bit 0) | end (bit 8),
 *   rec_acm .. rec_acm + ac - 1 the ACM action, rec_act .. rec_act + aout - 1 the stored actor output (fp32);
 * a sampled transition then reads one record and two obs rows.  obs_idx repeats word 0 as a contiguous
 * int64 array (the obs statistics walk every live row through it). */
typedef struct {
  float* obs;          /* [capacity][ob]        */
  int64_t* obs_idx;    /* [capacity]            */
  uint32_t* rec;       /* [capacity][rec_words] */
  int rec_words, rec_acm, rec_act;
} sppReplayView;
/* Raw device arrays of the ring; counts as a possible write (the next ObsStats re-brackets). */
sppStatus sppReplayGetView(sppReplayHandle h, sppReplayView* out);
/* The SURVEY §8b constructor: n_envs sizes the per-step metadata ring up front; compat_mode must
 * be 1 (the reference obs-index ring with the Q6 wrap -- the only ring rltoolkit has);
 * store_fp64 must be 0 (the reference's float64 arrays only ever receive float32 values, so
 * float32 storage is exact, Q5).  Other values return SPP_E_INVALID_ARG. */
sppStatus sppReplayCreateEx(sppReplayHandle* out, int64_t capacity, int ob, int aout, int ac, int n_envs,
                            int compat_mode, int store_fp64, int device);
/* BufferAcMOffPolicy.last_rollout (replay_buffer.py:335-383) with last_end (:170-177): the last
 * complete episode is the *length timesteps first, first+1, ... (cyclic over [0, current_len))
 * ending at the last end flag at or before ts_idx - 1.  Synchronous; SPP_E_STATE if the buffer
 * holds no episode end. */
sppStatus sppReplayLastRollout(sppReplayHandle h, int64_t* first, int64_t* length, void* stream);

/* ------------------------------------------------------------------ agent */
/* SPP_ALGO_SAC: vanilla SAC (rltoolkit/algorithms/sac/sac.py:138-280), BASELINE configs[0]: no ACM,
 * the actor emits the env action (aout == ac) and feeds the critics directly. */
enum { SPP_ALGO_SAC_ACM = 1, SPP_ALGO_DDPG_ACM = 2, SPP_ALGO_SAC = 3 };
enum { /* network ids for parameter binding (SAC_AcM) */
  SPP_NET_ACTOR = 0, SPP_NET_CRITIC1 = 1, SPP_NET_CRITIC2 = 2,
  SPP_NET_CRITIC1_TARG = 3, SPP_NET_CRITIC2_TARG = 4, SPP_NET_ACM = 5,
  SPP_NET_ACTOR_TARG = 6, /* DDPG_AcM only; DDPG's single critic / target use CRITIC1 / CRITIC1_TARG */
  SPP_NET_COUNT = 7
};

typedef struct {
  int algo;                 /* SPP_ALGO_SAC_ACM (ACM = AcM 64-32) | SPP_ALGO_DDPG_ACM (ACM = BasicAcM) */
  int ob, aout, ac;         /* obs dim, actor output dim (= len(acm_ob_idx) = ob), env action dim */
  int acm_critic;           /* critics see ACM(s, denorm a) (ac) instead of denorm a (aout) */
  int min_max_denormalize;  /* memory.py:107-121 min-max vs z-score */
  int norm_closs;           /* sac_acm.py:80-84 */
  float custom_loss;        /* sac_acm.py:78-86 */
  float gamma, tau;
  float actor_lr, critic_lr, alpha_lr, acm_lr;
  float target_entropy;     /* sac.py:104-106: -env ac_dim (Q4) */
  int max_batch;            /* workspace sizing (update batch B) */
  int mlp_bf16;             /* 1: MLP layers on bf16 MFMA (v_mfma_f32_32x32x16_bf16), fp32 accumulation, epilogues,
                               targets, losses and Adam (BASELINE configs[4]); SAC_AcM Hopper / Ant dims */
} sppAgentConfig;

typedef struct sppAgent* sppAgentHandle;
sppStatus sppAgentCreate(sppAgentHandle* out, const sppAgentConfig* cfg, int device);
sppStatus sppAgentDestroy(sppAgentHandle h);
/* Number of float32 parameters of network `net` (state_dict order). */
sppStatus sppAgentNetSize(sppAgentHandle h, int net, int64_t* n);
/* Bind caller-owned flat buffers.  grad / exp_avg / exp_avg_sq may be NULL for
 * target and frozen networks. */
sppStatus sppAgentBindNet(sppAgentHandle h, int net, float* params, float* grads, float* exp_avg,
                          float* exp_avg_sq);
/* Constant vectors: actor_ac_lim [aout] (acm.py:102-108), acm ac_lim [ac]. Host arrays, copied. */
sppStatus sppAgentSetLimits(sppAgentHandle h, const float* actor_lim_host, const float* acm_lim_host);
/* Replay normalizer (caller-owned device vectors [ob]; NULL allowed for unused pair). */
sppStatus sppAgentBindNormalizer(sppAgentHandle h, const float* min_obs, const float* max_obs,
                                 const float* obs_mean, const float* obs_std);
/* Temperature state: alpha_state_dev = double[4] {log_alpha, exp_avg, exp_avg_sq, alpha};
 * alpha_f32_dev = float[1] (the python float self.alpha, sac_acm.py:159). */
sppStatus sppAgentBindAlpha(sppAgentHandle h, double* alpha_state_dev, float* alpha_f32_dev);
/* Adam step counters (host). */
sppStatus sppAgentSetSteps(sppAgentHandle h, int64_t actor_step, int64_t critic_step, int64_t alpha_step,
                           int64_t acm_step);
/* Learning rates (torch.optim.lr_scheduler.StepLR of the ACM, acm.py:176-183); < 0 keeps the value. */
sppStatus sppAgentSetLr(sppAgentHandle h, float actor_lr, float critic_lr, float alpha_lr, float acm_lr);
sppStatus sppAgentGetSteps(sppAgentHandle h, int64_t* steps4);

/* Update batch in the reference row-major layout (sample_batch output). */
typedef struct {
  int B;
  const float* obs;       /* [B][ob]   */
  const float* next_obs;  /* [B][ob]   */
  const float* action;    /* [B][aout] (unused when acm_critic) */
  const float* reward;    /* [B]       */
  const int8_t* done;     /* [B]       */
  const float* acm_action;/* [B][ac]   */
} sppBatch;

/* Loss vector written by the update (device float[8]):
 * {critic_1, critic_2, actor, sac, dist, alpha_loss, alpha, 0}. */
#define SPP_NUM_LOSSES 8

/* SAC_AcM.update (rltoolkit/acm/off_policy/sac_acm.py:89-162): one full grad
 * step.  eps_next / eps_cur [B][aout] are the standard-normal draws of the two
 * rsample calls (sac_acm.py:44, :137); NULL -> drawn on device from (seed, step). */
sppStatus sppSacAcmUpdate(sppAgentHandle h, const sppBatch* batch, const float* eps_next, const float* eps_cur,
                          float* losses_dev, void* stream);
/* The same step split at its two exchange points for data-parallel training:
 * grads -> (caller all-reduces the flat grad buffers, averaging) -> apply.
 * batch == NULL / eps == NULL use the staged batch / staged eps (see below).
 * ActorGrads also writes the temperature-gradient operand mean(-logpi - H)
 * into the bound alpha-grad scalar, which the caller all-reduces with the
 * actor gradients; ActorApply consumes it. */
sppStatus sppSacAcmCriticGrads(sppAgentHandle h, const sppBatch* batch, const float* eps_next,
                               float* losses_dev, void* stream);
sppStatus sppSacAcmCriticApply(sppAgentHandle h, void* stream);
sppStatus sppSacAcmActorGrads(sppAgentHandle h, const float* eps_cur, float* losses_dev, void* stream);
sppStatus sppSacAcmActorApply(sppAgentHandle h, float* losses_dev, void* stream);
/* Caller-owned device float[1] receiving mean(-logpi - H) (sac.py:214-216). */
sppStatus sppAgentBindAlphaGrad(sppAgentHandle h, float* alpha_grad_dev);
/* Draw both rsample eps tensors of the staged batch on device (Philox, (seed, counter)). */
sppStatus sppSacAcmDrawEps(sppAgentHandle h, uint64_t seed, uint64_t counter, void* stream);
/* Test hook: copy the staged eps (which = 0: next-state draw, 1: current-state draw) to a
 * caller-owned row-major [B][aout] device buffer, so parity tests can replay the exact
 * device draws through the oracle. */
sppStatus sppAgentReadEps(sppAgentHandle h, int which, float* out_dev, void* stream);
/* Test hooks on the packed weight images the phase kernels read (no reference counterpart: the
 * reference reads nn.Linear weights directly).  ImageCount: how many images hold parameters of
 * `net`; UnpackImage: write image i back into a caller-owned device buffer laid out like the
 * net's flat parameters (every position the image covers; the rest untouched).  bf16 agents:
 * the values are the bf16 image entries, which must equal RNE(fp32 parameter) after each step. */
sppStatus sppAgentImageCount(sppAgentHandle h, int net, int* n_out);
sppStatus sppAgentUnpackImage(sppAgentHandle h, int net, int i, float* out_dev, void* stream);
/* Fused replay sample + gather into the agent's staging area (device indices). */
sppStatus sppAgentStageFromReplay(sppAgentHandle h, sppReplayHandle r, const int64_t* idx_dev, int B,
                                  void* stream);
/* The rest of sample_batch / make_update on the staged batch, in place:
 *   normalize          obs and next_obs through the bound normaliser (ReplayBuffer._sample_batch with
 *                      obs_norm, rltoolkit/buffer/replay_buffer.py:247-249): 1 = min-max or z-score per the
 *                      agent's min_max_denormalize (memory.py:76-88), 2 = z-score with the bound mean / std
 *                      whatever that flag (vanilla SAC's plain ReplayBuffer, whose MemoryMeta keeps
 *                      min_max_denormalize False: sac.py via ddpg.py:107-115)
 *   act_from_next_obs  the critic's action operand := the (normalised) next obs
 *                      (DDPG_AcM.make_unbiased_update, rltoolkit/acm/off_policy/ddpg_acm.py:59-73:
 *                      update(action=next_obs)); needs acm_critic = 0 and aout == ob. */
sppStatus sppAgentStagePost(sppAgentHandle h, int normalize, int act_from_next_obs, void* stream);
/* Update on the staged batch (after sppAgentStageFromReplay), eps drawn on
 * device from (seed, counter). */
sppStatus sppSacAcmUpdateStaged(sppAgentHandle h, uint64_t seed, uint64_t counter, float* losses_dev,
                                void* stream);

/* DDPG_AcM.update (rltoolkit/acm/off_policy/ddpg_acm.py:147-201): critic step on
 * y = r + gamma (1-d) Q_targ(s', BasicAcM(s', denorm mu_targ(s'))), actor step on
 * -Q(s, BasicAcM(s, denorm mu(s))).mean() + custom_loss * MSE, then polyak of the critic
 * AND actor targets (ddpg.py:273-284).  Losses (device float[8]): {critic, actor, ddpg, dist}.
 * Split at the same exchange points as SAC_AcM for data-parallel use; batch == NULL
 * uses the staged batch (sppAgentStageFromReplay). */
sppStatus sppDdpgAcmUpdate(sppAgentHandle h, const sppBatch* batch, float* losses_dev, void* stream);
sppStatus sppDdpgAcmCriticGrads(sppAgentHandle h, const sppBatch* batch, float* losses_dev, void* stream);
sppStatus sppDdpgAcmCriticApply(sppAgentHandle h, void* stream);
sppStatus sppDdpgAcmActorGrads(sppAgentHandle h, float* losses_dev, void* stream);
sppStatus sppDdpgAcmActorApply(sppAgentHandle h, void* stream);

/* ------------------------------------------------------------------ data-parallel exchange (§8e)
 * RCCL communicator for C/C++ hosts without torch.distributed (librccl resolved at run time).
 * Rank 0 fills a SPP_COMM_ID_BYTES unique id, the host ships it to every rank by any channel,
 * each rank calls sppCommInitRank on its device.  Replaces torch.distributed.all_reduce in the
 * Python DP path (spprl/dp.py); on ROCm both are RCCL over xGMI. */
#define SPP_COMM_ID_BYTES 128
sppStatus sppCommGetUniqueId(void* uid_out);
sppStatus sppCommInitRank(void** comm_out, int nranks, const void* uid, int rank, int device);
sppStatus sppCommDestroy(void* comm);
/* In-place average over the communicator's `world` ranks (ncclSum then x 1/world) of one gradient
 * bucket, stream-ordered between the *Grads and *Apply halves of an update:
 *   SPP_BUCKET_CRITIC  critic_1 (+ critic_2) grads          (after *CriticGrads)
 *   SPP_BUCKET_ACTOR   actor grads (+ the SAC alpha operand)  (after *ActorGrads)
 *   SPP_BUCKET_ACM     ACM grads                            (after sppAcmRegressGrads)
 *   SPP_BUCKET_ALL     all of them. */
enum { SPP_BUCKET_CRITIC = 0, SPP_BUCKET_ACTOR = 1, SPP_BUCKET_ACM = 2, SPP_BUCKET_ALL = 3 };
sppStatus sppAllReduceGrads(sppAgentHandle h, int bucket, int world, void* rccl_comm, void* stream);
/* In-place sum over the communicator of `count` elements (dtype 0 fp32, 1 fp64, 2 int32, 3 int64,
 * 4 uint32): the obs-statistics sums / counts of sppReplayObsStatsDP and the global row count. */
sppStatus sppCommAllReduceSum(void* rccl_comm, void* buf_dev, int64_t count, int dtype, void* stream);
/* Rank-major all-gather of `bytes` bytes per rank into recv (in place when send = recv + rank*bytes). */
sppStatus sppCommAllGather(void* rccl_comm, const void* send_dev, void* recv_dev, int64_t bytes, void* stream);

/* AcMTrainer.batch_update (rltoolkit/acm/acm.py:246-258): x [B][2ob], y [B][ac]
 * -> MSE loss (device float) and one Adam step on the bound ACM net. */
sppStatus sppAcmRegressStep(sppAgentHandle h, const float* x, const float* y, int B, float* loss_dev,
                            void* stream);
/* The same split for data-parallel use: grads (into the bound ACM grad buffer) / apply. */
sppStatus sppAcmRegressGrads(sppAgentHandle h, const float* x, const float* y, int B, float* loss_dev,
                             void* stream);
sppStatus sppAcmRegressApply(sppAgentHandle h, void* stream);
/* ACM regression batch straight from the ring (rbuffer_sample_acm, replay_buffer.py:404-430 +
 * acm_cat, acm.py:260-264): x = [obs | next_obs] [B][2ob], y = acm action [B][ac]. */
/* nsteps sequential AcM regression steps (acm.py:246-258 each: MSE + Adam at acm_lr) in ONE
 * launch: step k's batch = rows [k*bs, k*bs + bs) of x [nsteps*bs][2ob] / y [nsteps*bs][ac]
 * (acm_cat inputs and targets, e.g. from sppReplayGatherAcm), bs <= 32768.  Parameters stay in
 * LDS, moments in registers (update_acm epochs, update_acm_batches).  loss_sum += sum of the
 * steps' batch losses.  AcM agents (SAC_AcM / PPO_AcM) only.  bs <= 64: one workgroup; larger batches
 * spread each step over ceil(bs / 64) workgroups (all co-resident: bs <= sppAcmSgdMaxBatch) that sum
 * the step's gradient in a fixed order (deterministic): a reduce-scatter of per-workgroup gradient slabs,
 * Adam on each workgroup's shard, the new parameters gathered back (two arrival barriers per step). */
sppStatus sppAcmSgd(sppAgentHandle h, const float* x_dev, const float* y_dev, int nsteps, int bs, float* loss_sum,
                    void* stream);
/* One update_acm epoch (acm.py:270-297: DataLoader(batch_size=bs, shuffle=True), drop_last=False) in ONE
 * launch: ceil(nrows / bs) steps over rows [0, nrows) of x / y (gathered through the epoch's permutation),
 * the last step over the nrows % bs ragged remainder when there is one (its loss is that batch's mean, as
 * the reference's last DataLoader batch).  Otherwise as sppAcmSgd. */
sppStatus sppAcmSgdEpoch(sppAgentHandle h, const float* x_dev, const float* y_dev, int nrows, int bs,
                         float* loss_sum, void* stream);
/* Synchronous: 1 if a multi-workgroup sppAcmSgd launch timed out waiting for its workgroups (its
 * results are then invalid), else 0. */
sppStatus sppAcmSgdStatus(sppAgentHandle h, int* timed_out_host);
/* Stream-ordered form: enqueues a copy of the timeout flag into *timed_out_pinned (pinned host memory,
 * read after the stream has passed this point); 0 is written when no multi-workgroup launch ran. */
sppStatus sppAcmSgdStatusAsync(sppAgentHandle h, int* timed_out_pinned, void* stream);
/* Largest bs sppAcmSgd accepts on this device for this agent: every workgroup of a step must be resident
 * at once (the arrival barrier), so min(32768, 64 x occupancy x CUs).  Larger batches: SPP_E_SHAPE. */
int sppAcmSgdMaxBatch(sppAgentHandle h);
/* Co-resident workgroups (one per CU) one sppAcmSgd / sppAcmSgdEpoch step of bs rows runs on: 1 for bs <= 64,
 * else max(2, ceil(bs / 64)) workgroups of 4 waves (17 at bs = 1,049); 0 for handles without the AcM kernel.
 * (A library built with -DSPP_ACM_WV=8, the 8-wave A/B variant, returns max(2, ceil(bs / 128)).) */
int sppAcmSgdWorkgroups(sppAgentHandle h, int bs);
sppStatus sppReplayGatherAcm(sppReplayHandle h, const int64_t* idx_dev, int B, float* x, float* y, void* stream);
/* AcMTrainer(acm_ob_idx=...) (acm.py:94-99, 148, 260-264): sppReplayGatherAcm then writes
 * x = [obs[:, cols] | next_obs[:, cols]].  n = ob index entries (a permutation or any list of ob columns, each
 * in [0, ob)), or n = 0 for the identity (the default).  Lists of another length are refused: the reference's
 * AcM takes ob + n inputs (acm.py:148) while acm_cat gives it 2n, so only n = ob runs there.  Synchronous. */
sppStatus sppReplaySetAcmColumns(sppReplayHandle h, const int* cols_host, int n);

/* Per-kernel device timing (HIP events on the launch stream), for measurement:
 * kinds 0 critic-phase, 1 actor-phase, 2 weight-grad GEMMs, 3 Adam, 4 ACM regression.
 * GetTiming synchronises on the recorded events, returns total ms and launch
 * counts per kind, and clears them. */
sppStatus sppAgentSetTiming(sppAgentHandle h, int enable);
sppStatus sppAgentGetTiming(sppAgentHandle h, double* ms_out /*[5]*/, int64_t* count_out /*[5]*/);

/* Rollout action (rltoolkit/acm/off_policy/ddpg_acm.py:40-50 noise_action +
 * off_policy.py:50-54 initial_act + :89-106 process_action):
 *   mode 0 random : a = lim * eps                      (initial_act)
 *   mode 1 noisy  : a = clip(tanh(mu + sigma*eps)*lim + act_noise*lim*noise, +-1.1 lim)
 *   mode 2 det    : a = clip(tanh(mu)*lim, +-1.1 lim)
 *   mode 3 given  : a = eps (the caller's action; on-policy process_action, acm/on_policy.py:32-50)
 * then a_d = denormalize(a) if denormalize_actor_out, env action = ACM(cat(obs, a_d)).
 * target_state_out receives a_d (what the buffer stores as `action`). */
sppStatus sppPolicyAct(sppAgentHandle h, const float* obs /*[E][ob]*/, int E, const float* eps /*[E][aout]*/,
                       const float* noise /*[E][aout]*/, float act_noise, int mode, int denormalize_actor_out,
                       float* target_state_out /*[E][aout]*/, float* env_action_out /*[E][ac]*/, void* stream);

/* Synthetic fixed-shape env (SURVEY.md Appendix A SynthEnv), E instances in
 * lockstep on device: s' = tanh(A s) + 0.1*resize(a, ob); r = -|a|^2 + s'[0]. */
sppStatus sppSynthEnvStep(const float* A /*[ob][ob]*/, const float* obs /*[E][ob]*/, const float* action /*[E][ac]*/,
                          int E, int ob, int ac, float* next_obs, float* reward, void* stream);

/* gym Box.sample() stand-in for the pre-train collector (rltoolkit/acm/acm.py:187-196,
 * off_policy.py:56-87): out[j] ~ U[lo[j % period], hi[j % period]). */
sppStatus sppRandUniform(float* out_dev, int64_t n, const float* lo_dev, const float* hi_dev, int period,
                         uint64_t seed, uint64_t offset, void* stream);
/* Episode returns of E vectorized envs (StatsLogger.calc_running_return input,
 * rltoolkit/stats_logger.py:19-26; Memory.average_returns_per_rollout):
 * ep_ret[e] += rew[e]; where end[e], sums[0] += ep_ret[e], sums[1] += 1 (fp64) and
 * ep_ret[e] = 0.  end may be NULL. */
sppStatus sppEpisodeAccum(const float* rew, const uint8_t* end, int E, float* ep_ret, double* sums, void* stream);
/* SynthEnv.reset for the rows with mask[e] != 0 (all rows when mask is NULL). */
sppStatus sppSynthEnvReset(float* obs /*[E][ob]*/, const uint8_t* mask, int E, int ob, uint64_t seed,
                           uint64_t offset, void* stream);

/* MemoryMeta.normalize (inverse = 0) / denormalize (inverse = 1), rltoolkit/buffer/memory.py:76-127,
 * elementwise over x[rows][ob]; min_max selects (lo, hi) else (mean, std). out may alias x. */
sppStatus sppObsNormalize(const float* x, int64_t rows, int ob, const float* lo, const float* hi, const float* mean,
                          const float* std, int min_max, int inverse, float* out, void* stream);

/* ------------------------------------------------------------------ PPO path
 * PPO.calculate_q_val + calculate_gae (rltoolkit/algorithms/a2c/a2c.py:247-265,
 * algorithms/ppo/ppo.py:117-150) over E independent streams of T steps, time-major
 * [T][E] (E = 1 is the reference's single rollout buffer).  Inputs are the critic's
 * V(s), V(s') and the buffer's rewards / done / end (truncation) flags.
 *   q_out[t][e] = r + gamma (1 - d) V(s')          (optional, may be NULL)
 *   adv[t][e]   = reverse GAE with done reset and end bootstrap V(s') (quirk Q10)
 * mode 0: one lane per stream, the reference's float32 operation order (bit-exact);
 * mode 1: reverse affine scan with wavefront shuffles, one workgroup per stream
 *         (for few long streams; fp32 reassociation, not bit-exact);
 * mode -1: 0 when E >= 64, else 1. */
sppStatus sppGaeScan(const float* rew, const float* v, const float* v_next, const uint8_t* done,
                     const uint8_t* end, int64_t T, int64_t E, double gamma, double lam, int mode, float* q_out,
                     float* adv, void* stream);
/* PPO._clip_loss (ppo.py:194-204) and utils.kl_divergence (utils.py:48-59) on a
 * minibatch of B: out2[0] = -mean(min(r A, clip(r, 1-eps, 1+eps) A)), r = exp(lp_new - lp_old);
 * out2[1] = mean(lp_old - lp_new).  grad (optional) = d out2[0] / d lp_new with torch's
 * minimum (ties split) and clamp (inclusive bounds) backward rules. */
sppStatus sppPpoClipLoss(const float* lp_old, const float* lp_new, const float* adv, int B, float eps, float* grad,
                         float* out2, void* stream);
/* AdvantageDataset normalisation (algorithms/ppo/advantage_dataset.py:8-12):
 * out = (adv - mean) / (std(ddof=1) + 1.2e-7).  out may alias adv. */
sppStatus sppAdvNormalize(const float* adv, int64_t n, float* out, void* stream);
/* Data-parallel form: sppAdvSums writes the local fp64 {sum, sum of squares};
 * the caller all-reduces them (and n) and sppAdvNormalizeGlobal normalises the local shard with
 * the global moments (std ddof = 1, + 1.2e-7). */
sppStatus sppAdvSums(const float* adv, int64_t n, double* sums2, void* stream);
sppStatus sppAdvNormalizeGlobal(const float* adv, int64_t n_local, const double* sums2, int64_t n_global, float* out,
                                void* stream);

/* ------------------------------------------------------------------ on-policy nets (A2C / PPO)
 * The 64-wide tanh MLPs of rltoolkit/basic_model.py:7-76 used by A2C / PPO(_AcM):
 *   net 0 = Actor (continuous): log_scale [aout], fc1 ob->64, fc2 64->64, fc3 64->aout,
 *           mu = tanh(fc3) * lim, policy Independent(Normal(mu, exp(log_scale)))
 *   net 1 = Critic: fc1 ob->64, fc2 64->64, fc3 64->1
 * Flat buffers in state_dict order; inputs are the buffer's normalised obs, row-major. */
typedef struct sppOnPolicy* sppOnPolicyHandle;
typedef struct {
  int ob, aout;
  float actor_lr, critic_lr;   /* config.A_LR / C_LR */
  float ppo_epsilon;           /* PPO clip */
  float entropy_coef;          /* PPO_ENTROPY */
  int max_batch;               /* largest N of any call */
} sppOnPolicyConfig;
sppStatus sppOnpCreate(sppOnPolicyHandle* out, const sppOnPolicyConfig* cfg, int device);
sppStatus sppOnpDestroy(sppOnPolicyHandle h);
sppStatus sppOnpNetSize(sppOnPolicyHandle h, int net, int64_t* n);
sppStatus sppOnpBindNet(sppOnPolicyHandle h, int net, float* params, float* grads, float* exp_avg, float* exp_avg_sq);
sppStatus sppOnpSetLimits(sppOnPolicyHandle h, const float* actor_lim_host /*[aout]*/);
/* critic(x) -> v [N] (calculate_q_val / calculate_gae inputs, a2c.py:257-265, ppo.py:131). */
sppStatus sppOnpValue(sppOnPolicyHandle h, const float* x, int N, float* v, void* stream);
/* One critic step of A2C.update_critic (a2c.py:209-219): loss = 0.5 * mean((q - V(x))^2)
 * (device float[1]); grads into the critic buffer; Apply = Adam(critic_lr). */
sppStatus sppOnpCriticGrads(sppOnPolicyHandle h, const float* x, const float* q, int N, float* loss, void* stream);
sppStatus sppOnpCriticApply(sppOnPolicyHandle h, void* stream);
/* One PPO actor minibatch step (ppo.py:174-190 / on_policy.py:189-205): logp of the stored
 * actions under the current policy, loss = clip_loss - entropy_coef * entropy; grads into the
 * actor buffer (log_scale included).  out4 = {actor (clip) loss, KL = mean(lp_old - lp_new),
 * dist = MSE(actions, next_obs) (no gradient, as in the reference; next_obs may be NULL), entropy}. */
sppStatus sppOnpActorGrads(sppOnPolicyHandle h, const float* x, const float* act, const float* lp_old,
                           const float* adv, const float* next_obs, int N, float* out4, void* stream);
sppStatus sppOnpActorApply(sppOnPolicyHandle h, void* stream);
/* PPO_AcM.update_actor_acm / PPO.update_actor minibatch epoch (rltoolkit/acm/on_policy.py:176-207,
 * algorithms/ppo/ppo.py:174-190) in ONE launch: nsteps sequential Adam steps of the Gaussian actor on the
 * clip loss - entropy_coef * entropy over nsteps = ceil(nrows / bs) minibatches: step k's minibatch = rows
 * idx[k*bs .. min(k*bs + bs, nrows)) (the epoch's permutation, DataLoader(shuffle=True): the last minibatch
 * is the ragged remainder) of x [n][ob] (normalised obs), act [n][aout], lp_old [n], adv [n]
 * (normalised advantages) and next_obs [n][aout] (the dist loss, data only; NULL: 0).  out4 [nsteps][4]:
 * each step's actor loss, KL (mean lp_old - lp_new before the step), dist MSE, entropy.  Parameters stay in
 * LDS for the launch; bs > 64 spreads each step over ceil(bs / 64) co-resident workgroups whose gradients
 * are summed in a fixed order (deterministic).  Data-parallel PPO_AcM runs it on every rank over the all-gathered
 * union batch (replicated, no per-step exchange; sppOnpActorGrads / Apply + an all-reduce remain for callers
 * that shard the minibatch).  Instantiated for (ob, aout) = (17, 17), (11, 11). */
sppStatus sppOnpActorEpoch(sppOnPolicyHandle h, const float* x, const float* act, const float* lp_old,
                           const float* adv, const float* next_obs, const int64_t* idx, int nrows, int bs,
                           float* out4, void* stream);
/* Largest bs sppOnpActorEpoch accepts on this device (0: no instantiation for the handle's dims). */
int sppOnpActorEpochMaxBatch(sppOnPolicyHandle h);
/* The data-parallel form of one clip-loss minibatch step (replaces sppOnpActorGrads on ranks that shard the
 * minibatch; round 6): the sppOnpActorEpoch kernel run for ONE step of the N rows idx[0 .. N) with its gradient
 * (clip loss - entropy_coef * entropy, log_scale included, summed over the workgroups in a fixed order) written
 * times grad_scale (1 / ranks) to the actor's bound gradient buffer instead of applied; out4 = {actor loss, KL, dist,
 * entropy} of the step, times grad_scale too.  The caller sum-all-reduces the gradient and out4 and calls
 * sppOnpActorApply.  N <= sppOnpActorEpochMaxBatch. */
sppStatus sppOnpActorStepGrads(sppOnPolicyHandle h, const float* x, const float* act, const float* lp_old,
                               const float* adv, const float* next_obs, const int64_t* idx, int N, float* out4,
                               float grad_scale, void* stream);
/* Synchronous: 1 if a multi-workgroup sppOnpActorEpoch / sppOnpCriticSteps launch timed out at an arrival
 * barrier, else 0. */
sppStatus sppOnpActorEpochStatus(sppOnPolicyHandle h, int* timed_out_host);
/* Stream-ordered form (the product path: PPO_AcM.update_critic / update_actor, acm/on_policy.py:164-216,
 * a2c.py:186-225): enqueues a copy of the handle's sticky timeout flag into *timed_out_pinned (pinned host
 * memory, read once the stream has passed this point); 0 is written when no multi-workgroup launch ran. */
sppStatus sppOnpSyncStatusAsync(sppOnPolicyHandle h, int* timed_out_pinned, void* stream);
/* Test hook (no reference counterpart): polls before an arrival wait of any persistent SGD launch
 * (sppAcmSgd*, sppOnpActorEpoch, sppOnpCriticSteps) times out; 0 restores the default (~0.2 s).  A negative
 * value makes every wait give up at once (a co-residency miss, deterministically): how the tests force the
 * timeout path. */
sppStatus sppSetSgdSpinLimit(int polls);
/* Tuning knob of the multi-workgroup AcM SGD (sppAcmSgd / sppAcmSgdEpoch; process-wide): each workgroup takes
 * `passes` 64-row passes per step, so a step of bs rows runs on max(2, ceil(bs / (64 passes))) workgroups that
 * meet at its two hand-offs (0 or 1: one pass, the default).  Results are the same up to the gradient's
 * summation order. */
sppStatus sppSetAcmSgdPasses(int passes);
/* A2C.update_critic's inner loop (rltoolkit/algorithms/a2c/a2c.py:186-225): nsteps sequential full-batch
 * steps of 0.5 * mean((q - V(x))^2) + Adam at critic_lr on the same N rows (x [N][ob] normalised obs, q [N]
 * targets), in ONE launch: every workgroup runs ceil(rows / 64) passes of its share of the N rows, the
 * gradient is summed over the workgroups in a fixed order (deterministic), parameters stay in LDS.
 * loss_sum += sum over the steps of each step's loss.  Data-parallel PPO_AcM runs it on every rank over the
 * all-gathered union batch (replicated; sppOnpCriticGrads / Apply + an all-reduce remain for callers that shard
 * the batch).  N <= sppOnpCriticStepsMaxBatch (up to 64 passes of 64 rows per workgroup); ob 17 and 11. */
sppStatus sppOnpCriticSteps(sppOnPolicyHandle h, const float* x, const float* q, int N, int nsteps, float* loss_sum,
                            void* stream);
int sppOnpCriticStepsMaxBatch(sppOnPolicyHandle h);
/* The data-parallel form of one critic step (replaces sppOnpCriticGrads on ranks that shard the batch; round 6):
 * the same persistent kernel as sppOnpCriticSteps run for ONE step with its gradient (0.5 * mean((q - V(x))^2),
 * summed over the workgroups in a fixed order) written times grad_scale (1 / ranks) to the critic's bound gradient
 * buffer instead of applied; loss (device float[1], zeroed by the caller) += the step's (unscaled) loss.  The caller
 * sum-all-reduces the gradient and calls sppOnpCriticApply.  N <= sppOnpCriticStepsMaxBatch; ob 17 and 11. */
sppStatus sppOnpCriticStepGrads(sppOnPolicyHandle h, const float* x, const float* q, int N, float* loss,
                                float grad_scale, void* stream);
/* Leave n CUs of the device to a persistent launch of n workgroups running concurrently on another stream
 * (the PPO_AcM ACM epochs beside update(mem); every k_mlp_sgd workgroup fills a CU's LDS):
 * sppOnpCriticSteps / sppOnpActorEpoch size their grids from the co-resident capacity minus n x their own
 * per-CU occupancy, so both grids stay resident at once.  0 restores the whole device. */
sppStatus sppOnpReserveWorkgroups(sppOnPolicyHandle h, int n);
/* Actor.act (basic_model.py:32-51) continuous: a = mu + exp(log_scale) * eps (eps NULL:
 * deterministic mu), logp = Independent(Normal).log_prob(a). */
sppStatus sppOnpAct(sppOnPolicyHandle h, const float* x, int N, const float* eps, float* act_out, float* logp_out,
                    void* stream);

/* Debug / layout check: y = act(x W^T + b) through the MFMA register-tile path.
 * x [B][K], W [N][K], b [N], y [B][N]; act 0 none, 1 relu, 2 tanh. */
sppStatus sppDebugDense(const float* x, const float* W, const float* b, float* y, int B, int K, int N, int act,
                        void* stream);

/* Profiling builds only (-DSPP_PROF): per-region s_memtime totals of the phase kernels. */
sppStatus sppDebugReadProf(unsigned long long* out64 /*[64]*/, int reset);

#ifdef __cplusplus
}
#endif
#endif /* SPPRL_H */
