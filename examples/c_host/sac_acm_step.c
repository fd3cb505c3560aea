/* A C host of the SAC_AcM hot path through the C-ABI alone (include/spprl.h; no Python, no torch):
 * the state a host would hold for rltoolkit's SAC_AcM (acm/off_policy/sac_acm.py:89-162) -- flat parameter,
 * gradient and Adam buffers per network, the temperature, the normaliser -- bound to an agent handle; a replay
 * ring (BufferAcMOffPolicy, buffer/replay_buffer.py:303-401) filled step by step in env order; then one
 * device-sampled grad step (make_update's sample_batch + update: sppAgentStageFromReplay, sppAgentStagePost,
 * sppSacAcmUpdateStaged).
 *
 *   sac_acm_step IN OUT
 *
 * IN (little-endian, written by tests/test_gpu_c_host.py from a Python SAC_AcM's freshly built state):
 *   int32  ob aout ac acm_critic min_max norm_closs max_batch E T B capacity normalize
 *   float  custom_loss gamma tau actor_lr critic_lr alpha_lr acm_lr target_entropy
 *   per network 0..5 (SPP_NET_ACTOR .. SPP_NET_ACM): int64 n, float[n] parameters
 *   float  actor_lim[aout] acm_lim[ac]; double alpha_state[4]; float alpha
 *   float  min_obs[ob] max_obs[ob] obs_mean[ob] obs_std[ob]
 *   float  obs0[E][ob]; per step t < T: obs[E][ob] act[E][aout] acm[E][ac] rew[E], uint8 done[E] end[E]
 *   int64  idx[B]; uint64 seed counter
 * OUT: float losses[SPP_NUM_LOSSES]; per network 0..5 its parameters after the step; double alpha_state[4].
 * Exit status 0 on success; every C-ABI error is printed with sppGetLastError(). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "spprl.h"

/* the four HIP runtime calls a host needs for its own buffers (libamdhip64) */
typedef int hipError_t;
extern hipError_t hipMalloc(void** ptr, size_t size);
extern hipError_t hipFree(void* ptr);
extern hipError_t hipMemcpy(void* dst, const void* src, size_t size, int kind); /* 1: H2D, 2: D2H */
extern hipError_t hipMemset(void* ptr, int value, size_t size);
extern hipError_t hipDeviceSynchronize(void);

#define H2D 1
#define D2H 2
#define NNET 6

static void die(const char* what) {
  fprintf(stderr, "sac_acm_step: %s\n", what);
  exit(1);
}
#define CK(call)                                                                 \
  do {                                                                           \
    sppStatus s_ = (call);                                                       \
    if (s_ != SPP_OK) {                                                          \
      fprintf(stderr, "sac_acm_step: %s -> %d: %s\n", #call, (int)s_, sppGetLastError()); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)
#define HK(call)                                     \
  do {                                               \
    if ((call) != 0) die(#call " failed");           \
  } while (0)

static FILE* fin;
static void rd(void* p, size_t bytes) {
  if (fread(p, 1, bytes, fin) != bytes) die("short input");
}
static void* rd_host(size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (!p) die("malloc");
  rd(p, bytes);
  return p;
}
static void* dev_zero(size_t bytes) {
  void* p = NULL;
  HK(hipMalloc(&p, bytes));
  HK(hipMemset(p, 0, bytes));
  return p;
}
static void* dev_from(const void* host, size_t bytes) {
  void* p = NULL;
  HK(hipMalloc(&p, bytes));
  HK(hipMemcpy(p, host, bytes, H2D));
  return p;
}
static void* dev_read(size_t bytes) {
  void* h = rd_host(bytes);
  void* d = dev_from(h, bytes);
  free(h);
  return d;
}

int main(int argc, char** argv) {
  if (argc != 3) die("usage: sac_acm_step IN OUT");
  fin = fopen(argv[1], "rb");
  if (!fin) die("cannot open IN");
  int32_t hi[12];
  float hf[8];
  rd(hi, sizeof hi);
  rd(hf, sizeof hf);
  const int ob = hi[0], aout = hi[1], ac = hi[2], E = hi[7], T = hi[8], B = hi[9], normalize = hi[11];
  const int64_t capacity = hi[10];

  sppAgentConfig cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.algo = SPP_ALGO_SAC_ACM;
  cfg.ob = ob, cfg.aout = aout, cfg.ac = ac;
  cfg.acm_critic = hi[3], cfg.min_max_denormalize = hi[4], cfg.norm_closs = hi[5];
  cfg.custom_loss = hf[0], cfg.gamma = hf[1], cfg.tau = hf[2];
  cfg.actor_lr = hf[3], cfg.critic_lr = hf[4], cfg.alpha_lr = hf[5], cfg.acm_lr = hf[6];
  cfg.target_entropy = hf[7];
  cfg.max_batch = hi[6];
  sppAgentHandle ag;
  CK(sppAgentCreate(&ag, &cfg, 0));

  /* parameters of every network; gradients and Adam moments of the trained ones (sac_acm.py:115-131) */
  float* params[NNET];
  int64_t sizes[NNET];
  for (int net = 0; net < NNET; ++net) {
    int64_t n = 0, m = 0;
    rd(&n, sizeof n);
    CK(sppAgentNetSize(ag, net, &m));
    if (m != n) die("network size mismatch");
    sizes[net] = n;
    params[net] = (float*)dev_read((size_t)n * 4);
    const int trained = net == SPP_NET_ACTOR || net == SPP_NET_CRITIC1 || net == SPP_NET_CRITIC2 || net == SPP_NET_ACM;
    float* g = trained ? (float*)dev_zero((size_t)n * 4) : NULL;
    float* m1 = trained ? (float*)dev_zero((size_t)n * 4) : NULL;
    float* m2 = trained ? (float*)dev_zero((size_t)n * 4) : NULL;
    CK(sppAgentBindNet(ag, net, params[net], g, m1, m2));
  }
  float* alim = (float*)rd_host((size_t)aout * 4);
  float* mlim = (float*)rd_host((size_t)ac * 4);
  CK(sppAgentSetLimits(ag, alim, mlim));
  double* alpha_state = (double*)dev_read(4 * sizeof(double));
  float* alpha_f32 = (float*)dev_read(sizeof(float));
  float* alpha_grad = (float*)dev_zero(sizeof(float));
  CK(sppAgentBindAlpha(ag, alpha_state, alpha_f32));
  CK(sppAgentBindAlphaGrad(ag, alpha_grad));
  float* norm[4];
  for (int k = 0; k < 4; ++k) norm[k] = (float*)dev_read((size_t)ob * 4);
  CK(sppAgentBindNormalizer(ag, norm[0], norm[1], norm[2], norm[3]));

  /* the replay ring, one vector step at a time in env order (add_obs, add_acm_action, add_timestep) */
  sppReplayHandle rb;
  CK(sppReplayCreateEx(&rb, capacity, ob, aout, ac, E, 1, 0, 0));
  int64_t* prev = (int64_t*)malloc((size_t)E * 8);
  int64_t* next = (int64_t*)malloc((size_t)E * 8);
  float* obs = (float*)dev_read((size_t)E * ob * 4);
  CK(sppReplayAddObs(rb, obs, E, prev, NULL));
  HK(hipFree(obs));
  for (int t = 0; t < T; ++t) {
    float* o = (float*)dev_read((size_t)E * ob * 4);
    float* act = (float*)dev_read((size_t)E * aout * 4);
    float* acm = (float*)dev_read((size_t)E * ac * 4);
    float* rew = (float*)dev_read((size_t)E * 4);
    uint8_t* done = (uint8_t*)dev_read((size_t)E);
    uint8_t* end = (uint8_t*)dev_read((size_t)E);
    CK(sppReplayAddObs(rb, o, E, next, NULL));
    CK(sppReplayAddStep(rb, prev, next, E, act, acm, rew, done, end, NULL));
    HK(hipDeviceSynchronize());
    HK(hipFree(o)); HK(hipFree(act)); HK(hipFree(acm)); HK(hipFree(rew)); HK(hipFree(done)); HK(hipFree(end));
    int64_t* sw = prev;
    prev = next;
    next = sw;
  }

  /* one device-sampled grad step: sample_batch's gather + normalisation, then update with device eps */
  int64_t* idx = (int64_t*)dev_read((size_t)B * 8);
  uint64_t sc[2];
  rd(sc, sizeof sc);
  fclose(fin);
  float* losses = (float*)dev_zero(SPP_NUM_LOSSES * 4);
  CK(sppAgentStageFromReplay(ag, rb, idx, B, NULL));
  if (normalize) CK(sppAgentStagePost(ag, 1, 0, NULL));
  CK(sppSacAcmUpdateStaged(ag, sc[0], sc[1], losses, NULL));
  HK(hipDeviceSynchronize());

  FILE* fo = fopen(argv[2], "wb");
  if (!fo) die("cannot open OUT");
  float lh[SPP_NUM_LOSSES];
  HK(hipMemcpy(lh, losses, sizeof lh, D2H));
  fwrite(lh, 4, SPP_NUM_LOSSES, fo);
  for (int net = 0; net < NNET; ++net) {
    float* h = (float*)malloc((size_t)sizes[net] * 4);
    HK(hipMemcpy(h, params[net], (size_t)sizes[net] * 4, D2H));
    fwrite(h, 4, (size_t)sizes[net], fo);
    free(h);
  }
  double as[4];
  HK(hipMemcpy(as, alpha_state, sizeof as, D2H));
  fwrite(as, 8, 4, fo);
  fclose(fo);
  CK(sppReplayDestroy(rb));
  CK(sppAgentDestroy(ag));
  printf("{\"losses\": [%.9g, %.9g, %.9g], \"B\": %d}\n", lh[0], lh[1], lh[2], B);
  return 0;
}
