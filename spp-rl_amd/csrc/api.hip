// libspprl C-ABI implementation (unity build: kernels included below).
#include <dlfcn.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/spprl.h"
#include "internal.h"
#include "replay.h"
#include "sac_kernels.h"

#include "optim.hip"
#include "ppo.hip"
#include "replay.hip"
#include "stats.hip"
#include "sac.hip"
#include "ddpg.hip"
#include "kset.h"
#ifdef SPP_SINGLE_TU  // profiling / development builds: everything in one TU
#include "ks_dw.hip"
#include "ks_sac_hopper.hip"
#if defined(SPP_WITH_HCHEETAH)  // region-profiling builds of the HalfCheetah AcM SGD: + the HalfCheetah set
#include "ks_sac_hcheetah.hip"
#endif
#if defined(SPP_ONLY_BF16)  // region-profiling builds of the bf16 sets: Hopper fp32 + bf16 only
#define SPP_ONLY_HOPPER
#include "ks_sac_bf16.hip"
#endif
#ifndef SPP_ONLY_HOPPER
#include "ks_sac_hcheetah.hip"
#include "ks_sac_ant.hip"
#include "ks_sac_small.hip"
#include "ks_ddpg.hip"
#include "ks_ddpg_ant.hip"
#include "ks_sac_bf16.hip"
#include "ks_sac_vanilla.hip"
#endif
#endif
#include "onp.hip"
#include "sgd.hip"
#include "sgd_mlp.hip"

namespace spp {

static thread_local std::string g_err;
void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}
const char* get_error() { return g_err.c_str(); }

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ================================================================== MT19937 (numpy legacy)
struct MT {
  uint32_t mt[624];
  int mti;
  void seed(uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    mti = 624;
  }
  uint32_t next() {
    if (mti >= 624) {
      for (int k = 0; k < 624; k++) {
        uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
        mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      mti = 0;
    }
    uint32_t y = mt[mti++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
};

}  // namespace spp

struct sppMT19937 {
  spp::MT mt;
};

using namespace spp;

// ================================================================== replay handle
struct sppReplay {
  ReplayDev d{};
  int device = 0, num_cu = 256;
  int64_t obs_idx = 0, ts_idx = 0, len = 0;
  // pinned ring for per-step index uploads
  static constexpr int kRing = 4;
  int64_t* pinned[kRing] = {};
  int64_t* dev_meta[kRing] = {};
  hipEvent_t ev[kRing] = {};
  int ring_cap = 0, ring_pos = 0;
  // obs-stats scratch
  double* st_part = nullptr;
  double* st_mean = nullptr;
  uint32_t* st_state = nullptr;
  uint32_t* st_hist = nullptr;
  // sample-bracketed single-device path (stats.hip)
  uint32_t *sf_samp = nullptr, *sf_bounds = nullptr, *sf_cpart = nullptr, *sf_wgl = nullptr, *sf_wgn = nullptr, *sf_ovf = nullptr,
           *sf_ovf_n = nullptr;
  double* sf_part = nullptr;
  // Ring generation: bumped by every entry point that can change the live rows (AddObs / AddStep /
  // Reset / GetView, whose caller may write).  sf_bounds holds the bracket of generation sf_gen
  // over sf_len rows: a later call on the same rows reuses it (the sample and its bracket would be
  // recomputed bit for bit).  Any bounds give the exact result (a rank outside the bracket falls
  // back to the raw column), so the generation only decides the cost, never the value.
  uint64_t gen = 0, sf_gen = ~0ull;
  int64_t sf_len = -1;
  bool bounds_dp1 = false;  // sf_bounds holds the union bracket of the last sppReplayObsStatsDP1 phase 1
  int st_cap_lim = 0, st_ovf_lim = 0;  // sppReplaySetObsStatsCaps (0: the full capacities)
  void* dp_q = nullptr;  // one-pass data-parallel statistics: per (column, target, rank) query state
  uint32_t* dp_cand = nullptr;  // and the compacted local candidates + counts
};

extern "C" {

const char* sppGetLastError(void) { return get_error(); }
int sppGetVersion(void) { return 1; }

sppStatus sppMTCreate(sppMTHandle* out, uint32_t seed) {
  SPP_REQUIRE(out, SPP_E_INVALID_ARG, "null out");
  auto* h = new sppMT19937;
  h->mt.seed(seed);
  *out = h;
  return SPP_OK;
}
sppStatus sppMTRandint(sppMTHandle h, int64_t high, int64_t n, int64_t* out) {
  SPP_REQUIRE(h && out && high >= 1 && high <= (int64_t)1 << 32, SPP_E_INVALID_ARG, "randint: bad args (high=%lld)",
              (long long)high);
  const uint64_t rng = (uint64_t)(high - 1);
  if (rng == 0) {
    for (int64_t i = 0; i < n; ++i) out[i] = 0;
    return SPP_OK;
  }
  uint64_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t v;
    do { v = h->mt.next() & (uint32_t)mask; } while (v > rng);
    out[i] = v;
  }
  return SPP_OK;
}
sppStatus sppMTDestroy(sppMTHandle h) {
  delete h;
  return SPP_OK;
}

sppStatus sppRandNormal(float* out, int64_t n, uint64_t seed, uint64_t offset, void* stream) {
  SPP_REQUIRE(out || n == 0, SPP_E_INVALID_ARG, "null out");
  if (n == 0) return SPP_OK;
  const int64_t groups = (n + 3) / 4;
  hipLaunchKernelGGL(k_rand_normal, dim3(cdiv(groups, 256)), dim3(256), 0, S(stream), out, n, seed, offset);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}
sppStatus sppRandIndex(int64_t* out, int64_t n, int64_t high, uint64_t seed, uint64_t offset, void* stream) {
  SPP_REQUIRE((out || n == 0) && high >= 1, SPP_E_INVALID_ARG, "bad args");
  if (n == 0) return SPP_OK;
  hipLaunchKernelGGL(k_rand_index, dim3(cdiv(n, 256)), dim3(256), 0, S(stream), out, n, high, seed, offset);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

// ------------------------------------------------------------------ replay
sppStatus sppReplayCreate(sppReplayHandle* out, int64_t cap, int ob, int aout, int ac, int device) {
  SPP_REQUIRE(out && cap > 0 && ob > 0 && aout > 0 && ac > 0, SPP_E_INVALID_ARG, "replay create: bad args");
  SPP_REQUIRE(cap < (int64_t)1 << 31, SPP_E_INVALID_ARG, "replay create: capacity %lld >= 2^31 (32-bit slots)",
              (long long)cap);
  SPP_CHECK_HIP(hipSetDevice(device));
  auto* h = new sppReplay;
  h->device = device;
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) h->num_cu = prop.multiProcessorCount;
  }
  ReplayDev& d = h->d;
  d.cap = cap;
  d.ob = ob;
  d.aout = aout;
  d.ac = ac;
  d.rw = rec_words(aout, ac);
  hipError_t e = hipSuccess;
  e = e ? e : hipMalloc(&d.obs, sizeof(float) * cap * ob);
  e = e ? e : hipMalloc(&d.obs_idx, sizeof(int64_t) * cap);
  e = e ? e : hipMalloc(&d.rec, sizeof(uint32_t) * cap * d.rw);  // (hipMalloc: 256-B aligned, records 64 B)
  e = e ? e : hipMemset(d.obs, 0, sizeof(float) * cap * ob);
  e = e ? e : hipMemset(d.obs_idx, 0, sizeof(int64_t) * cap);
  e = e ? e : hipMemset(d.rec, 0, sizeof(uint32_t) * cap * d.rw);
  if (e != hipSuccess) {
    set_error("replay alloc (%lld x %d): %s", (long long)cap, ob, hipGetErrorString(e));
    delete h;
    return SPP_E_OOM;
  }
  for (int i = 0; i < sppReplay::kRing; ++i) SPP_CHECK_HIP(hipEventCreateWithFlags(&h->ev[i], hipEventDisableTiming));
  *out = h;
  return SPP_OK;
}

sppStatus sppReplayDestroy(sppReplayHandle h) {
  if (!h) return SPP_OK;
  hipSetDevice(h->device);
  hipDeviceSynchronize();
  ReplayDev& d = h->d;
  hipFree(d.obs); hipFree(d.obs_idx); hipFree(d.rec); hipFree((void*)d.acm_cols);
  for (int i = 0; i < sppReplay::kRing; ++i) {
    if (h->pinned[i]) hipHostFree(h->pinned[i]);
    if (h->dev_meta[i]) hipFree(h->dev_meta[i]);
    hipEventDestroy(h->ev[i]);
  }
  hipFree(h->st_part); hipFree(h->st_mean); hipFree(h->st_state); hipFree(h->st_hist);
  hipFree(h->sf_samp); hipFree(h->sf_bounds); hipFree(h->sf_part); hipFree(h->sf_cpart); hipFree(h->sf_wgl); hipFree(h->sf_wgn);
  hipFree(h->sf_ovf); hipFree(h->sf_ovf_n); hipFree(h->dp_q); hipFree(h->dp_cand);
  delete h;
  return SPP_OK;
}

sppStatus sppReplayAddObs(sppReplayHandle h, const float* obs, int E, int64_t* slots, void* stream) {
  SPP_REQUIRE(h && obs && E > 0 && E <= h->d.cap, SPP_E_INVALID_ARG, "add_obs: bad args");
  const int64_t base = h->obs_idx;
  ++h->gen;
  hipLaunchKernelGGL(k_replay_add_obs, dim3(cdiv((int64_t)E * h->d.ob, 256)), dim3(256), 0, S(stream), h->d.obs,
                     h->d.cap, h->d.ob, obs, E, base);
  SPP_CHECK_HIP(hipGetLastError());
  for (int e = 0; e < E; ++e) {
    if (slots) slots[e] = (base + e) % h->d.cap;
  }
  h->obs_idx = (base + E) % h->d.cap;
  return SPP_OK;
}

// pinned host / device metadata ring of the per-step (prev, next, ts) uploads, >= E entries
static sppStatus ring_reserve(sppReplayHandle h, int E) {
  if (E <= h->ring_cap) return SPP_OK;
  hipDeviceSynchronize();
  for (int i = 0; i < sppReplay::kRing; ++i) {
    if (h->pinned[i]) hipHostFree(h->pinned[i]);
    if (h->dev_meta[i]) hipFree(h->dev_meta[i]);
    h->pinned[i] = nullptr;
    h->dev_meta[i] = nullptr;
    SPP_CHECK_HIP(hipHostMalloc(&h->pinned[i], sizeof(int64_t) * 3 * E));
    SPP_CHECK_HIP(hipMalloc(&h->dev_meta[i], sizeof(int64_t) * 3 * E));
  }
  h->ring_cap = E;
  return SPP_OK;
}

sppStatus sppReplayAddStep(sppReplayHandle h, const int64_t* prev, const int64_t* next, int E, const float* act,
                           const float* acm, const float* rew, const uint8_t* done, const uint8_t* end, void* stream) {
  SPP_REQUIRE(h && prev && next && E > 0 && rew && done && end, SPP_E_INVALID_ARG, "add_step: bad args");
  sppStatus rs = ring_reserve(h, E);
  if (rs) return rs;
  const int slot = h->ring_pos;
  h->ring_pos = (h->ring_pos + 1) % sppReplay::kRing;
  ++h->gen;
  SPP_CHECK_HIP(hipEventSynchronize(h->ev[slot]));  // the copy that last used this slot is done
  int64_t* m = h->pinned[slot];
  // add_timestep wrap rule (replay_buffer.py:65-75) applied sequentially in env order
  for (int e = 0; e < E; ++e) {
    SPP_REQUIRE(prev[e] >= 0 && prev[e] < h->d.cap && next[e] >= 0 && next[e] < h->d.cap, SPP_E_INVALID_ARG,
                "add_step: slot out of range");
    m[e] = prev[e];
    m[E + e] = next[e];
    m[2 * E + e] = h->ts_idx;
    if (next[e] < h->ts_idx) {
      h->len = h->ts_idx + 1;
      h->ts_idx = 0;
    } else {
      h->ts_idx += 1;
    }
    h->len = std::max(h->ts_idx, h->len);
    SPP_REQUIRE(h->ts_idx <= h->d.cap, SPP_E_STATE, "add_step: ts ring overflow (obs ring too small)");
    if (h->ts_idx == h->d.cap) h->ts_idx = h->d.cap - 1;  // unreachable with the reference wrap rule
  }
  SPP_CHECK_HIP(hipMemcpyAsync(h->dev_meta[slot], m, sizeof(int64_t) * 3 * E, hipMemcpyHostToDevice, S(stream)));
  SPP_CHECK_HIP(hipEventRecord(h->ev[slot], S(stream)));
  const int64_t n_el = (int64_t)E * (h->d.aout + h->d.ac + 1);
  hipLaunchKernelGGL(k_replay_add_step, dim3(cdiv(n_el, 256)), dim3(256), 0, S(stream), h->d, h->dev_meta[slot], E,
                     act, acm, rew, done, end);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppReplayState(sppReplayHandle h, int64_t* obs_idx, int64_t* ts_idx, int64_t* len) {
  SPP_REQUIRE(h, SPP_E_INVALID_ARG, "null handle");
  if (obs_idx) *obs_idx = h->obs_idx;
  if (ts_idx) *ts_idx = h->ts_idx;
  if (len) *len = h->len;
  return SPP_OK;
}
sppStatus sppReplayReset(sppReplayHandle h) {
  SPP_REQUIRE(h, SPP_E_INVALID_ARG, "null handle");
  h->obs_idx = h->ts_idx = h->len = 0;
  ++h->gen;
  return SPP_OK;
}

sppStatus sppReplayGather(sppReplayHandle h, const int64_t* idx, int B, float* obs, float* nobs, float* act,
                          float* rew, int8_t* done, float* acm, void* stream) {
  SPP_REQUIRE(h && idx && B > 0, SPP_E_INVALID_ARG, "gather: bad args");
  hipLaunchKernelGGL(k_replay_gather_rm, dim3(cdiv(B, 256)), dim3(256), 0, S(stream), h->d, idx, B, obs, nobs, act,
                     rew, done, acm);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppReplayGetView(sppReplayHandle h, sppReplayView* v) {
  SPP_REQUIRE(h && v, SPP_E_INVALID_ARG, "null");
  ++h->gen;  // the caller may write the ring through the view
  v->obs = h->d.obs;
  v->obs_idx = h->d.obs_idx;
  v->rec = h->d.rec;
  v->rec_words = h->d.rw;
  v->rec_acm = kRecAcm;
  v->rec_act = rec_act(h->d);
  return SPP_OK;
}

// §8b form of the constructor.  n_envs sizes the pinned per-step metadata ring up front;
// compat_mode 1 is the reference obs-index ring with the Q6 wrap rule (the only ring the
// reference has); store_fp64 0: the reference's float64 arrays only ever receive float32
// values (torch float32 obs, actions and rewards), so float32 storage is exact (Q5).
sppStatus sppReplayCreateEx(sppReplayHandle* out, int64_t cap, int ob, int aout, int ac, int n_envs,
                            int compat_mode, int store_fp64, int device) {
  SPP_REQUIRE(compat_mode == 1, SPP_E_INVALID_ARG,
              "replay create: compat_mode %d (only 1, the reference obs-index ring with the Q6 wrap, exists)",
              compat_mode);
  SPP_REQUIRE(store_fp64 == 0, SPP_E_INVALID_ARG,
              "replay create: store_fp64 %d (float32 storage is exact for every value the reference stores, Q5)",
              store_fp64);
  SPP_REQUIRE(n_envs > 0, SPP_E_INVALID_ARG, "replay create: n_envs %d", n_envs);
  sppStatus s = sppReplayCreate(out, cap, ob, aout, ac, device);
  if (s) return s;
  s = ring_reserve(*out, n_envs);
  if (s) {
    sppReplayDestroy(*out);
    *out = nullptr;
  }
  return s;
}

// BufferAcMOffPolicy.last_rollout (replay_buffer.py:335-383): the last complete episode is the
// *length timesteps first, first+1, ... (cyclic over [0, current_len)) ending at the last `end`
// at or before ts_idx - 1 (last_end, :170-177).  Synchronous (returns host values).
sppStatus sppReplayLastRollout(sppReplayHandle h, int64_t* first, int64_t* length, void* stream) {
  SPP_REQUIRE(h && first && length, SPP_E_INVALID_ARG, "last_rollout: null");
  const int64_t len = h->len;
  SPP_REQUIRE(len > 0, SPP_E_STATE, "last_rollout: empty buffer");
  hipStream_t st = S(stream);
  if (h->ts_idx == 0 && len == h->d.cap) {
    // python index ts_idx - 1 = -1 is the array's last element; when it is an end, the reference's
    // walk wraps to that same element at once (i = -2 -> current_len - 1) and stops: a 1-step rollout
    uint32_t w3 = 0;  // the last record's done | end word
    SPP_CHECK_HIP(hipMemcpyAsync(&w3, h->d.rec + (len - 1) * h->d.rw + 3, 4, hipMemcpyDeviceToHost, st));
    SPP_CHECK_HIP(hipStreamSynchronize(st));
    if ((w3 >> 8) & 1u) {
      *first = len - 1;
      *length = 1;
      return SPP_OK;
    }
  }
  const int64_t p = h->ts_idx > 0 ? std::min(h->ts_idx - 1, len - 1) : len - 1;
  int64_t* d = nullptr;
  SPP_CHECK_HIP(hipMallocAsync((void**)&d, 2 * sizeof(int64_t), st));
  hipLaunchKernelGGL(k_replay_last_rollout, dim3(1), dim3(1024), 0, st, (const uint32_t*)h->d.rec, h->d.rw, len, p,
                     d);
  int64_t hb[2] = {-1, -1};
  SPP_CHECK_HIP(hipMemcpyAsync(hb, d, sizeof(hb), hipMemcpyDeviceToHost, st));
  SPP_CHECK_HIP(hipFreeAsync(d, st));
  SPP_CHECK_HIP(hipStreamSynchronize(st));
  SPP_REQUIRE(hb[0] >= 0 && hb[1] >= 0, SPP_E_STATE, "last_rollout: no episode end in the buffer");
  int64_t T = (hb[0] - hb[1]) % len;
  if (T <= 0) T += len;
  *first = (hb[1] + 1) % len;
  *length = T;
  return SPP_OK;
}

static sppStatus stats_alloc(sppReplayHandle h) {
  const int ob = h->d.ob;
  const int G = std::min(ob, 32);
  if (!h->st_part) {
    SPP_CHECK_HIP(hipMalloc(&h->st_part, sizeof(double) * kStatsBlocks * ob * 2));
    SPP_CHECK_HIP(hipMalloc(&h->st_mean, sizeof(double) * ob * 2));
    SPP_CHECK_HIP(hipMalloc(&h->st_state, sizeof(uint32_t) * ob * 4 * 3));
    SPP_CHECK_HIP(hipMalloc(&h->st_hist, sizeof(uint32_t) * std::max(ob, G * 4) * 256));
    SPP_CHECK_HIP(hipMemset(h->st_hist, 0, sizeof(uint32_t) * std::max(ob, G * 4) * 256));  // k_stats_sel re-zeroes
    static bool attr = false;
    if (!attr) {  // > 64 KiB dynamic LDS for wide observations
      hipFuncSetAttribute((const void*)k_stats_p1, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      // (k_stats_pk: at most [32][4][256] or [128][4][64] counters = 128 KiB, beside its 4 KiB static table)
      hipFuncSetAttribute((const void*)k_stats_pk, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
      attr = true;
    }
  }
  return SPP_OK;
}

static void stats_pass1(sppReplayHandle h, uint32_t* hist, const float* pivot, hipStream_t st) {
  const int ob = h->d.ob;
  const size_t lds1 = sizeof(uint32_t) * (((ob * 256 + 1) & ~1)) + sizeof(double) * 16 * 16 * 2;
  hipLaunchKernelGGL(k_stats_p1, dim3(kStatsBlocks), dim3(256), lds1, st, h->d, h->len, hist, h->st_part, pivot);
}

// digit pass p (0-based) after the top byte, all columns: 8-bit digits at bits 16, 8, 0 when the
// [ob][4][256] LDS histogram fits 128 KiB (ob <= 32), else 6-bit digits at bits 18, 12, 6, 0
static int stats_dbits(sppReplayHandle h) { return h->d.ob <= 32 ? 8 : 6; }
static int stats_npass(sppReplayHandle h) { return 24 / stats_dbits(h); }
static int stats_shift(sppReplayHandle h, int p) { return 24 - stats_dbits(h) * (p + 1); }

static void stats_pk(sppReplayHandle h, int p, uint32_t* hist, hipStream_t st) {
  const size_t ldsk = sizeof(uint32_t) * h->d.ob * 4 * (1u << stats_dbits(h));
  // one 1024-thread block per CU (each flushes its LDS histogram with device atomics at the end)
  const int resident = 1;
  hipLaunchKernelGGL(k_stats_pk, dim3(h->num_cu * resident), dim3(kStatsPkThreads), ldsk, st, h->d, h->len,
                     stats_shift(h, p), stats_dbits(h), (const uint32_t*)h->st_state, hist);
}

static void stats_sel(sppReplayHandle h, int p, uint32_t* hist, int64_t n, float* max_obs, float* min_obs,
                      int first_update, hipStream_t st) {
  hipLaunchKernelGGL(k_stats_sel, dim3(h->d.ob), dim3(256), 0, st, hist, kStatsBlocks, h->d.ob, 0, h->d.ob,
                     stats_shift(h, p), stats_dbits(h), 0, (const double*)nullptr, n, h->st_state, h->st_mean,
                     max_obs, min_obs,
                     first_update);
}

static int st_nblk(sppReplayHandle h) {  // every pass workgroup resident at once (4 per CU)
  return std::max(1, std::min(kStNblkMax, 4 * h->num_cu));
}

// candidate-list capacities of the sample-bracketed statistics (sppReplaySetObsStatsCaps may lower them so
// the overflow paths run at small sizes; the allocations keep the full strides)
static int st_cap(sppReplayHandle h) {
  const int c = st_list_cap(h->d.ob);
  return h->st_cap_lim > 0 ? std::min(c, h->st_cap_lim) : c;
}
static int st_ovf_cap(sppReplayHandle h) {
  return h->st_ovf_lim > 0 ? std::min(kStOvfCap, h->st_ovf_lim) : kStOvfCap;
}

sppStatus sppReplaySetObsStatsCaps(sppReplayHandle h, int list_cap, int ovf_cap) {
  SPP_REQUIRE(h && list_cap >= 0 && ovf_cap >= 0, SPP_E_INVALID_ARG, "set_obs_stats_caps: bad args");
  h->st_cap_lim = list_cap;
  h->st_ovf_lim = ovf_cap;
  return SPP_OK;
}

static sppStatus stats_fast_alloc(sppReplayHandle h) {
  if (h->sf_bounds) return SPP_OK;
  const int ob = h->d.ob, nb = kStNblkMax;
  SPP_CHECK_HIP(hipMalloc(&h->sf_bounds, sizeof(uint32_t) * ob * 4));
  SPP_CHECK_HIP(hipMalloc(&h->sf_samp, sizeof(uint32_t) * (size_t)ob * kStSampBig));
  SPP_CHECK_HIP(hipMalloc(&h->sf_part, sizeof(double) * nb * ob * 2));
  SPP_CHECK_HIP(hipMalloc(&h->sf_cpart, sizeof(uint32_t) * nb * ob * 6));
  SPP_CHECK_HIP(hipMalloc(&h->sf_wgl, sizeof(uint32_t) * (size_t)nb * ob * 2 * st_list_cap(ob)));
  SPP_CHECK_HIP(hipMalloc(&h->sf_wgn, sizeof(uint32_t) * (size_t)nb * ob * 2));
  SPP_CHECK_HIP(hipMalloc(&h->sf_ovf, sizeof(uint32_t) * (size_t)ob * 2 * kStOvfCap));
  SPP_CHECK_HIP(hipMalloc(&h->sf_ovf_n, sizeof(uint32_t) * ob * 2));
  SPP_CHECK_HIP(hipMemset(h->sf_ovf_n, 0, sizeof(uint32_t) * ob * 2));  // k_st_select re-zeroes
  return SPP_OK;
}

sppStatus sppReplayObsStats(sppReplayHandle h, float* mean, float* std, float* max_obs, float* min_obs,
                            int first_update, void* stream) {
  SPP_REQUIRE(h && mean && std && max_obs && min_obs, SPP_E_INVALID_ARG, "obs_stats: bad args");
  const int64_t len = h->len;
  if (len <= 10) return SPP_OK;  // replay_buffer.py:84
  const int ob = h->d.ob;
  SPP_REQUIRE(ob <= 128, SPP_E_SHAPE, "obs_stats: ob %d > 128", ob);
  const int nblk = st_nblk(h);
  // per-lane counters are 16-bit: rows per lane = len / (waves * G) < 65536
  SPP_REQUIRE(len / ((int64_t)nblk * (kStPassThreads / 64) * st_groups(ob)) < 60000, SPP_E_INVALID_ARG,
              "obs_stats: len too large");
  sppStatus s = stats_fast_alloc(h);
  if (s) return s;
  hipStream_t st = S(stream);
  const bool big = len > kStBigLen;
  const int ns = (int)std::min<int64_t>(len, big ? kStSampBig : kStSampSmall);
  if (h->sf_gen != h->gen || h->sf_len != len) {  // else: the same rows' bracket is in sf_bounds
    hipLaunchKernelGGL(k_st_sample, dim3(cdiv(ns, 256)), dim3(256), 0, st, h->d, len, ns, h->sf_samp);
    if (big)
      hipLaunchKernelGGL(k_st_bracket<kStSampBig / 1024>, dim3(ob), dim3(1024), 0, st, h->sf_samp, ns, h->sf_bounds,
                         ns, (int64_t)0, 4);
    else
      hipLaunchKernelGGL(k_st_bracket<kStSampSmall / 1024>, dim3(ob), dim3(1024), 0, st, h->sf_samp, ns,
                         h->sf_bounds, ns, (int64_t)0, 4);
    h->sf_gen = h->gen;
    h->sf_len = len;
    h->bounds_dp1 = false;
  }
  const int cap = st_cap(h), ovf_cap = st_ovf_cap(h);
  StPassArgs pa{h->d, len, h->sf_bounds, nullptr, h->sf_part, h->sf_cpart, h->sf_wgl, h->sf_wgn, h->sf_ovf,
                h->sf_ovf_n, cap, ovf_cap};
  st_launch_pass(pa, nblk, st);
  StSelArgs sa{h->d, len, nblk, cap, h->sf_part, h->sf_cpart, h->sf_bounds, h->sf_wgl, h->sf_wgn, h->sf_ovf,
               h->sf_ovf_n, nullptr, mean, std, max_obs, min_obs, first_update, ovf_cap};
  hipLaunchKernelGGL(k_st_select, dim3(ob, 2), dim3(kStSelThreads), 0, st, sa);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

// ---- data-parallel statistics, one data pass per call (stats.hip "data-parallel: one data pass")
int sppReplayObsStatsDP1SampleRows(sppReplayHandle h, int world, int64_t n_global) {
  if (!h || world < 1) return -1;
  const int S = n_global > kStBigLen ? kStSampBig : kStSampSmall;
  return std::max(1, S / world);
}

sppStatus sppReplayObsStatsDP1(sppReplayHandle h, int phase, int world, int rank, const float* pivot, uint32_t* samp,
                               double* exch, uint32_t* hist, int64_t n_global, float* mean, float* std,
                               float* max_obs, float* min_obs, int first_update, void* stream) {
  const bool reuse = phase == (1 | SPP_DP1_REUSE_BRACKET);
  if (reuse) phase = 1;
  SPP_REQUIRE(h && pivot && samp && exch && hist && mean && std && max_obs && min_obs && phase >= 0 && phase <= 6 &&
                  world >= 1 && rank >= 0 && rank < world,
              SPP_E_INVALID_ARG, "obs_stats_dp1: bad args (phase %d, rank %d of %d)", phase, rank, world);
  SPP_REQUIRE(n_global > 10 && n_global < ((int64_t)1 << 31), SPP_E_INVALID_ARG, "obs_stats_dp1: n_global %lld",
              (long long)n_global);
  const int ob = h->d.ob;
  SPP_REQUIRE(ob <= 128, SPP_E_SHAPE, "obs_stats_dp1: ob %d > 128", ob);
  const int64_t len = h->len;
  const int nblk = st_nblk(h);
  SPP_REQUIRE(len / ((int64_t)nblk * (kStPassThreads / 64) * st_groups(ob)) < 60000, SPP_E_INVALID_ARG,
              "obs_stats_dp1: len too large");
  sppStatus s = stats_fast_alloc(h);
  if (s) return s;
  if (!h->dp_q) {
    SPP_CHECK_HIP(hipMalloc(&h->dp_q, sizeof(DpQuery) * ob * 4));
    SPP_CHECK_HIP(hipMalloc(&h->dp_cand, sizeof(uint32_t) * ((size_t)ob * 2 * kDpCandCap + ob * 2)));
  }
  uint32_t* dp_ncand = h->dp_cand + (size_t)ob * 2 * kDpCandCap;
  hipStream_t st = S(stream);
  const int Sl = sppReplayObsStatsDP1SampleRows(h, world, n_global);
  uint32_t* mine = samp + (int64_t)rank * ob * Sl;
  const int cap = st_cap(h), ovf_cap = st_ovf_cap(h);
  StDpArgs da{h->d, len, n_global, nblk, cap, ovf_cap, h->sf_bounds, h->sf_wgl, h->sf_wgn, h->sf_ovf, h->sf_ovf_n,
              h->dp_cand, dp_ncand, exch, hist, (DpQuery*)h->dp_q, pivot, mean, std, max_obs, min_obs, first_update};
  if (phase == 0) {
    if (len > 0) hipLaunchKernelGGL(k_st_sample, dim3(cdiv(Sl, 256)), dim3(256), 0, st, h->d, len, Sl, mine);
    else SPP_CHECK_HIP(hipMemsetAsync(mine, 0, sizeof(uint32_t) * ob * Sl, st));  // (lockstep shards: not reached)
  } else if (phase == 1) {
    const int S = world * Sl;  // <= kStSampBig
    // margin 5 sigma + 4 sample ranks: a miss costs the raw-column select of the rounds, not correctness.
    // reuse (decided alike on every rank): keep the last union bracket; if the N = 1 path overwrote the
    // bounds since, recompute them from samp (the same union sample on every rank)
    if (!(reuse && h->bounds_dp1)) {
      if (S > kStSampSmall)
        hipLaunchKernelGGL(k_st_bracket<kStSampBig / 1024>, dim3(ob), dim3(1024), 0, st, (const uint32_t*)samp, S,
                           h->sf_bounds, Sl, (int64_t)ob * Sl, 5);
      else
        hipLaunchKernelGGL(k_st_bracket<kStSampSmall / 1024>, dim3(ob), dim3(1024), 0, st, (const uint32_t*)samp, S,
                           h->sf_bounds, Sl, (int64_t)ob * Sl, 5);
      h->bounds_dp1 = true;
      h->sf_gen = ~0ull;  // the N = 1 path must not take these (union) bounds for its own
    }
    StPassArgs pa{h->d, len, h->sf_bounds, pivot, h->sf_part, h->sf_cpart, h->sf_wgl, h->sf_wgn, h->sf_ovf,
                  h->sf_ovf_n, cap, ovf_cap};
    st_launch_pass(pa, nblk, st);
    hipLaunchKernelGGL(k_dp_reduce, dim3(ob, 2), dim3(kStSelThreads), 0, st, ob, nblk, cap, ovf_cap,
                       (const double*)h->sf_part,
                       (const uint32_t*)h->sf_cpart, (const uint32_t*)h->sf_wgl, (const uint32_t*)h->sf_wgn,
                       (const uint32_t*)h->sf_ovf, (const uint32_t*)h->sf_ovf_n, exch, h->dp_cand, dp_ncand);
  } else if (phase <= 5) {
    hipLaunchKernelGGL(k_dp_round, dim3(ob, 2), dim3(kStSelThreads), 0, st, da, phase - 2);
  } else {
    hipLaunchKernelGGL(k_dp_final, dim3(ob, 2), dim3(128), 0, st, da);
  }
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

int sppReplayObsStatsDPHistSize(sppReplayHandle h) {
  if (!h) return -1;
  const int ob = h->d.ob;
  return std::max(ob, std::min(ob, 32) * 4) * 256;
}

sppStatus sppReplayObsStatsDP(sppReplayHandle h, int step, const float* pivot, double* sums, uint32_t* hist,
                              int64_t n_global, float* mean, float* std, float* max_obs, float* min_obs,
                              int first_update, int* done, void* stream) {
  SPP_REQUIRE(h && pivot && sums && hist && mean && std && max_obs && min_obs && done && step >= 0,
              SPP_E_INVALID_ARG, "obs_stats_dp: bad args");
  const int ob = h->d.ob;
  SPP_REQUIRE(ob <= 16 * kStatsColsPerThread, SPP_E_SHAPE, "obs_stats_dp: ob %d > %d", ob, 16 * kStatsColsPerThread);
  // counts travel as int32 (the host's fused first exchange converts fp64 sums back to int32)
  SPP_REQUIRE(n_global > 10 && n_global < ((int64_t)1 << 31), SPP_E_INVALID_ARG, "obs_stats_dp: n_global %lld",
              (long long)n_global);
  sppStatus s = stats_alloc(h);
  if (s) return s;
  hipStream_t st = S(stream);
  const int npass = stats_npass(h);
  SPP_REQUIRE(step <= npass + 1, SPP_E_INVALID_ARG, "obs_stats_dp: step %d > %d", step, npass + 1);
  *done = 0;
  if (step == 0) {  // local pass 1 -> sums [ob][2] about the shared pivot, top-byte histogram
    SPP_CHECK_HIP(hipMemsetAsync(hist, 0, sizeof(uint32_t) * sppReplayObsStatsDPHistSize(h), st));
    if (h->len > 0) {
      stats_pass1(h, hist, pivot, st);
      hipLaunchKernelGGL(k_stats_reduce_part, dim3(ob), dim3(256), 0, st, (const double*)h->st_part, kStatsBlocks,
                         ob, sums);
    } else {
      SPP_CHECK_HIP(hipMemsetAsync(sums, 0, sizeof(double) * ob * 2, st));
    }
  } else {
    if (step == 1) {  // global top byte + moments
      hipLaunchKernelGGL(k_stats_sel, dim3(ob), dim3(256), 0, st, hist, 1, ob, 0, ob, 24, 8, 1, (const double*)sums,
                         n_global, h->st_state, h->st_mean, max_obs, min_obs, first_update);
      hipLaunchKernelGGL(k_stats_moments_out, dim3(1), dim3(128), 0, st, h->d, (const double*)h->st_mean, mean, std,
                         pivot);
    } else {
      stats_sel(h, step - 2, hist, n_global, max_obs, min_obs, first_update, st);
    }
    if (step - 1 < npass) {
      if (h->len > 0) stats_pk(h, step - 1, hist, st);
    } else {
      *done = 1;
    }
  }
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppGaeScan(const float* rew, const float* v, const float* v_next, const uint8_t* done,
                     const uint8_t* end, int64_t T, int64_t E, double gamma, double lam, int mode, float* q_out,
                     float* adv, void* stream) {
  SPP_REQUIRE(T >= 0 && E > 0 && mode >= -1 && mode <= 1, SPP_E_INVALID_ARG, "gae: T=%lld E=%lld mode=%d",
              (long long)T, (long long)E, mode);
  if (T == 0) return SPP_OK;
  SPP_REQUIRE(rew && v && v_next && done && end && adv, SPP_E_INVALID_ARG, "gae: null input");
  if (mode < 0) mode = E >= 64 ? 0 : 1;
  const double disc = lam * gamma;  // python floats: discount = gae_lambda * gamma (ppo.py:136)
  if (mode == 0)
    hipLaunchKernelGGL(k_gae_seq, dim3(cdiv(E, 256)), dim3(256), 0, S(stream), rew, v, v_next, done, end, T, E,
                       (float)gamma, disc, q_out, adv);
  else
    hipLaunchKernelGGL(k_gae_scan, dim3(E), dim3(kScanThreads), 0, S(stream), rew, v, v_next, done, end, T, E,
                       (float)gamma, (float)disc, q_out, adv);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppPpoClipLoss(const float* lp_old, const float* lp_new, const float* adv, int B, float eps, float* grad,
                         float* out2, void* stream) {
  SPP_REQUIRE(lp_old && lp_new && adv && out2 && B > 0, SPP_E_INVALID_ARG, "clip loss: bad args");
  const int nblk = cdiv(B, 256);
  double* part = nullptr;
  SPP_CHECK_HIP(hipMallocAsync((void**)&part, sizeof(double) * 2 * nblk, S(stream)));
  hipLaunchKernelGGL(k_ppo_clip, dim3(nblk), dim3(256), 0, S(stream), lp_old, lp_new, adv, B, eps, grad, part);
  hipLaunchKernelGGL(k_ppo_clip_finish, dim3(1), dim3(256), 0, S(stream), (const double*)part, nblk, B, out2);
  SPP_CHECK_HIP(hipFreeAsync(part, S(stream)));
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppAdvNormalize(const float* adv, int64_t n, float* out, void* stream) {
  SPP_REQUIRE(adv && out && n > 0, SPP_E_INVALID_ARG, "adv normalize: bad args");
  const int nblk = (int)std::min<int64_t>(cdiv(n, 256), 1024);
  double* part = nullptr;
  SPP_CHECK_HIP(hipMallocAsync((void**)&part, sizeof(double) * 2 * nblk, S(stream)));
  hipLaunchKernelGGL(k_adv_moments, dim3(nblk), dim3(256), 0, S(stream), adv, n, part);
  hipLaunchKernelGGL(k_adv_norm, dim3(nblk), dim3(256), 0, S(stream), adv, n, (const double*)part, nblk, out);
  SPP_CHECK_HIP(hipFreeAsync(part, S(stream)));
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppAdvSums(const float* adv, int64_t n, double* sums2, void* stream) {
  SPP_REQUIRE(adv && sums2 && n >= 0, SPP_E_INVALID_ARG, "adv sums: bad args");
  if (n == 0) {
    SPP_CHECK_HIP(hipMemsetAsync(sums2, 0, sizeof(double) * 2, S(stream)));
    return SPP_OK;
  }
  const int nblk = (int)std::min<int64_t>(cdiv(n, 256), 1024);
  double* part = nullptr;
  SPP_CHECK_HIP(hipMallocAsync((void**)&part, sizeof(double) * 2 * nblk, S(stream)));
  hipLaunchKernelGGL(k_adv_moments, dim3(nblk), dim3(256), 0, S(stream), adv, n, part);
  hipLaunchKernelGGL(k_adv_sum2, dim3(1), dim3(64), 0, S(stream), (const double*)part, nblk, sums2);
  SPP_CHECK_HIP(hipFreeAsync(part, S(stream)));
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppAdvNormalizeGlobal(const float* adv, int64_t n_local, const double* sums2, int64_t n_global, float* out,
                                void* stream) {
  SPP_REQUIRE(adv && out && sums2 && n_local >= 0 && n_global > 0, SPP_E_INVALID_ARG, "adv normalize dp: bad args");
  if (n_local == 0) return SPP_OK;
  hipLaunchKernelGGL(k_adv_norm_g, dim3((int)std::min<int64_t>(cdiv(n_local, 256), 1024)), dim3(256), 0, S(stream),
                     adv, n_local, sums2, n_global, out);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppSynthEnvStep(const float* A, const float* obs, const float* action, int E, int ob, int ac,
                          float* next_obs, float* reward, void* stream) {
  SPP_REQUIRE(A && obs && action && next_obs && reward && E > 0, SPP_E_INVALID_ARG, "synth env: bad args");
  hipLaunchKernelGGL(k_synth_env, dim3(cdiv((int64_t)E * ob, 256)), dim3(256), 0, S(stream), A, obs, action, E, ob, ac, next_obs,
                     reward);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}


sppStatus sppRandUniform(float* out, int64_t n, const float* lo, const float* hi, int period, uint64_t seed,
                         uint64_t offset, void* stream) {
  SPP_REQUIRE((out || n == 0) && lo && hi && period > 0, SPP_E_INVALID_ARG, "rand uniform: bad args");
  if (n == 0) return SPP_OK;
  hipLaunchKernelGGL(k_rand_uniform, dim3(cdiv((n + 3) / 4, 256)), dim3(256), 0, S(stream), out, n, lo, hi, period,
                     seed, offset);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppEpisodeAccum(const float* rew, const uint8_t* end, int E, float* ep_ret, double* sums, void* stream) {
  SPP_REQUIRE(rew && ep_ret && sums && E > 0, SPP_E_INVALID_ARG, "episode accum: bad args");
  hipLaunchKernelGGL(k_episode_accum, dim3(cdiv(E, 256)), dim3(256), 0, S(stream), rew, end, E, ep_ret, sums);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppSynthEnvReset(float* obs, const uint8_t* mask, int E, int ob, uint64_t seed, uint64_t offset,
                           void* stream) {
  SPP_REQUIRE(obs && E > 0 && ob > 0, SPP_E_INVALID_ARG, "synth reset: bad args");
  hipLaunchKernelGGL(k_synth_reset, dim3(cdiv((int64_t)E * ob, 256)), dim3(256), 0, S(stream), obs, mask, E, ob, seed,
                     offset);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppObsNormalize(const float* x, int64_t rows, int ob, const float* lo, const float* hi, const float* mean,
                          const float* std, int min_max, int inverse, float* out, void* stream) {
  SPP_REQUIRE(x && out && rows >= 0 && ob > 0, SPP_E_INVALID_ARG, "normalize: bad args");
  SPP_REQUIRE(min_max ? (lo && hi) : (mean && std), SPP_E_INVALID_ARG, "normalize: missing statistics");
  if (rows == 0) return SPP_OK;
  const int64_t n = rows * ob;
  hipLaunchKernelGGL(k_obs_normalize, dim3(cdiv(n, 256)), dim3(256), 0, S(stream), x, n, ob, lo, hi, mean, std,
                     min_max, inverse, out);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}
}  // extern "C"

// ================================================================== agent
namespace spp {

struct NetBufs {
  float *p = nullptr, *g = nullptr, *m = nullptr, *v = nullptr;
  int64_t n = 0;
};

template <typename T>
struct DevArray {
  T* ptr = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t count) {
    n = count;
    return hipMalloc(&ptr, sizeof(T) * std::max<size_t>(count, 1));
  }
  void release() {
    if (ptr) hipFree(ptr);
    ptr = nullptr;
  }
};

// A weight-gradient job set (dw.hip): up to two phases launched separately.
struct DwSet {
  DevArray<float> slab;
  DevArray<DwJob> jobs;
  DevArray<int> items;
  int B = -1;
  int j0[2] = {0, 0}, nj[2] = {0, 0}, ioff[2] = {0, 0}, nitems[2] = {0, 0};
  int nlds[2] = {0, 0};  // leading items of a phase that run as k_dw_big / k_dw_big16 (256 x 256 jobs)
  int64_t max_elems[2] = {1, 1};  // reduce lanes per phase: largest [N*K | N] image x its dw_red_group
  bool bf16 = false;              // bf16 MFMA job set (k_dw<true>)
  void release() { slab.release(); jobs.release(); items.release(); }
};

// dims -> kernel instantiation: one translation unit per config family (ks_*.hip),
// compiled in parallel by build.py and linked into libspprl.so.
static bool find_kset(int algo, int ob, int aout, int ac, bool acmc, bool bf16, KernelSet* ks) {
  if (bf16) {
#if !defined(SPP_ONLY_HOPPER) || defined(SPP_ONLY_BF16)
    return algo == SPP_ALGO_SAC_ACM && kset_sac_bf16(ob, aout, ac, acmc, ks);
#else
    return false;
#endif
  }
  if (algo == SPP_ALGO_SAC) {
#ifndef SPP_ONLY_HOPPER
    return kset_sac_vanilla(ob, aout, ac, acmc, ks);
#else
    return false;
#endif
  }
  if (algo == SPP_ALGO_SAC_ACM) {
    if (kset_sac_hopper(ob, aout, ac, acmc, ks)) return true;
#if defined(SPP_ONLY_HOPPER) && defined(SPP_WITH_HCHEETAH)
    if (kset_sac_hcheetah(ob, aout, ac, acmc, ks)) return true;
#endif
#ifndef SPP_ONLY_HOPPER  // kernel-development builds: one instantiation, fast compile
    if (kset_sac_hcheetah(ob, aout, ac, acmc, ks)) return true;
    if (kset_sac_ant(ob, aout, ac, acmc, ks)) return true;
    if (kset_sac_small(ob, aout, ac, acmc, ks)) return true;
  } else if (algo == SPP_ALGO_DDPG_ACM) {
    if (kset_ddpg(ob, aout, ac, acmc, ks)) return true;
    if (kset_ddpg_ant(ob, aout, ac, acmc, ks)) return true;
#endif
  }
  return false;
}

}  // namespace spp

struct sppAgent {
  sppAgentConfig cfg{};
  int device = 0, num_cu = 256;
  bool team_ok = true;  // SPP_SAC_TEAM=0: the one-wave phase kernels at every batch (A/B)
  KernelSet ks{};
  NetBufs net[SPP_NET_COUNT];
  int64_t nsize[SPP_NET_COUNT] = {};
  int cin = 0, Bmax = 0, Bpmax = 0;
  int64_t steps[4] = {0, 0, 0, 0};  // actor, critic, alpha, acm
  const float *lo = nullptr, *hi = nullptr, *mean = nullptr, *std = nullptr;
  double* alpha_state = nullptr;
  float* alpha_f32 = nullptr;
  DevArray<float> limits;  // [aout] actor lim | [ac] acm lim
  // packed images
  DevArray<float4> pk;     // all matrix images
  std::vector<PackJob> pj_actor, pj_acm, pj_targ, pj_critic_fwd, pj_critic_all, pj_acmreg;
  bool ddpg = false;
  bool plain = false;  // vanilla SAC (SPP_ALGO_SAC): the ACM net exists but is never evaluated
  DevArray<PackJob> d_pj;
  // job-table offsets inside d_pj
  int o_actor = 0, o_acm = 0, o_targ = 0, o_cfwd = 0, o_call = 0, o_acmreg = 0;
  // LDS constant-table segments (canonical bias / fc3 vectors, read at kernel start)
  std::vector<TabSeg> tab;
  int tab_floats = 0;  // weight part of the table (make_args appends the limit / normaliser segments)
  ActorDev actor{};
  CriticDev critic[2]{}, targ[2]{};
  AcmDev acm{};
  const float4* acm_W1n = nullptr;  // ACM W1 natural input packing (regression)
  // DDPG_AcM
  BAcmDev bacm{};
  ActorDev actor_targ{};
  const float4 *bacm_W1n = nullptr, *bacm_W21n = nullptr;  // natural-input packings (regression)
  BAcmScratch bz{};  // agent-phase BasicAcM activations
  float *RBH = nullptr, *RBH1 = nullptr, *RS21 = nullptr, *RBP1 = nullptr, *RPZ = nullptr, *RPZ21 = nullptr;
  // scratch
  DevArray<float> scratch;
  float *S = nullptr, *S2 = nullptr, *ACT = nullptr, *AENV = nullptr, *R = nullptr, *DN = nullptr, *EPS1 = nullptr,
        *EPS2 = nullptr;
  float *H1[2] = {}, *H2[2] = {}, *D1[2] = {}, *D2[2] = {}, *DQ[2] = {};
  float *AH1 = nullptr, *AH2 = nullptr, *AD1 = nullptr, *AD2 = nullptr, *ADH = nullptr;
  float *Z1 = nullptr, *Z2 = nullptr, *T3 = nullptr, *part = nullptr;
  float *aux = nullptr;  // [4] alpha grad operand (all-reduced in DP)
  float* GAD = nullptr;       // wide-head actor phase: d a_d hand-over [aout][Bp]
  uint64_t* MASK = nullptr;   // and the trunk's ReLU masks [tile][4][64]
  // ACM regression scratch
  float *RX = nullptr, *RZ1 = nullptr, *RZ2 = nullptr, *RP1 = nullptr, *RP2 = nullptr, *RP3 = nullptr;
  // weight-gradient job sets: [0] SAC (critic phase, actor phase), [1] ACM regression
  DwSet dws[2];
  DevArray<AdamJob> d_adam;  // [critic1, critic2 | actor | acm]
  int cur_B = -1;            // staged batch size
  float* w3p[2] = {};         // SAC critics' fused fc3 gradient partials (slabs of the reduce-only dW jobs)
  int64_t w3p_stride = 0;
  float* alpha_grad = nullptr;  // bound operand (defaults to internal scratch)
  // multi-workgroup AcM SGD (sppAcmSgd with bs > kMlR): gradient slabs + parameter buffer, {counter, timeout flag}
  DevArray<float> sgd_slab;
  DevArray<int> sgd_sync;
  int sgd_max_wg = -1;  // co-resident k_mlp_sgd workgroups (acm_sgd_max_wg, cached)
  // per-kernel timing (HIP events on the launch stream)
  bool timing = false;
  std::vector<hipEvent_t> tev[5];
  size_t tused[5] = {0, 0, 0, 0, 0};
};

static void tmark(sppAgent* a, int kind, hipStream_t st) {
  if (!a->timing) return;
  auto& v = a->tev[kind];
  if (a->tused[kind] == v.size()) {
    hipEvent_t e;
    hipEventCreate(&e);
    v.push_back(e);
  }
  hipEventRecord(v[a->tused[kind]++], st);
}

namespace spp {

static int64_t sac_actor_size(int ob, int aout) { return 256LL * ob + 256 + 65536 + 256 + 2LL * (aout * 256 + aout); }
static int64_t critic_size(int cin) { return 256LL * cin + 256 + 65536 + 256 + 256 + 1; }
static int64_t acm_size(int in, int ac) { return 64LL * in + 64 + 32 * 64 + 32 + (int64_t)ac * 32 + ac; }
static int64_t ddpg_actor_size(int ob, int aout) { return 256LL * ob + 256 + 65536 + 256 + (int64_t)aout * 256 + aout; }
// BasicAcM state_dict: t, t1, fc1, fc2, fc21, fc3 (basic_acm.py:11-21)
static int64_t bacm_size(int in, int ac) {
  return 1 + ac + 100LL * in + 100 + 50 * 100 + 50 + 50LL * in + 50 + (int64_t)ac * 50 + ac;
}

static MapDesc nat(int n) { return MapDesc{MAP_NAT, n, 0, 0, 0}; }
static MapDesc cat(int n0, int n1) { return MapDesc{MAP_CAT, n0, blocks_of(n0), n1, n0}; }
static MapDesc pair(int n) { return MapDesc{MAP_PAIR, n, 0, 0, 0}; }

}  // namespace spp

// Build all pack jobs (the parameter pointers must be bound).
static sppStatus build_packs(sppAgent* a) {
  const int ob = a->cfg.ob, aout = a->cfg.aout, ac = a->cfg.ac;
  const int ca = a->cfg.acm_critic ? ac : aout;
  const int cin = ob + ca;
  for (int k = 0; k < SPP_NET_COUNT; ++k) {
    const bool used = a->ddpg ? (k == SPP_NET_ACTOR || k == SPP_NET_CRITIC1 || k == SPP_NET_CRITIC1_TARG ||
                                 k == SPP_NET_ACM || k == SPP_NET_ACTOR_TARG)
                              : k != SPP_NET_ACTOR_TARG;
    SPP_REQUIRE(!used || a->net[k].p, SPP_E_STATE, "network %d parameters not bound", k);
  }
  // sizes: count float4 and vector slots first
  struct MatSpec {
    std::vector<PackJob>* list;
    PackJob job;
    const float4** slot;
  };
  std::vector<MatSpec> ms;
  // ib = 1: ib-major image for dense_lds (256-input layers)
  auto M = [&](std::vector<PackJob>* list, const float* W, const float* W2, int split, int ld, int trans, int coff,
               MapDesc out, MapDesc in, int NBO, int NBI, const float4** slot, int ib = 0) {
    PackJob j{W, W2, split, ld, trans, coff, out, in, NBO, NBI, ib, nullptr, a->cfg.mlp_bf16 ? 1 : 0};
    ms.push_back({list, j, slot});
  };
  // LDS table: each vector starts on a 32-float boundary, zero padded to a whole block
  a->tab.clear();
  int toff = 0;
  auto T = [&](const float* v, int n, const float* v2 = nullptr, int n2 = 0) {
    const int off = toff, tot = (int)round_up(n + n2, 32);
    a->tab.push_back(TabSeg{v, n, v2 ? n : tot, off, 0});
    if (v2) a->tab.push_back(TabSeg{v2, n2, tot - n, off + n, 0});
    toff += tot;
    return off;
  };
  if (!a->ddpg) {
    // ---- actor (sac/models.py:12-22): fc1 [256][ob], fc2, fc_prob [aout][256], fc_scale
    {
      const float* P = a->net[SPP_NET_ACTOR].p;
      const float *W1 = P, *b1 = W1 + 256 * ob, *W2 = b1 + 256, *b2 = W2 + 65536, *Wp = b2 + 256, *bp = Wp + aout * 256,
                  *Ws = bp + aout, *bs = Ws + aout * 256;
      M(&a->pj_actor, W1, nullptr, 1 << 30, ob, 0, 0, nat(256), nat(ob), 8, blocks_of(ob), &a->actor.W1);
      M(&a->pj_actor, W2, nullptr, 1 << 30, 256, 0, 0, nat(256), nat(256), 8, 8, &a->actor.W2, 1);
      M(&a->pj_actor, Wp, Ws, aout, 256, 0, 0, nat(2 * aout), nat(256), blocks_of(2 * aout), 8, &a->actor.Wh, 1);
      M(&a->pj_actor, W2, nullptr, 1 << 30, 256, 1, 0, nat(256), nat(256), 8, 8, &a->actor.W2T, 1);
      M(&a->pj_actor, Wp, Ws, aout, 256, 1, 0, nat(256), pair(aout), 8, (aout + 15) / 16, &a->actor.WhT);
      if (a->cfg.mlp_bf16)  // the two-tile bf16 critic phase squashes in the heads' epilogue (sac_bf.h)
        M(&a->pj_actor, Wp, Ws, aout, 256, 0, 0, pair(aout), nat(256), (aout + 15) / 16, 8, &a->actor.WhP, 1);
      a->actor.tb1 = T(b1, 256);
      a->actor.tb2 = T(b2, 256);
      a->actor.tbh = T(bp, aout, bs, aout);
    }
  } else {
    // ---- DDPG actor and its target (ddpg/models.py:5-22): fc1 [256][ob], fc2, fc3 [aout][256]
    for (int t = 0; t < 2; ++t) {
      const float* P = a->net[t == 0 ? SPP_NET_ACTOR : SPP_NET_ACTOR_TARG].p;
      ActorDev& ad = t == 0 ? a->actor : a->actor_targ;
      std::vector<PackJob>* l = t == 0 ? &a->pj_actor : &a->pj_targ;
      const float *W1 = P, *b1 = W1 + 256 * ob, *W2 = b1 + 256, *b2 = W2 + 65536, *W3 = b2 + 256, *b3 = W3 + aout * 256;
      M(l, W1, nullptr, 1 << 30, ob, 0, 0, nat(256), nat(ob), 8, blocks_of(ob), &ad.W1);
      M(l, W2, nullptr, 1 << 30, 256, 0, 0, nat(256), nat(256), 8, 8, &ad.W2, 1);
      M(l, W3, nullptr, 1 << 30, 256, 0, 0, nat(aout), nat(256), blocks_of(aout), 8, &ad.Wh, 1);
      if (t == 0) {
        M(l, W2, nullptr, 1 << 30, 256, 1, 0, nat(256), nat(256), 8, 8, &ad.W2T, 1);
        M(l, W3, nullptr, 1 << 30, 256, 1, 0, nat(256), nat(aout), 8, blocks_of(aout), &ad.WhT);
      }
      ad.tb1 = T(b1, 256);
      ad.tb2 = T(b2, 256);
      ad.tbh = T(b3, aout);
    }
  }
  if (!a->ddpg) {
    // ---- ACM (basic_model.py:108-117): fc1 [64][2ob], fc2 [32][64], fc3 [ac][32]
    {
      const float* P = a->net[SPP_NET_ACM].p;
      const int in = 2 * ob;
      const float *W1 = P, *b1 = W1 + 64 * in, *W2 = b1 + 64, *b2 = W2 + 32 * 64, *W3 = b2 + 32, *b3 = W3 + ac * 32;
      M(&a->pj_acm, W1, nullptr, 1 << 30, in, 0, 0, nat(64), cat(ob, aout), 2, blocks_of(ob) + blocks_of(aout),
        &a->acm.W1);
      M(&a->pj_acm, W2, nullptr, 1 << 30, 64, 0, 0, nat(32), nat(64), 1, 2, &a->acm.W2);
      M(&a->pj_acm, W3, nullptr, 1 << 30, 32, 0, 0, nat(ac), nat(32), 1, 1, &a->acm.W3);
      M(&a->pj_acm, W3, nullptr, 1 << 30, 32, 1, 0, nat(32), nat(ac), 1, 1, &a->acm.W3T);
      M(&a->pj_acm, W2, nullptr, 1 << 30, 64, 1, 0, nat(64), nat(32), 2, 1, &a->acm.W2T);
      M(&a->pj_acm, W1, nullptr, 1 << 30, in, 1, ob, nat(aout), nat(64), blocks_of(aout), 2, &a->acm.W1Ta);
      M(&a->pj_acm, W1, nullptr, 1 << 30, in, 0, 0, nat(64), nat(in), 2, blocks_of(in), &a->acm_W1n);
      a->acm.tb1 = T(b1, 64);
      a->acm.tb2 = T(b2, 32);
      a->acm.tb3 = T(b3, ac);
    }
  } else {
    // ---- BasicAcM (acm/models/basic_acm.py:11-21): t, t1, fc1 [100][2ob], fc2 [50][100],
    //      fc21 [50][2ob], fc3 [ac][50]
    const float* P = a->net[SPP_NET_ACM].p;
    const int in = 2 * ob;
    const float *t = P, *t1 = P + 1, *W1 = t1 + ac, *b1 = W1 + 100 * in, *W2 = b1 + 100, *b2 = W2 + 50 * 100,
                *W21 = b2 + 50, *b21 = W21 + 50 * in, *W3 = b21 + 50, *b3 = W3 + ac * 50;
    BAcmDev& B = a->bacm;
    const int nbi = blocks_of(ob) + blocks_of(aout);
    M(&a->pj_acm, W1, nullptr, 1 << 30, in, 0, 0, nat(100), cat(ob, aout), 4, nbi, &B.W1);
    M(&a->pj_acm, W21, nullptr, 1 << 30, in, 0, 0, nat(50), cat(ob, aout), 2, nbi, &B.W21);
    M(&a->pj_acm, W2, nullptr, 1 << 30, 100, 0, 0, nat(50), nat(100), 2, 4, &B.W2);
    M(&a->pj_acm, W3, nullptr, 1 << 30, 50, 0, 0, nat(ac), nat(50), 1, 2, &B.W3);
    M(&a->pj_acm, W3, nullptr, 1 << 30, 50, 1, 0, nat(50), nat(ac), 2, 1, &B.W3T);
    M(&a->pj_acm, W2, nullptr, 1 << 30, 100, 1, 0, nat(100), nat(50), 4, 2, &B.W2T);
    M(&a->pj_acm, W1, nullptr, 1 << 30, in, 1, ob, nat(aout), nat(100), blocks_of(aout), 4, &B.W1Ta);
    M(&a->pj_acm, W21, nullptr, 1 << 30, in, 1, ob, nat(aout), nat(50), blocks_of(aout), 2, &B.W21Ta);
    M(&a->pj_acm, W1, nullptr, 1 << 30, in, 0, 0, nat(100), nat(in), 4, blocks_of(in), &a->bacm_W1n);
    M(&a->pj_acm, W21, nullptr, 1 << 30, in, 0, 0, nat(50), nat(in), 2, blocks_of(in), &a->bacm_W21n);
    B.tb1 = T(b1, 100);
    B.tb21 = T(b21, 50);
    B.tb2 = T(b2, 50);
    B.tb3 = T(b3, ac);
    B.t = t;
    B.t1 = t1;
  }
  // ---- critics and targets (sac/models.py:75-91): fc1 [256][cin], fc2, fc3 [1][256]
  for (int t = 0; t < 4; ++t) {
    if (a->ddpg && (t == 1 || t == 3)) continue;  // DDPG: one critic and its target
    const int netid = t < 2 ? SPP_NET_CRITIC1 + t : SPP_NET_CRITIC1_TARG + (t - 2);
    CriticDev& cd = t < 2 ? a->critic[t] : a->targ[t - 2];
    const float* P = a->net[netid].p;
    const float *W1 = P, *b1 = W1 + 256 * cin, *W2 = b1 + 256, *b2 = W2 + 65536, *w3 = b2 + 256, *b3 = w3 + 256;
    std::vector<PackJob>* fl = t < 2 ? &a->pj_critic_fwd : &a->pj_targ;
    M(fl, W1, nullptr, 1 << 30, cin, 0, 0, nat(256), cat(ob, ca), 8, blocks_of(ob) + blocks_of(ca), &cd.W1);
    M(fl, W2, nullptr, 1 << 30, 256, 0, 0, nat(256), nat(256), 8, 8, &cd.W2, 1);
    if (t < 2) {
      M(fl, W2, nullptr, 1 << 30, 256, 1, 0, nat(256), nat(256), 8, 8, &cd.W2T, 1);
      M(fl, W1, nullptr, 1 << 30, cin, 1, ob, nat(ca), nat(256), blocks_of(ca), 8, &cd.W1Ta, 1);
    }
    cd.tb1 = T(b1, 256);
    cd.tb2 = T(b2, 256);
    cd.tw3 = T(w3, 256);
    cd.b3 = b3;
  }
  // + the per-launch limit / normaliser segments appended by make_args
  a->tab_floats = toff;
  const int extra = 3 * (int)round_up(aout, 32) + (int)round_up(std::max(ac, 1), 32);
  SPP_REQUIRE(toff + extra <= kTabMax && (int)a->tab.size() + 4 <= kTabSegs, SPP_E_SHAPE,
              "LDS table too large (%d floats, %d segments)", toff + extra, (int)a->tab.size() + 4);
  // allocate images
  size_t nf4 = 0;
  for (auto& m : ms) nf4 += (size_t)m.job.NBO * m.job.NBI * 4 * 64;
  a->pk.release();
  SPP_CHECK_HIP(a->pk.alloc(nf4));
  size_t of = 0;
  for (auto& m : ms) {
    m.job.dst = a->pk.ptr + of;
    *m.slot = m.job.dst;
    of += (size_t)m.job.NBO * m.job.NBI * 4 * 64;
    m.list->push_back(m.job);
  }
  // critics: "all" list = fwd list (already includes transposes)
  a->pj_critic_all = a->pj_critic_fwd;
  // device job tables: [actor | acm | targ | critic]
  std::vector<PackJob> all;
  a->o_actor = (int)all.size(); all.insert(all.end(), a->pj_actor.begin(), a->pj_actor.end());
  a->o_acm = (int)all.size(); all.insert(all.end(), a->pj_acm.begin(), a->pj_acm.end());
  a->o_targ = (int)all.size(); all.insert(all.end(), a->pj_targ.begin(), a->pj_targ.end());
  a->o_cfwd = (int)all.size(); all.insert(all.end(), a->pj_critic_fwd.begin(), a->pj_critic_fwd.end());
  a->d_pj.release();
  SPP_CHECK_HIP(a->d_pj.alloc(all.size()));
  SPP_CHECK_HIP(hipMemcpy(a->d_pj.ptr, all.data(), sizeof(PackJob) * all.size(), hipMemcpyHostToDevice));
  return SPP_OK;
}

static void launch_pack(sppAgent* a, int off, int n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_pack_matrix, dim3(64, n), dim3(256), 0, st, (const PackJob*)(a->d_pj.ptr + off));
}

// bf16 sets' 256 x 256 bf16-operand weight gradients on the LDS-staged k_dw_big16 (0: k_dw<true>, the A/B)
#ifndef SPP_DW_BIG16
#define SPP_DW_BIG16 1
#endif
// Split assignment, slab arena, item table and upload of a job set.
static sppStatus finalize_dw(DwSet& D, std::vector<DwJob>& jobs, int nph, int Bp, int B, int num_cu) {
  // Sample splits: the large (>= 128x128 padded) GEMMs of a phase share ~one
  // workgroup per CU in proportion to their MACs; the small, HBM-bound ones
  // take 2048-sample items.
  auto is_big = [](const DwJob& j) {
    return (int64_t)round_up(j.N, 32) * round_up(j.K0 + j.K1, 32) >= 128 * 128;
  };
  // 256 x 256 fp32 jobs run as their own launch (k_dw_big); the other large jobs share k_dw's launch
  // (small batches -- vanilla SAC's B = 100, PPO minibatches -- keep one launch: k_dw's register tiles)
  // (bf16 sets: the 256 x 256 jobs whose A and X rows are both bf16 run as k_dw_big16, in 64-sample steps)
  auto lds_big = [Bp](const DwJob& j) {
    return Bp >= 8192 && j.N == 256 && j.K0 == 256 && j.K1 == 0 &&
           (!j.bf16 || (SPP_DW_BIG16 && j.a_bf && j.x_bf && Bp % 64 == 0));
  };
  auto assign_splits = [&](int first, int count) {
    double big[2] = {0.0, 0.0};  // MACs of the large jobs per launch
    for (int i = first; i < first + count; ++i)
      if (!jobs[i].fused && is_big(jobs[i]))
        big[lds_big(jobs[i]) ? 0 : 1] += (double)round_up(jobs[i].N, 32) * round_up(jobs[i].K0 + jobs[i].K1, 32);
    for (int i = first; i < first + count; ++i) {
      DwJob& j = jobs[i];
      if (j.fused) continue;  // nsplit = the phase kernel's waves, set by the caller
      const double pm = (double)round_up(j.N, 32) * round_up(j.K0 + j.K1, 32);
      // outputs that fit one 128x128 wave quadrant: the 4 waves split each item's samples
      const bool thin_n = j.N <= 128, thin_k = j.K0 + j.K1 <= 128;
      j.wsplit = thin_n && thin_k ? 4 : (thin_n != thin_k ? 2 : 1);
      // large jobs: ~one workgroup per CU over their launch, in proportion to their MACs; small jobs:
      // >= 2048 samples per item, and at most ~256 slabs (the fixed-order reduce is serial over slabs)
      int ns = is_big(j) ? (int)std::lround(num_cu * pm / big[lds_big(j) ? 0 : 1])
                         : std::min(cdiv(Bp, 2048), std::max(1, 256 / j.wsplit));
      // small batches (PPO minibatches of 512): at least 4 items, so each wave of an item takes one
      // 32-sample unit instead of a serial chain over the whole batch
      if (!is_big(j)) ns = std::max(ns, std::min(cdiv(Bp, 32 * j.wsplit), 4));
      ns = std::max(1, std::min(ns, std::max(1, Bp / 32)));
      j.split_len = (int)round_up(cdiv(Bp, ns), lds_big(j) && j.bf16 ? 64 : 32 * j.wsplit);
      j.nsplit = cdiv(Bp, j.split_len);
    }
  };
  for (int ph = 0; ph < nph; ++ph) assign_splits(D.j0[ph], D.nj[ph]);
  // slabs: phases run back to back on one stream -> they share one arena
  size_t need = 0;
  for (int ph = 0; ph < nph; ++ph) {
    size_t off = 0;
    for (int j = D.j0[ph]; j < D.j0[ph] + D.nj[ph]; ++j) {
      if (jobs[j].nsplit * jobs[j].wsplit > 1) {
        jobs[j].slab = nullptr;
        off += (size_t)jobs[j].nsplit * jobs[j].wsplit * jobs[j].slab_stride;
      }
    }
    need = std::max(need, off);
  }
  if (need > D.slab.n) {
    D.slab.release();
    SPP_CHECK_HIP(D.slab.alloc(need));
  }
  std::vector<int> items;
  for (int ph = 0; ph < nph; ++ph) {
    size_t off = 0;
    std::vector<int> jj, ss;
    for (int j = D.j0[ph]; j < D.j0[ph] + D.nj[ph]; ++j) {
      if (jobs[j].nsplit * jobs[j].wsplit > 1) {
        jobs[j].slab = D.slab.ptr + off;
        off += (size_t)jobs[j].nsplit * jobs[j].wsplit * jobs[j].slab_stride;
      }
    }
    // large-GEMM items first (they set the phase's critical path): the 256 x 256 fp32 jobs (k_dw_big,
    // LDS-DMA operands), then the other large ones, then the thin ones (k_dw)
    D.nlds[ph] = 0;
    for (int pass = 0; pass < 3; ++pass)
      for (int j = D.j0[ph]; j < D.j0[ph] + D.nj[ph]; ++j) {
        const int cls = lds_big(jobs[j]) ? 0 : (is_big(jobs[j]) ? 1 : 2);
        if (cls != pass || jobs[j].fused) continue;
        for (int sp = 0; sp < jobs[j].nsplit; ++sp) {
          jj.push_back(j - D.j0[ph]);
          ss.push_back(sp);
          if (pass == 0) ++D.nlds[ph];
        }
      }
    D.max_elems[ph] = 1;
    for (int j = D.j0[ph]; j < D.j0[ph] + D.nj[ph]; ++j) {
      const int64_t el = (int64_t)jobs[j].N * (jobs[j].K0 + jobs[j].K1) + jobs[j].N;
      D.max_elems[ph] = std::max<int64_t>(D.max_elems[ph], el * dw_red_group(jobs[j].nsplit * jobs[j].wsplit, el));
    }
    D.ioff[ph] = (int)items.size();
    D.nitems[ph] = (int)jj.size();
    items.insert(items.end(), jj.begin(), jj.end());
    items.insert(items.end(), ss.begin(), ss.end());
  }
  D.jobs.release();
  D.items.release();
  SPP_CHECK_HIP(D.jobs.alloc(jobs.size()));
  SPP_CHECK_HIP(D.items.alloc(items.size()));
  SPP_CHECK_HIP(hipMemcpy(D.jobs.ptr, jobs.data(), sizeof(DwJob) * jobs.size(), hipMemcpyHostToDevice));
  SPP_CHECK_HIP(hipMemcpy(D.items.ptr, items.data(), sizeof(int) * items.size(), hipMemcpyHostToDevice));
  D.B = B;
  D.bf16 = !jobs.empty() && jobs[0].bf16;
  for (const DwJob& j : jobs)
    if ((j.bf16 != 0) != D.bf16) return SPP_E_STATE;
  return SPP_OK;
}

// (Re)build a weight-gradient job set for batch size B.
//   set 0: SAC (phase 0 = both critics, phase 1 = actor); set 1: ACM regression
static int phase_grid(sppAgent* a, int Bp);
static int sac_grid(sppAgent* a, int Bp);
static int sac_critic_grid(sppAgent* a, int Bp);
static bool sac_team(sppAgent* a, int Bp);
static sppStatus build_dw(sppAgent* a, int set, int B) {
  const int Bp = (int)round_up(B, 32);
  const int ob = a->cfg.ob, aout = a->cfg.aout, ac = a->cfg.ac;
  const int ca = a->cfg.acm_critic ? ac : aout, cin = ob + ca;
  std::vector<DwJob> jobs;
  // bf16 SAC kernel sets write these operand arrays as bf16 (op_st, sac.hip)
  std::vector<const float*> b16;
  if (a->cfg.mlp_bf16 && !a->ddpg && set == 0)
    b16 = {a->H1[0], a->H1[1], a->H2[0], a->H2[1], a->D1[0], a->D1[1], a->D2[0], a->D2[1],
           a->AH1, a->AH2, a->AD1, a->AD2};
  auto is16 = [&](const float* p) { return p && std::find(b16.begin(), b16.end(), p) != b16.end(); };
  // rows >= nrow2 of a job go to (dW2, db2)
  auto J = [&](const float* A, int N, const float* X0, int K0, const float* X1, int K1, float* dW, float* db,
               int nrow2 = -1, float* dW2 = nullptr, float* db2 = nullptr) {
    DwJob j{};
    j.A = A; j.N = N; j.X0 = X0; j.K0 = K0; j.X1 = X1; j.K1 = K1; j.dW = dW; j.db = db; j.Bp = Bp;
    j.nrow2 = nrow2 < 0 ? N : nrow2;
    j.dW2 = dW2; j.db2 = db2;
    j.slab_stride = round_up((int64_t)N * (K0 + K1) + N, 4);
    j.bf16 = a->cfg.mlp_bf16 ? 1 : 0;
    j.a_bf = is16(A) ? 1 : 0;
    j.x_bf = is16(X0) ? 1 : 0;
    jobs.push_back(j);  // (an X1 segment is always staged fp32 input, like X0)
  };
  DwSet& D = a->dws[set];
  int nph = 0;
  if (a->ddpg) {
    if (set == 0) {
      // critic phase (ddpg_acm.py:174-185): fc1 (delta1 x [s|a]), fc2 (delta2 x h1), fc3 (dq x h2)
      float* G = a->net[SPP_NET_CRITIC1].g;
      float *gW1 = G, *gb1 = gW1 + 256 * cin, *gW2 = gb1 + 256, *gb2 = gW2 + 65536, *gw3 = gb2 + 256, *gb3 = gw3 + 256;
      J(a->D1[0], 256, a->S, ob, a->cfg.acm_critic ? a->AENV : a->ACT, ca, gW1, gb1);
      J(a->D2[0], 256, a->H1[0], 256, nullptr, 0, gW2, gb2);
      int fused0 = -1;
      if (ob <= 32) {  // fc3: fused into k_ddpg_critic_phase (reduce only; its kFuse3)
        J(nullptr, 1, nullptr, 256, nullptr, 0, gw3, gb3);
        jobs.back().fused = 1;
        jobs.back().nsplit = phase_grid(a, Bp) * kWavesPerWG;
        jobs.back().wsplit = 1;
        fused0 = (int)jobs.size() - 1;
      } else {
        J(a->DQ[0], 1, a->H2[0], 256, nullptr, 0, gw3, gb3);
      }
      D.j0[0] = 0;
      D.nj[0] = (int)jobs.size();
      // actor phase (:187-196): fc1 (delta1 x s), fc2 (delta2 x h1), fc3 (dhead x h2)
      float* A = a->net[SPP_NET_ACTOR].g;
      float *aW1 = A, *ab1 = aW1 + 256 * ob, *aW2 = ab1 + 256, *ab2 = aW2 + 65536, *aW3 = ab2 + 256,
            *ab3 = aW3 + aout * 256;
      J(a->AD1, 256, a->S, ob, nullptr, 0, aW1, ab1);
      J(a->AD2, 256, a->AH1, 256, nullptr, 0, aW2, ab2);
      J(a->ADH, aout, a->AH2, 256, nullptr, 0, aW3, ab3);
      D.j0[1] = D.nj[0];
      D.nj[1] = (int)jobs.size() - D.nj[0];
      nph = 2;
      sppStatus s = finalize_dw(D, jobs, nph, Bp, B, a->num_cu);
      a->w3p[0] = a->w3p[1] = fused0 >= 0 ? jobs[fused0].slab : nullptr;
      a->w3p_stride = fused0 >= 0 ? jobs[fused0].slab_stride : 0;
      return s;
    } else {
      // BasicAcM regression (acm.py:246-258): fc1, fc2, fc21 (grad of its output = t * dz), fc3;
      // t / t1 come from the per-tile partials (k_finalize_bacm)
      float* G = a->net[SPP_NET_ACM].g;
      const int in = 2 * ob;
      float *gW1 = G + 1 + ac, *gb1 = gW1 + 100 * in, *gW2 = gb1 + 100, *gb2 = gW2 + 50 * 100, *gW21 = gb2 + 50,
            *gb21 = gW21 + 50 * in, *gW3 = gb21 + 50, *gb3 = gW3 + ac * 50;
      J(a->RBP1, 100, a->RX, in, nullptr, 0, gW1, gb1);
      J(a->RPZ, 50, a->RBH, 100, nullptr, 0, gW2, gb2);
      J(a->RPZ21, 50, a->RX, in, nullptr, 0, gW21, gb21);
      J(a->RP3, ac, a->RBH1, 50, nullptr, 0, gW3, gb3);
      D.j0[0] = 0;
      D.nj[0] = (int)jobs.size();
      nph = 1;
    }
  } else if (set == 0) {
    // critic phase: fc1 (delta1 x [s|a]), fc2 (delta2 x h1) per critic; fc3 (dq x h2) is fused into the
    // critic-phase kernel, which writes one [256 | 1] partial per wave: a reduce-only job
    // (bf16 sets with SPP_BF16_FUSE3 = 0: the critic phase stores h2 (bf16) and dq; fc3 is a k_dw job)
    const bool fuse3 = !a->cfg.mlp_bf16 || SPP_BF16_FUSE3;
    int fused_idx[2] = {-1, -1};
    for (int i = 0; i < 2; ++i) {
      float* G = a->net[SPP_NET_CRITIC1 + i].g;
      float *gW1 = G, *gb1 = gW1 + 256 * cin, *gW2 = gb1 + 256, *gb2 = gW2 + 65536, *gw3 = gb2 + 256, *gb3 = gw3 + 256;
      J(a->D1[i], 256, a->S, ob, a->cfg.acm_critic ? a->AENV : a->ACT, ca, gW1, gb1);
      J(a->D2[i], 256, a->H1[i], 256, nullptr, 0, gW2, gb2);
      if (!fuse3) {
        J(a->DQ[i], 1, a->H2[i], 256, nullptr, 0, gw3, gb3);
        continue;
      }
      J(nullptr, 1, nullptr, 256, nullptr, 0, gw3, gb3);
      jobs.back().fused = 1;
      jobs.back().nsplit = sac_critic_grid(a, Bp) * (sac_team(a, Bp) ? kTeamCritic : kWavesPerWG);
      jobs.back().wsplit = 1;
      fused_idx[i] = (int)jobs.size() - 1;
    }
    D.j0[0] = 0;
    D.nj[0] = (int)jobs.size();
    float* G = a->net[SPP_NET_ACTOR].g;
    float *gW1 = G, *gb1 = gW1 + 256 * ob, *gW2 = gb1 + 256, *gb2 = gW2 + 65536, *gWp = gb2 + 256,
          *gbp = gWp + aout * 256, *gWs = gbp + aout, *gbs = gWs + aout * 256;
    J(a->AD1, 256, a->S, ob, nullptr, 0, gW1, gb1);
    J(a->AD2, 256, a->AH1, 256, nullptr, 0, gW2, gb2);
    J(a->ADH, 2 * aout, a->AH2, 256, nullptr, 0, gWp, gbp, aout, gWs, gbs);  // [mu | log-std] heads
    D.j0[1] = D.nj[0];
    D.nj[1] = (int)jobs.size() - D.nj[0];
    nph = 2;
    sppStatus s = finalize_dw(D, jobs, nph, Bp, B, a->num_cu);
    for (int i = 0; i < 2; ++i) a->w3p[i] = fuse3 ? jobs[fused_idx[i]].slab : nullptr;
    a->w3p_stride = fuse3 ? jobs[fused_idx[0]].slab_stride : 0;
    return s;
  } else {
    float* G = a->net[SPP_NET_ACM].g;
    const int in = 2 * ob;
    float *gW1 = G, *gb1 = gW1 + 64 * in, *gW2 = gb1 + 64, *gb2 = gW2 + 32 * 64, *gW3 = gb2 + 32, *gb3 = gW3 + ac * 32;
    J(a->RP1, 64, a->RX, in, nullptr, 0, gW1, gb1);
    J(a->RP2, 32, a->RZ1, 64, nullptr, 0, gW2, gb2);
    J(a->RP3, ac, a->RZ2, 32, nullptr, 0, gW3, gb3);
    D.j0[0] = 0;
    D.nj[0] = (int)jobs.size();
    nph = 1;
  }
  return finalize_dw(D, jobs, nph, Bp, B, a->num_cu);
}


static void launch_dw_set(DwSet& D, int ph, hipStream_t st) {
  const int* ij = D.items.ptr + D.ioff[ph];
  const int* is = ij + D.nitems[ph];
  const DwJob* jobs = D.jobs.ptr + D.j0[ph];
  launch_dw_kernels(jobs, ij, is, D.nitems[ph], D.nlds[ph], D.nj[ph], D.max_elems[ph], D.bf16, st);
}
static void launch_dw(sppAgent* a, int set, int ph, hipStream_t st) { launch_dw_set(a->dws[set], ph, st); }

// Adam job table [critic1, critic2 (+polyak targets) | actor | acm]; pointers only.
// DDPG_AcM: [critic (+polyak) | - | actor (+polyak of the target actor, ddpg.py:273-284) | acm].
static sppStatus build_adam(sppAgent* a) {
  AdamJob jobs[4] = {};
  for (int i = 0; i < (a->ddpg ? 1 : 2); ++i) {
    NetBufs& n = a->net[SPP_NET_CRITIC1 + i];
    jobs[i] = AdamJob{n.p, n.g, n.m, n.v, a->net[SPP_NET_CRITIC1_TARG + i].p, n.n};
  }
  NetBufs& na = a->net[SPP_NET_ACTOR];
  jobs[2] = AdamJob{na.p, na.g, na.m, na.v, a->ddpg ? a->net[SPP_NET_ACTOR_TARG].p : nullptr, na.n};
  NetBufs& nm = a->net[SPP_NET_ACM];
  jobs[3] = AdamJob{nm.p, nm.g, nm.m, nm.v, nullptr, nm.n};
  if (!a->d_adam.ptr) SPP_CHECK_HIP(a->d_adam.alloc(4));
  SPP_CHECK_HIP(hipMemcpy(a->d_adam.ptr, jobs, sizeof(jobs), hipMemcpyHostToDevice));
  return SPP_OK;
}

static void launch_adam(sppAgent* a, int first, int count, int64_t n, int64_t step, float lr, float tau,
                        hipStream_t st) {
  const double bc1 = 1.0 - std::pow(0.9, (double)step), bc2s = std::sqrt(1.0 - std::pow(0.999, (double)step));
  hipLaunchKernelGGL(k_adam, dim3(std::max(1, std::min(cdiv(n, 256 * 4), 1024)), count), dim3(256), 0, st,
                     (const AdamJob*)(a->d_adam.ptr + first), (float)(-(lr / bc1)), (float)bc2s, tau);
}

static SacArgs make_args(sppAgent* a, int B) {
  SacArgs p{};
  p.B = B;
  p.Bp = (int)round_up(B, 32);
  p.inv_B = 1.f / (float)B;
  p.S = a->S; p.S2 = a->S2; p.ACT = a->ACT; p.AENV = a->AENV; p.R = a->R; p.DN = a->DN;
  p.EPS1 = a->EPS1; p.EPS2 = a->EPS2;
  p.min_max = a->cfg.min_max_denormalize;
  p.lo = a->lo; p.hi = a->hi; p.mean = a->mean; p.std = a->std;
  p.actor_lim = a->limits.ptr;
  p.acm_lim = a->limits.ptr + a->cfg.aout;
  p.gamma = a->cfg.gamma;
  p.custom_loss = a->cfg.custom_loss;
  p.norm_closs = a->cfg.norm_closs;
  p.alpha = a->alpha_f32;
  p.actor = a->actor;
  for (int i = 0; i < 2; ++i) {
    p.critic[i] = a->critic[i];
    p.targ[i] = a->targ[i];
    p.H1[i] = a->H1[i]; p.H2[i] = a->H2[i]; p.D1[i] = a->D1[i]; p.D2[i] = a->D2[i]; p.DQ[i] = a->DQ[i];
    p.W3P[i] = a->w3p[i];
  }
  p.w3p_stride = a->w3p_stride;
  p.acm = a->acm;
  p.bacm = a->bacm;
  p.actor_targ = a->actor_targ;
  p.AH1 = a->AH1; p.AH2 = a->AH2; p.AD1 = a->AD1; p.AD2 = a->AD2; p.ADH = a->ADH;
  p.part = a->part;
  p.nseg = (int)a->tab.size();
  for (int i = 0; i < p.nseg; ++i) p.seg[i] = a->tab[i];
  // limits and normaliser vectors (read per output slot by the squash / head epilogues: LDS
  // instead of a global round trip each); unbound vectors read as zeros
  int off = a->tab_floats;
  auto X = [&](const float* v, int n) {
    const int o = off, np = (int)round_up(std::max(n, 1), 32);
    p.seg[p.nseg++] = TabSeg{v ? v : a->limits.ptr, v ? n : 0, np, o, 0};
    off += np;
    return o;
  };
  const int aout = a->cfg.aout;
  p.t_lim = X(a->limits.ptr, aout);
  p.t_alim = X(a->limits.ptr + aout, a->cfg.ac);
  p.t_n0 = X(p.min_max ? a->lo : a->mean, aout);
  p.t_n1 = X(p.min_max ? a->hi : a->std, aout);
  return p;
}

static int phase_grid(sppAgent* a, int Bp) {
  const int ntiles = Bp / 32;
  return std::max(1, std::min(cdiv(ntiles, kWavesPerWG), a->num_cu));
}
// SAC phases: the team kernels (one workgroup per tile, sac_team.h) while the tiles fit one per CU
static bool sac_team(sppAgent* a, int Bp) {
  return a->ks.critic_team && a->ks.actor_team && a->team_ok && Bp / 32 <= a->num_cu;
}
static int sac_grid(sppAgent* a, int Bp) {
  return sac_team(a, Bp) ? std::max(1, std::min(Bp / 32, a->num_cu)) : phase_grid(a, Bp);
}
// the team critic phase splits each tile's two critics over two workgroups while 2 x tiles fit the CUs
static int sac_critic_grid(sppAgent* a, int Bp) {
  const int nt = std::max(1, Bp / 32);
  return sac_team(a, Bp) && 2 * nt <= a->num_cu ? 2 * nt : sac_grid(a, Bp);
}

static sppStatus check_ready(sppAgent* a) {
  SPP_REQUIRE(a->ddpg || (a->alpha_state && a->alpha_f32), SPP_E_STATE, "alpha not bound");
  SPP_REQUIRE(a->cfg.min_max_denormalize ? (a->lo && a->hi) : (a->mean && a->std), SPP_E_STATE,
              "normalizer not bound");
  SPP_REQUIRE(a->limits.ptr, SPP_E_STATE, "limits not set");
  if (!a->pk.ptr) {
    sppStatus s = build_packs(a);
    if (s) return s;
    if ((s = build_adam(a))) return s;
    a->dws[0].B = a->dws[1].B = -1;
  }
  return SPP_OK;
}

extern "C" {

sppStatus sppAgentCreate(sppAgentHandle* out, const sppAgentConfig* cfg, int device) {
  SPP_REQUIRE(out && cfg, SPP_E_INVALID_ARG, "null arg");
  SPP_REQUIRE(cfg->algo == SPP_ALGO_SAC_ACM || cfg->algo == SPP_ALGO_DDPG_ACM || cfg->algo == SPP_ALGO_SAC,
              SPP_E_INVALID_ARG, "unsupported algo %d", cfg->algo);
  SPP_REQUIRE(cfg->algo != SPP_ALGO_SAC || (cfg->acm_critic == 0 && cfg->aout == cfg->ac && cfg->custom_loss == 0.f),
              SPP_E_INVALID_ARG, "vanilla SAC: the actor emits the env action (aout == ac), no ACM critic / loss");
  SPP_REQUIRE(cfg->max_batch > 0, SPP_E_INVALID_ARG, "max_batch must be > 0");
  KernelSet ks;
  SPP_REQUIRE(find_kset(cfg->algo, cfg->ob, cfg->aout, cfg->ac, cfg->acm_critic != 0, cfg->mlp_bf16 != 0, &ks),
              SPP_E_SHAPE, "no kernel instantiation for algo %d (ob=%d, aout=%d, ac=%d, bf16=%d)", cfg->algo, cfg->ob,
              cfg->aout, cfg->ac, cfg->mlp_bf16);
  SPP_CHECK_HIP(hipSetDevice(device));
  auto a = std::make_unique<sppAgent>();
  a->cfg = *cfg;
  a->device = device;
  a->ks = ks;
  hipDeviceProp_t prop;
  SPP_CHECK_HIP(hipGetDeviceProperties(&prop, device));
  a->num_cu = prop.multiProcessorCount;
  {
    const char* t = getenv("SPP_SAC_TEAM");
    a->team_ok = !(t && t[0] == '0');
  }
  const int ob = cfg->ob, aout = cfg->aout, ac = cfg->ac;
  a->cin = ob + (cfg->acm_critic ? ac : aout);
  a->ddpg = cfg->algo == SPP_ALGO_DDPG_ACM;
  a->plain = cfg->algo == SPP_ALGO_SAC;
  const bool dd = a->ddpg;
  a->nsize[SPP_NET_ACTOR] = dd ? ddpg_actor_size(ob, aout) : sac_actor_size(ob, aout);
  a->nsize[SPP_NET_ACTOR_TARG] = dd ? ddpg_actor_size(ob, aout) : 0;
  a->nsize[SPP_NET_CRITIC1] = a->nsize[SPP_NET_CRITIC1_TARG] = critic_size(a->cin);
  a->nsize[SPP_NET_CRITIC2] = a->nsize[SPP_NET_CRITIC2_TARG] = dd ? 0 : critic_size(a->cin);
  a->nsize[SPP_NET_ACM] = dd ? bacm_size(2 * ob, ac) : acm_size(2 * ob, ac);
  a->Bmax = cfg->max_batch;
  const int64_t Bp = round_up(cfg->max_batch, 32);
  SPP_REQUIRE((int64_t)Bp * 256 * 4 < ((int64_t)1 << 31), SPP_E_SHAPE, "max_batch %d too large (31-bit buffer offsets)",
              cfg->max_batch);
  a->Bpmax = (int)Bp;
  const int64_t ntiles = Bp / 32;
  // scratch arena
  const int64_t per = Bp;
  int64_t total = 0;
  auto take = [&](int64_t rows) { int64_t o = total; total += rows * per; return o; };
  const int64_t oS = take(ob), oS2 = take(ob), oACT = take(aout), oAENV = take(ac), oR = take(1), oDN = take(1),
                oE1 = take(aout), oE2 = take(aout);
  int64_t oH1[2] = {}, oH2[2] = {}, oD1[2] = {}, oD2[2] = {}, oDQ[2] = {};
  for (int i = 0; i < (dd ? 1 : 2); ++i) {
    oH1[i] = take(256); oH2[i] = take(256); oD1[i] = take(256); oD2[i] = take(256); oDQ[i] = take(1);
  }
  const int64_t oAH1 = take(256), oAH2 = take(256), oAD1 = take(256), oAD2 = take(256), oADH = take(2 * aout);
  // ACM activations kept for its backward: AcM z1 [64], z2 [32], t3 [ac]; BasicAcM h [128], h1 [64], r3 [ac]
  const int64_t oZ1 = take(dd ? 128 : 64), oZ2 = take(dd ? 64 : 32), oT3 = take(ac);
  const int64_t oRX = take(2 * ob), oRZ1 = take(dd ? 128 : 64), oRZ2 = take(dd ? 64 : 32), oRP1 = take(dd ? 128 : 64),
                oRP2 = take(dd ? 64 : 32), oRP3 = take(ac);
  const int64_t oRS21 = dd ? take(64) : 0, oRPZ21 = dd ? take(64) : 0;
  // wide-head actor phase hand-over: d a_d [aout][Bp], ReLU masks (4 x u64 per lane = 16 floats per sample)
  const int64_t oGAD = take(aout), oMASK = take(16);
  const int64_t oPart = total;
  total += ntiles * kBParts + 64;
  const int64_t oAux = total;
  total += 16;
  hipError_t e = a->scratch.alloc(total);
  if (e != hipSuccess) {
    set_error("scratch alloc %.2f GB: %s", total * 4.0 / 1e9, hipGetErrorString(e));
    return SPP_E_OOM;
  }
  SPP_CHECK_HIP(hipMemset(a->scratch.ptr, 0, sizeof(float) * total));
  float* b = a->scratch.ptr;
  a->S = b + oS; a->S2 = b + oS2; a->ACT = b + oACT; a->AENV = b + oAENV; a->R = b + oR; a->DN = b + oDN;
  a->EPS1 = b + oE1; a->EPS2 = b + oE2;
  for (int i = 0; i < 2; ++i) {
    a->H1[i] = b + oH1[i]; a->H2[i] = b + oH2[i]; a->D1[i] = b + oD1[i]; a->D2[i] = b + oD2[i]; a->DQ[i] = b + oDQ[i];
  }
  a->AH1 = b + oAH1; a->AH2 = b + oAH2; a->AD1 = b + oAD1; a->AD2 = b + oAD2; a->ADH = b + oADH;
  a->Z1 = b + oZ1; a->Z2 = b + oZ2; a->T3 = b + oT3;
  a->GAD = b + oGAD;
  a->MASK = reinterpret_cast<uint64_t*>(b + oMASK);
  a->RX = b + oRX; a->RZ1 = b + oRZ1; a->RZ2 = b + oRZ2; a->RP1 = b + oRP1; a->RP2 = b + oRP2; a->RP3 = b + oRP3;
  if (dd) {
    a->bz = BAcmScratch{a->Z1, a->Z2, a->T3};
    a->RBH = a->RZ1; a->RBH1 = a->RZ2; a->RBP1 = a->RP1; a->RPZ = a->RP2;
    a->RS21 = b + oRS21; a->RPZ21 = b + oRPZ21;
  }
  a->part = b + oPart;
  a->aux = b + oAux;
  SPP_CHECK_HIP(a->limits.alloc(aout + ac));
  *out = a.release();
  return SPP_OK;
}

sppStatus sppAgentDestroy(sppAgentHandle a) {
  if (!a) return SPP_OK;
  hipSetDevice(a->device);
  hipDeviceSynchronize();
  a->limits.release(); a->pk.release(); a->d_pj.release();
  for (auto& v : a->tev)
    for (auto e : v) hipEventDestroy(e);
  a->scratch.release(); a->d_adam.release();
  for (auto& D : a->dws) D.release();
  delete a;
  return SPP_OK;
}

sppStatus sppAgentNetSize(sppAgentHandle a, int net, int64_t* n) {
  SPP_REQUIRE(a && n && net >= 0 && net < SPP_NET_COUNT, SPP_E_INVALID_ARG, "bad net id");
  *n = a->nsize[net];
  return SPP_OK;
}

sppStatus sppAgentBindNet(sppAgentHandle a, int net, float* p, float* g, float* m, float* v) {
  SPP_REQUIRE(a && net >= 0 && net < SPP_NET_COUNT && p, SPP_E_INVALID_ARG, "bind: bad args");
  const bool trainable = net == SPP_NET_ACTOR || net == SPP_NET_CRITIC1 || net == SPP_NET_CRITIC2 || net == SPP_NET_ACM;
  SPP_REQUIRE(!trainable || (g && m && v), SPP_E_INVALID_ARG, "bind: trainable net %d needs grad/m/v", net);
  const bool changed = a->net[net].p != p || a->net[net].g != g;
  a->net[net] = NetBufs{p, g, m, v, a->nsize[net]};
  if (changed) {  // pack tables and gradient jobs hold these pointers
    a->pk.release();
    a->pj_actor.clear(); a->pj_acm.clear(); a->pj_targ.clear(); a->pj_critic_fwd.clear(); a->pj_critic_all.clear();
    a->tab.clear();
  }
  return SPP_OK;
}

sppStatus sppAgentSetLimits(sppAgentHandle a, const float* actor_lim, const float* acm_lim) {
  SPP_REQUIRE(a && actor_lim && acm_lim, SPP_E_INVALID_ARG, "null");
  SPP_CHECK_HIP(hipMemcpy(a->limits.ptr, actor_lim, sizeof(float) * a->cfg.aout, hipMemcpyHostToDevice));
  SPP_CHECK_HIP(hipMemcpy(a->limits.ptr + a->cfg.aout, acm_lim, sizeof(float) * a->cfg.ac, hipMemcpyHostToDevice));
  return SPP_OK;
}

sppStatus sppAgentBindNormalizer(sppAgentHandle a, const float* lo, const float* hi, const float* mean,
                                 const float* std) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null");
  a->lo = lo; a->hi = hi; a->mean = mean; a->std = std;
  return SPP_OK;
}

sppStatus sppAgentBindAlpha(sppAgentHandle a, double* st, float* af) {
  SPP_REQUIRE(a && st && af, SPP_E_INVALID_ARG, "null");
  a->alpha_state = st;
  a->alpha_f32 = af;
  return SPP_OK;
}

sppStatus sppAgentSetLr(sppAgentHandle a, float actor_lr, float critic_lr, float alpha_lr, float acm_lr) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null handle");
  if (actor_lr >= 0.f) a->cfg.actor_lr = actor_lr;
  if (critic_lr >= 0.f) a->cfg.critic_lr = critic_lr;
  if (alpha_lr >= 0.f) a->cfg.alpha_lr = alpha_lr;
  if (acm_lr >= 0.f) a->cfg.acm_lr = acm_lr;
  return SPP_OK;
}
sppStatus sppAgentSetSteps(sppAgentHandle a, int64_t s0, int64_t s1, int64_t s2, int64_t s3) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null");
  a->steps[0] = s0; a->steps[1] = s1; a->steps[2] = s2; a->steps[3] = s3;
  return SPP_OK;
}
sppStatus sppAgentGetSteps(sppAgentHandle a, int64_t* s) {
  SPP_REQUIRE(a && s, SPP_E_INVALID_ARG, "null");
  for (int i = 0; i < 4; ++i) s[i] = a->steps[i];
  return SPP_OK;
}

static sppStatus stage(sppAgentHandle a, const sppBatch* bt, const float* e1, const float* e2, hipStream_t st) {
  SPP_REQUIRE(bt && bt->B > 0 && bt->B <= a->Bmax, SPP_E_SHAPE, "batch B=%d outside (0, max_batch=%d]",
              bt ? bt->B : -1, a->Bmax);
  SPP_REQUIRE(bt->obs && bt->next_obs && bt->reward && bt->done && bt->acm_action, SPP_E_INVALID_ARG,
              "batch: null field");
  SPP_REQUIRE(a->cfg.acm_critic || bt->action, SPP_E_INVALID_ARG, "batch.action required without acm_critic");
  StageArgs s{};
  s.B = bt->B; s.Bp = (int)round_up(bt->B, 32); s.ob = a->cfg.ob; s.aout = a->cfg.aout; s.ac = a->cfg.ac;
  s.obs = bt->obs; s.next_obs = bt->next_obs; s.act = bt->action; s.rew = bt->reward; s.acm = bt->acm_action;
  s.done = bt->done; s.eps1 = e1; s.eps2 = e2;
  s.S = a->S; s.S2 = a->S2; s.ACT = a->ACT; s.AENV = a->AENV; s.R = a->R; s.DN = a->DN; s.EPS1 = a->EPS1;
  s.EPS2 = a->EPS2;
  hipLaunchKernelGGL(k_stage_batch, dim3(cdiv(s.Bp, 256)), dim3(256), 0, st, s);
  a->cur_B = bt->B;
  return SPP_OK;
}

static sppStatus critic_grads_staged(sppAgentHandle a, float* losses, hipStream_t st) {
  SPP_REQUIRE(!a->ddpg, SPP_E_STATE, "not a SAC_AcM agent");
  const int B = a->cur_B;
  SPP_REQUIRE(B > 0, SPP_E_STATE, "no staged batch");
  sppStatus s = check_ready(a);
  if (s) return s;
  if (a->dws[0].B != B) {
    s = build_dw(a, 0, B);
    if (s) return s;
  }
  // pack actor, ACM, targets, critics (current weights)
  launch_pack(a, a->o_actor, (int)(a->pj_actor.size() + a->pj_acm.size() + a->pj_targ.size() + a->pj_critic_fwd.size()),
              st);
  SacArgs p = make_args(a, B);
  const int grid = sac_critic_grid(a, p.Bp);
  tmark(a, 0, st);
  const bool team = sac_team(a, p.Bp);
  hipLaunchKernelGGL(team ? a->ks.critic_team : a->ks.critic, dim3(grid), dim3(team ? 64 * kTeamCritic : 256), 0, st, p);
  tmark(a, 0, st);
  SPP_CHECK_HIP(hipGetLastError());
  tmark(a, 2, st);
  launch_dw(a, 0, 0, st);
  tmark(a, 2, st);
  hipLaunchKernelGGL(k_finalize_critic, dim3(1), dim3(kFinThreads), 0, st, (const float*)a->part, p.Bp / 32, B, losses);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppSacAcmCriticGrads(sppAgentHandle a, const sppBatch* bt, const float* eps_next, float* losses,
                               void* stream) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null");
  if (bt) {
    sppStatus s = stage(a, bt, eps_next, nullptr, S(stream));
    if (s) return s;
  } else if (eps_next) {
    const int Bp = (int)round_up(a->cur_B, 32);
    SPP_REQUIRE(a->cur_B > 0, SPP_E_STATE, "no staged batch");
    hipLaunchKernelGGL(k_eps_copy_fm, dim3(cdiv((int64_t)a->cfg.aout * Bp, 256)), dim3(256), 0, S(stream), eps_next,
                       a->EPS1, a->cfg.aout, a->cur_B, Bp);
  }
  return critic_grads_staged(a, losses, S(stream));
}

sppStatus sppSacAcmCriticApply(sppAgentHandle a, void* stream) {
  SPP_REQUIRE(a && a->d_adam.ptr, SPP_E_STATE, "agent not ready");
  a->steps[1] += 1;
  tmark(a, 3, S(stream));
  launch_adam(a, 0, 2, a->net[SPP_NET_CRITIC1].n, a->steps[1], a->cfg.critic_lr, a->cfg.tau, S(stream));
  tmark(a, 3, S(stream));
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

static sppStatus actor_grads(sppAgentHandle a, float* losses, hipStream_t st) {
  SPP_REQUIRE(!a->ddpg, SPP_E_STATE, "not a SAC_AcM agent");
  const int B = a->cur_B;
  SPP_REQUIRE(B > 0, SPP_E_STATE, "no staged batch");
  // repack the updated critics
  launch_pack(a, a->o_cfwd, (int)a->pj_critic_fwd.size(), st);
  SacArgs p = make_args(a, B);
  AcmScratch z{a->Z1, a->Z2, a->T3, a->GAD, a->MASK};
  const int grid = sac_grid(a, p.Bp);
  tmark(a, 1, st);
  const bool team = sac_team(a, p.Bp);
  hipLaunchKernelGGL(team ? a->ks.actor_team : a->ks.actor, dim3(grid), dim3(team ? 64 * kTeamActor : 256), 0, st, p, z);
  if (a->ks.actor_heads) hipLaunchKernelGGL(a->ks.actor_heads, dim3(grid), dim3(256), 0, st, p, z);
  tmark(a, 1, st);
  SPP_CHECK_HIP(hipGetLastError());
  tmark(a, 2, st);
  launch_dw(a, 0, 1, st);
  tmark(a, 2, st);
  hipLaunchKernelGGL(k_actor_partials, dim3(1), dim3(kFinThreads), 0, st, (const float*)a->part, p.Bp / 32, B, a->cfg.aout,
                     a->cfg.custom_loss, (double)a->cfg.target_entropy, a->alpha_grad ? a->alpha_grad : a->aux,
                     losses);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppSacAcmActorGrads(sppAgentHandle a, const float* eps_cur, float* losses, void* stream) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null");
  const int B = a->cur_B;
  SPP_REQUIRE(B > 0, SPP_E_STATE, "no staged batch");
  const int Bp = (int)round_up(B, 32);
  if (eps_cur)
    hipLaunchKernelGGL(k_eps_copy_fm, dim3(cdiv((int64_t)a->cfg.aout * Bp, 256)), dim3(256), 0, S(stream), eps_cur,
                       a->EPS2, a->cfg.aout, B, Bp);
  return actor_grads(a, losses, S(stream));
}

sppStatus sppAgentBindAlphaGrad(sppAgentHandle a, float* g) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null");
  a->alpha_grad = g;
  return SPP_OK;
}

sppStatus sppSacAcmDrawEps(sppAgentHandle a, uint64_t seed, uint64_t counter, void* stream) {
  SPP_REQUIRE(a && a->cur_B > 0, SPP_E_STATE, "no staged batch");
  const int B = a->cur_B, Bp = (int)round_up(B, 32);
  SPP_REQUIRE((int64_t)a->cfg.aout * Bp < ((int64_t)1 << 31), SPP_E_SHAPE, "draw_eps: aout * Bp >= 2^31");
  const int64_t quads = (int64_t)a->cfg.aout * Bp / 4;
  // EPS1 (counter 2c) and EPS2 (2c + 1) in one launch (grid.y)
  hipLaunchKernelGGL(k_eps_fm, dim3(cdiv(quads, 256), 2), dim3(256), 0, S(stream), a->EPS1, a->cfg.aout, B, Bp, seed,
                     2 * counter, a->EPS2, 2 * counter + 1);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppAgentReadEps(sppAgentHandle a, int which, float* out, void* stream) {
  SPP_REQUIRE(a && out && (which == 0 || which == 1), SPP_E_INVALID_ARG, "read_eps: bad args");
  SPP_REQUIRE(a->cur_B > 0, SPP_E_STATE, "no staged batch");
  const int B = a->cur_B, Bp = (int)round_up(B, 32);
  hipLaunchKernelGGL(k_eps_read_fm, dim3(cdiv((int64_t)a->cfg.aout * B, 256)), dim3(256), 0, S(stream),
                     (const float*)(which ? a->EPS2 : a->EPS1), out, a->cfg.aout, B, Bp);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

// The packed weight images that hold parameters of `net` (test access, see sppAgentUnpackImage).
static std::vector<PackJob> images_of(sppAgent* a, int net) {
  std::vector<PackJob> out;
  const NetBufs& nb = a->net[net];
  if (!nb.p) return out;
  for (auto* l : {&a->pj_actor, &a->pj_acm, &a->pj_targ, &a->pj_critic_fwd})
    for (const PackJob& j : *l)
      if (j.W >= nb.p && j.W < nb.p + nb.n) out.push_back(j);
  return out;
}

sppStatus sppAgentImageCount(sppAgentHandle a, int net, int* n) {
  SPP_REQUIRE(a && n && net >= 0 && net < SPP_NET_COUNT, SPP_E_INVALID_ARG, "image_count: bad args");
  *n = (int)images_of(a, net).size();
  return SPP_OK;
}

sppStatus sppAgentUnpackImage(sppAgentHandle a, int net, int i, float* out, void* stream) {
  SPP_REQUIRE(a && out && net >= 0 && net < SPP_NET_COUNT, SPP_E_INVALID_ARG, "unpack_image: bad args");
  const std::vector<PackJob> js = images_of(a, net);
  SPP_REQUIRE(i >= 0 && i < (int)js.size(), SPP_E_INVALID_ARG, "unpack_image: image %d of %d", i, (int)js.size());
  hipLaunchKernelGGL(k_unpack_matrix, dim3(64), dim3(256), 0, S(stream), js[i], (const float*)a->net[net].p, out);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppAgentSetTiming(sppAgentHandle a, int enable) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null");
  a->timing = enable != 0;
  return SPP_OK;
}

sppStatus sppAgentGetTiming(sppAgentHandle a, double* ms, int64_t* cnt) {
  SPP_REQUIRE(a && ms && cnt, SPP_E_INVALID_ARG, "null");
  for (int k = 0; k < 5; ++k) {
    double t = 0.0;
    for (size_t i = 0; i + 1 < a->tused[k]; i += 2) {
      SPP_CHECK_HIP(hipEventSynchronize(a->tev[k][i + 1]));
      float e = 0.f;
      SPP_CHECK_HIP(hipEventElapsedTime(&e, a->tev[k][i], a->tev[k][i + 1]));
      t += e;
    }
    ms[k] = t;
    cnt[k] = (int64_t)(a->tused[k] / 2);
    a->tused[k] = 0;
  }
  return SPP_OK;
}

static sppStatus actor_apply(sppAgentHandle a, float* losses, hipStream_t st) {
  a->steps[0] += 1;
  a->steps[2] += 1;
  tmark(a, 3, st);
  launch_adam(a, 2, 1, a->net[SPP_NET_ACTOR].n, a->steps[0], a->cfg.actor_lr, 0.f, st);
  tmark(a, 3, st);
  hipLaunchKernelGGL(k_alpha_step, dim3(1), dim3(64), 0, st, (const float*)(a->alpha_grad ? a->alpha_grad : a->aux),
                     (double)a->cfg.alpha_lr, a->steps[2], a->alpha_state, a->alpha_f32, losses);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppSacAcmActorApply(sppAgentHandle a, float* losses, void* stream) {
  SPP_REQUIRE(a, SPP_E_INVALID_ARG, "null");
  return actor_apply(a, losses, S(stream));
}

sppStatus sppSacAcmUpdate(sppAgentHandle a, const sppBatch* bt, const float* eps_next, const float* eps_cur,
                          float* losses, void* stream) {
  SPP_REQUIRE(a && !a->ddpg, SPP_E_STATE, "not a SAC_AcM agent");
  SPP_REQUIRE(a && eps_next && eps_cur, SPP_E_INVALID_ARG, "eps required (use sppSacAcmUpdateStaged for device draws)");
  hipStream_t st = S(stream);
  sppStatus s = stage(a, bt, eps_next, eps_cur, st);
  if (s) return s;
  if ((s = critic_grads_staged(a, losses, st))) return s;
  if ((s = sppSacAcmCriticApply(a, stream))) return s;
  if ((s = actor_grads(a, losses, st))) return s;
  return actor_apply(a, losses, st);
}

// ------------------------------------------------------------------ DDPG_AcM (ddpg_acm.py:147-201)
sppStatus sppDdpgAcmCriticGrads(sppAgentHandle a, const sppBatch* bt, float* losses, void* stream) {
  SPP_REQUIRE(a && a->ddpg, SPP_E_STATE, "not a DDPG_AcM agent");
  hipStream_t st = S(stream);
  sppStatus s;
  if (bt && (s = stage(a, bt, nullptr, nullptr, st))) return s;
  const int B = a->cur_B;
  SPP_REQUIRE(B > 0, SPP_E_STATE, "no staged batch");
  if ((s = check_ready(a))) return s;
  if (a->dws[0].B != B && (s = build_dw(a, 0, B))) return s;
  launch_pack(a, a->o_actor, (int)(a->pj_actor.size() + a->pj_acm.size() + a->pj_targ.size() + a->pj_critic_fwd.size()),
              st);
  SacArgs p = make_args(a, B);
  tmark(a, 0, st);
  hipLaunchKernelGGL(a->ks.dcritic, dim3(phase_grid(a, p.Bp)), dim3(256), 0, st, p, a->bz);
  tmark(a, 0, st);
  SPP_CHECK_HIP(hipGetLastError());
  tmark(a, 2, st);
  launch_dw(a, 0, 0, st);
  tmark(a, 2, st);
  hipLaunchKernelGGL(k_finalize_ddpg_critic, dim3(1), dim3(kFinThreads), 0, st, (const float*)a->part, p.Bp / 32, B, losses);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppDdpgAcmCriticApply(sppAgentHandle a, void* stream) {
  SPP_REQUIRE(a && a->ddpg && a->d_adam.ptr, SPP_E_STATE, "DDPG_AcM agent not ready");
  a->steps[1] += 1;
  tmark(a, 3, S(stream));
  launch_adam(a, 0, 1, a->net[SPP_NET_CRITIC1].n, a->steps[1], a->cfg.critic_lr, a->cfg.tau, S(stream));
  tmark(a, 3, S(stream));
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppDdpgAcmActorGrads(sppAgentHandle a, float* losses, void* stream) {
  SPP_REQUIRE(a && a->ddpg && a->cur_B > 0, SPP_E_STATE, "DDPG_AcM agent: no staged batch");
  hipStream_t st = S(stream);
  const int B = a->cur_B;
  launch_pack(a, a->o_cfwd, (int)a->pj_critic_fwd.size(), st);  // the updated critic
  SacArgs p = make_args(a, B);
  tmark(a, 1, st);
  hipLaunchKernelGGL(a->ks.dactor, dim3(phase_grid(a, p.Bp)), dim3(256), 0, st, p, a->bz);
  tmark(a, 1, st);
  SPP_CHECK_HIP(hipGetLastError());
  tmark(a, 2, st);
  launch_dw(a, 0, 1, st);
  tmark(a, 2, st);
  hipLaunchKernelGGL(k_finalize_ddpg_actor, dim3(1), dim3(kFinThreads), 0, st, (const float*)a->part, p.Bp / 32, B,
                     a->cfg.aout, a->cfg.custom_loss, losses);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

// actor Adam step, then polyak of the critic target (already fused into the critic
// step: the critic does not change afterwards) and of the actor target (ddpg.py:273-284)
sppStatus sppDdpgAcmActorApply(sppAgentHandle a, void* stream) {
  SPP_REQUIRE(a && a->ddpg && a->d_adam.ptr, SPP_E_STATE, "DDPG_AcM agent not ready");
  a->steps[0] += 1;
  tmark(a, 3, S(stream));
  launch_adam(a, 2, 1, a->net[SPP_NET_ACTOR].n, a->steps[0], a->cfg.actor_lr, a->cfg.tau, S(stream));
  tmark(a, 3, S(stream));
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppDdpgAcmUpdate(sppAgentHandle a, const sppBatch* bt, float* losses, void* stream) {
  sppStatus s;
  if ((s = sppDdpgAcmCriticGrads(a, bt, losses, stream))) return s;
  if ((s = sppDdpgAcmCriticApply(a, stream))) return s;
  if ((s = sppDdpgAcmActorGrads(a, losses, stream))) return s;
  return sppDdpgAcmActorApply(a, stream);
}

sppStatus sppAgentStageFromReplay(sppAgentHandle a, sppReplayHandle r, const int64_t* idx, int B, void* stream) {
  SPP_REQUIRE(a && r && idx && B > 0 && B <= a->Bmax, SPP_E_INVALID_ARG, "stage_from_replay: bad args");
  SPP_REQUIRE(r->d.ob == a->cfg.ob && r->d.ac == a->cfg.ac && r->d.aout == a->cfg.aout, SPP_E_SHAPE, "dims differ");
  const int Bp = (int)round_up(B, 32);
  // Wide rows (Ant, ob > 64) stage faster with k_replay_stage_fm2 (four gathers before one barrier,
  // division-free lane geometry: 0.30 -> 0.22 ms at B = 409,600); narrow rows (Hopper, HalfCheetah)
  // are faster with the 64-sample tiles of k_replay_stage_fm (0.059 vs 0.128 ms, 0.154 vs 0.292 ms).
  float* act = a->cfg.acm_critic ? nullptr : a->ACT;
  if (r->d.ob > 64)
    hipLaunchKernelGGL(k_replay_stage_fm2, dim3(cdiv(Bp, kStage2Tile)), dim3(256),
                       stage2_lds_bytes(r->d.ob, r->d.aout, r->d.ac, act != nullptr), S(stream), r->d, idx, B, Bp,
                       a->S, a->S2, act, a->AENV, a->R, a->DN);
  else
    hipLaunchKernelGGL(k_replay_stage_fm, dim3(cdiv(Bp, kStageTile)), dim3(256),
                       sizeof(float) * kStageTile * std::max(r->d.ob, r->d.aout), S(stream), r->d, idx, B, Bp, a->S,
                       a->S2, act, a->AENV, a->R, a->DN);
  SPP_CHECK_HIP(hipGetLastError());
  a->cur_B = B;
  return SPP_OK;
}

sppStatus sppAgentStagePost(sppAgentHandle a, int normalize, int act_from_next_obs, void* stream) {
  SPP_REQUIRE(a && a->cur_B > 0, SPP_E_STATE, "stage_post: no staged batch");
  if (!normalize && !act_from_next_obs) return SPP_OK;
  SPP_REQUIRE(!act_from_next_obs || (!a->cfg.acm_critic && a->cfg.aout == a->cfg.ob && a->ACT), SPP_E_INVALID_ARG,
              "stage_post: action = next_obs needs a critic on (obs, actor output) with aout == ob");
  SPP_REQUIRE(normalize >= 0 && normalize <= 2, SPP_E_INVALID_ARG, "stage_post: normalize %d", normalize);
  const int mm = normalize == 2 ? 0 : a->cfg.min_max_denormalize;  // 2: z-score whatever the agent's mode
  SPP_REQUIRE(!normalize || (mm ? (a->lo && a->hi) : (a->mean && a->std)), SPP_E_STATE,
              "stage_post: normalizer not bound");
  const int B = a->cur_B, Bp = (int)round_up(B, 32), ob = a->cfg.ob;
  hipLaunchKernelGGL(k_stage_post, dim3(cdiv((int64_t)ob * B, 256)), dim3(256), 0, S(stream), a->S, a->S2, a->ACT, ob,
                     B, Bp, a->lo, a->hi, a->mean, a->std, mm, normalize != 0, act_from_next_obs);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppSacAcmUpdateStaged(sppAgentHandle a, uint64_t seed, uint64_t counter, float* losses, void* stream) {
  SPP_REQUIRE(a && a->cur_B > 0, SPP_E_STATE, "no staged batch");
  hipStream_t st = S(stream);
  sppStatus s = sppSacAcmDrawEps(a, seed, counter, stream);
  if (s) return s;
  if ((s = critic_grads_staged(a, losses, st))) return s;
  if ((s = sppSacAcmCriticApply(a, stream))) return s;
  if ((s = actor_grads(a, losses, st))) return s;
  return actor_apply(a, losses, st);
}

sppStatus sppAcmRegressGrads(sppAgentHandle a, const float* x, const float* y, int B, float* loss, void* stream) {
  SPP_REQUIRE(a && x && y && B > 0 && B <= a->Bmax, SPP_E_INVALID_ARG, "acm step: bad args (B=%d, max %d)", B,
              a->Bmax);
  hipStream_t st = S(stream);
  sppStatus s = check_ready(a);
  if (s) return s;
  if (a->dws[1].B != B) {
    if ((s = build_dw(a, 1, B))) return s;
  }
  launch_pack(a, a->o_acm, (int)a->pj_acm.size(), st);
  SacArgs p = make_args(a, B);
  if (a->ddpg) {  // BasicAcM: natural-input fc1 / fc21 packings
    p.bacm.W1 = a->bacm_W1n;
    p.bacm.W21 = a->bacm_W21n;
    BAcmRegArgs g{};
    g.B = B; g.Bp = (int)round_up(B, 32); g.x = x; g.y = y;
    g.XT = a->RX; g.H = a->RBH; g.H1 = a->RBH1; g.S21 = a->RS21; g.P1 = a->RBP1; g.PZ = a->RPZ; g.PZ21 = a->RPZ21;
    g.P3 = a->RP3; g.part = a->part;
    tmark(a, 4, st);
    hipLaunchKernelGGL(a->ks.dreg, dim3(phase_grid(a, g.Bp)), dim3(256), 0, st, p, g);
    SPP_CHECK_HIP(hipGetLastError());
    launch_dw(a, 1, 0, st);
    tmark(a, 4, st);
    hipLaunchKernelGGL(k_finalize_bacm, dim3(1), dim3(256), 0, st, (const float*)a->part, g.Bp / 32, kBParts, B,
                       a->cfg.ac, a->net[SPP_NET_ACM].g, loss);
    SPP_CHECK_HIP(hipGetLastError());
    return SPP_OK;
  }
  p.acm.W1 = a->acm_W1n;
  AcmRegArgs g{};
  g.B = B; g.Bp = (int)round_up(B, 32); g.x = x; g.y = y;
  g.XT = a->RX; g.Z1 = a->RZ1; g.Z2 = a->RZ2; g.P1 = a->RP1; g.P2 = a->RP2; g.P3 = a->RP3; g.part = a->part;
  tmark(a, 4, st);
  hipLaunchKernelGGL(a->ks.acmreg, dim3(phase_grid(a, g.Bp)), dim3(256), 0, st, p, g);
  SPP_CHECK_HIP(hipGetLastError());
  launch_dw(a, 1, 0, st);
  tmark(a, 4, st);
  hipLaunchKernelGGL(k_finalize_acm, dim3(1), dim3(256), 0, st, (const float*)a->part, g.Bp / 32, B, a->cfg.ac, loss);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppAcmRegressApply(sppAgentHandle a, void* stream) {
  SPP_REQUIRE(a && a->d_adam.ptr, SPP_E_STATE, "agent not ready");
  a->steps[3] += 1;
  launch_adam(a, 3, 1, a->net[SPP_NET_ACM].n, a->steps[3], a->cfg.acm_lr, 0.f, S(stream));
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

// co-resident workgroups of the multi-workgroup AcM k_mlp_sgd on this device (0: no instantiation)
extern "C++" {
template <int IN, int H2, int OUT, int HEAD, int WV = 4>
static int mlp_sgd_max_wg(int num_cu) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_mlp_sgd<IN, H2, OUT, HEAD, true, WV>,
                                                   64 * WV, 0) != hipSuccess)
    per_cu = 0;
  return std::min(MlCfg<IN, H2, OUT, HEAD, WV>::MAXG, per_cu * num_cu);
}
}
// waves per workgroup of the multi-workgroup AcM regression kernel (HEAD 0, bs > 64).  8 = two waves per SIMD,
// up to 128 rows per workgroup, at least 2 workgroups (its LDS has no room for the single-workgroup form's
// canonical gradient staging).  Measured round 5 (1049-row PPO ACM steps, profiles/r05/ab_acm_wv.txt): 8 waves
// on 9 workgroups 17.3 us per step against 13.4 us for 4 waves on 17: the MFMA work per CU doubles while the
// second wave per SIMD hides less than that, so the default stays 4 (A/B: -DSPP_ACM_WV=8; 2 waves on 33
// workgroups measured 17.0 us too).  bs <= 64 always runs
// the single-workgroup 4-wave form.
#ifndef SPP_ACM_WV
#define SPP_ACM_WV 4
#endif
constexpr int kAcmWV = SPP_ACM_WV, kAcmR = 16 * kAcmWV;
// Passes of kAcmR rows per workgroup and step (sppSetAcmSgdPasses; 0: one): P passes put a step on
// ceil(bs / (P kAcmR)) workgroups (k_mlp_sgd's MP form).
static int g_acm_passes = 0;
static int acm_passes(int bs) {
  const int P = std::max(1, g_acm_passes);
  return bs <= kMlR || cdiv(bs, kAcmR) < 2 * P ? 1 : P;  // (>= 2 workgroups after the split)
}
static int acm_sgd_nwg(int bs) { return bs <= kMlR ? 1 : std::max(2, cdiv(bs, kAcmR * acm_passes(bs))); }
static int acm_sgd_max_wg(sppAgentHandle a, int ob, int ac) {
  if (a->sgd_max_wg >= 0) return a->sgd_max_wg;
  int n = 0;
  if (ob == 11 && ac == 3) n = mlp_sgd_max_wg<22, 32, 3, 0, kAcmWV>(a->num_cu);
  else if (ob == 17 && ac == 6) n = mlp_sgd_max_wg<34, 32, 6, 0, kAcmWV>(a->num_cu);
  else if (ob == 3 && ac == 1) n = mlp_sgd_max_wg<6, 32, 1, 0, kAcmWV>(a->num_cu);
  a->sgd_max_wg = n;
  return n;
}

int sppAcmSgdWorkgroups(sppAgentHandle a, int bs) { return (a && !a->ddpg && bs > 0) ? acm_sgd_nwg(bs) : 0; }

sppStatus sppSetAcmSgdPasses(int passes) {
  SPP_REQUIRE(passes >= 0 && passes <= 16, SPP_E_INVALID_ARG, "acm passes %d", passes);
  g_acm_passes = passes;
  return SPP_OK;
}

int sppAcmSgdMaxBatch(sppAgentHandle a) {
  if (!a || a->ddpg) return 0;
  return kAcmR * std::max(1, g_acm_passes) * std::max(1, acm_sgd_max_wg(a, a->cfg.ob, a->cfg.ac));
}

// polls before a k_mlp_sgd arrival wait times out (0: the kernel's default); test hook sppSetSgdSpinLimit
static int g_sgd_spin = 0;

// slabs [2][kMlMaxWG][kMlSlabMax] + the parameter buffer [kSgdPubReps][kMlSlabMax] + {arrival counter, timeout flag}
// sync: [0] unused, [1] the sticky timeout flag, [kSgdShardStride (1 + k)] arrival counter shard k (sgd.hip)
constexpr int kSgdSyncInts = kSgdShardStride * (1 + kSgdShards);
static int* sgd_ctr(DevArray<int>& sync) { return sync.ptr + kSgdShardStride; }
static sppStatus mlp_sgd_buffers(DevArray<float>& slab, DevArray<int>& sync, hipStream_t st) {
  if (!slab.ptr) {
    SPP_CHECK_HIP(slab.alloc((size_t)(2 * kMlMaxWG + kSgdPubReps) * kMlSlabMax));  // slabs, published replicas
    SPP_CHECK_HIP(sync.alloc(kSgdSyncInts));
    SPP_CHECK_HIP(hipMemsetAsync(sync.ptr, 0, kSgdSyncInts * sizeof(int), st));
  }
  // the arrival counter shards (the flag is sticky)
  SPP_CHECK_HIP(hipMemsetAsync(sgd_ctr(sync), 0, kSgdShards * kSgdShardStride * sizeof(int), st));
  return SPP_OK;
}

sppStatus sppAcmSgdStatusAsync(sppAgentHandle a, int* timed_out_pinned, void* stream) {
  SPP_REQUIRE(a && timed_out_pinned, SPP_E_INVALID_ARG, "acm_sgd_status_async: null");
  if (a->sgd_sync.ptr)
    SPP_CHECK_HIP(hipMemcpyAsync(timed_out_pinned, a->sgd_sync.ptr + 1, sizeof(int), hipMemcpyDeviceToHost, S(stream)));
  else
    *timed_out_pinned = 0;
  return SPP_OK;
}

// nsteps sequential steps: bs rows each, the last one bs_last (<= bs) rows
static sppStatus acm_sgd_run(sppAgentHandle a, const float* x, const float* y, int nsteps, int bs, int bs_last,
                             float* loss_sum, void* stream) {
  SPP_REQUIRE(a && x && y && loss_sum && nsteps >= 0 && bs > 0 && bs_last > 0 && bs_last <= bs, SPP_E_INVALID_ARG,
              "acm_sgd: bad args");
  SPP_REQUIRE(!a->ddpg, SPP_E_INVALID_ARG, "acm_sgd: the persistent kernel is for the AcM (SAC_AcM / PPO_AcM handles)");
  SPP_REQUIRE(bs <= kAcmR * kMlMaxWG, SPP_E_SHAPE, "acm_sgd: batch %d > %d", bs, kAcmR * kMlMaxWG);
  sppStatus s = check_ready(a);
  if (s) return s;
  if (nsteps == 0) return SPP_OK;
  const NetBufs& n = a->net[SPP_NET_ACM];
  SPP_REQUIRE(n.p && n.m && n.v, SPP_E_STATE, "acm_sgd: ACM buffers not bound");
  MlpSgdArgs g{};
  g.x = x; g.y = y; g.nsteps = nsteps; g.bs = bs; g.bsl = bs; g.bs_last = bs_last;
  g.params = n.p; g.m = n.m; g.v = n.v; g.lr = a->cfg.acm_lr; g.step0 = a->steps[3];
  g.lim = a->limits.ptr + a->cfg.aout; g.loss_sum = loss_sum; g.spin = g_sgd_spin;
  const int ob = a->cfg.ob, ac = a->cfg.ac;
  hipStream_t st = S(stream);
  // <= kAcmR rows per workgroup (sgd_mlp.hip); the per-step arrival barriers need every workgroup resident at once
  const int nwg = acm_sgd_nwg(bs);
  SPP_REQUIRE(nwg <= acm_sgd_max_wg(a, ob, ac), SPP_E_SHAPE, "acm_sgd: batch %d needs %d co-resident workgroups > %d",
              bs, nwg, acm_sgd_max_wg(a, ob, ac));
  if (nwg > 1) {
    g.bsl = cdiv(bs, nwg);
    s = mlp_sgd_buffers(a->sgd_slab, a->sgd_sync, st);
    if (s) return s;
    g.slab = a->sgd_slab.ptr;
    g.pbuf = a->sgd_slab.ptr + (size_t)2 * kMlMaxWG * kMlSlabMax;
    g.ctr = sgd_ctr(a->sgd_sync);
    g.err = a->sgd_sync.ptr + 1;
  }
  const bool mw = nwg > 1, mp = mw && g.bsl > kAcmR;
#define SPP_SGD_LAUNCH(IN_, AC_)                                                                              \
  if (mp) hipLaunchKernelGGL((k_mlp_sgd<IN_, 32, AC_, 0, true, kAcmWV, true>), dim3(nwg), dim3(64 * kAcmWV), 0, st, g); \
  else if (mw) hipLaunchKernelGGL((k_mlp_sgd<IN_, 32, AC_, 0, true, kAcmWV>), dim3(nwg), dim3(64 * kAcmWV), 0, st, g); \
  else hipLaunchKernelGGL((k_mlp_sgd<IN_, 32, AC_, 0, false>), dim3(1), dim3(kMlTH), 0, st, g)
  if (ob == 11 && ac == 3) SPP_SGD_LAUNCH(22, 3);
  else if (ob == 17 && ac == 6) SPP_SGD_LAUNCH(34, 6);
  else if (ob == 3 && ac == 1) SPP_SGD_LAUNCH(6, 1);
  else SPP_REQUIRE(false, SPP_E_SHAPE, "acm_sgd: no instantiation for ob=%d ac=%d", ob, ac);
#undef SPP_SGD_LAUNCH
  a->steps[3] += nsteps;
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppAcmSgd(sppAgentHandle a, const float* x, const float* y, int nsteps, int bs, float* loss_sum,
                    void* stream) {
  return acm_sgd_run(a, x, y, nsteps, bs, bs, loss_sum, stream);
}

sppStatus sppAcmSgdEpoch(sppAgentHandle a, const float* x, const float* y, int nrows, int bs, float* loss_sum,
                         void* stream) {
  SPP_REQUIRE(nrows >= 0 && bs > 0, SPP_E_INVALID_ARG, "acm_sgd_epoch: bad args");
  if (nrows == 0) return SPP_OK;
  const int nsteps = cdiv(nrows, bs);
  return acm_sgd_run(a, x, y, nsteps, bs, nrows - (nsteps - 1) * bs, loss_sum, stream);
}

sppStatus sppAcmSgdStatus(sppAgentHandle a, int* timed_out) {
  SPP_REQUIRE(a && timed_out, SPP_E_INVALID_ARG, "acm_sgd_status: null");
  *timed_out = 0;
  if (a->sgd_sync.ptr) SPP_CHECK_HIP(hipMemcpy(timed_out, a->sgd_sync.ptr + 1, sizeof(int), hipMemcpyDeviceToHost));
  return SPP_OK;
}

sppStatus sppAcmRegressStep(sppAgentHandle a, const float* x, const float* y, int B, float* loss, void* stream) {
  sppStatus s = sppAcmRegressGrads(a, x, y, B, loss, stream);
  if (s) return s;
  return sppAcmRegressApply(a, stream);
}

sppStatus sppReplaySetAcmColumns(sppReplayHandle h, const int* cols, int n) {
  SPP_REQUIRE(h && (n == 0 || (cols && n == h->d.ob)), SPP_E_INVALID_ARG,
              "acm columns: %d columns for ob = %d (acm_cat feeds the AcM 2 x len(acm_ob_idx) inputs, which it takes "
              "only when len(acm_ob_idx) = ob)", n, h ? h->d.ob : 0);
  for (int i = 0; i < n; ++i)
    SPP_REQUIRE(cols[i] >= 0 && cols[i] < h->d.ob, SPP_E_INVALID_ARG, "acm columns: index %d out of range", cols[i]);
  SPP_CHECK_HIP(hipSetDevice(h->device));
  SPP_CHECK_HIP(hipDeviceSynchronize());  // (a gather in flight may still read the old map)
  SPP_CHECK_HIP(hipFree((void*)h->d.acm_cols));
  h->d.acm_cols = nullptr;
  if (n == 0) return SPP_OK;
  int* d = nullptr;
  SPP_CHECK_HIP(hipMalloc(&d, sizeof(int) * n));
  SPP_CHECK_HIP(hipMemcpy(d, cols, sizeof(int) * n, hipMemcpyHostToDevice));
  h->d.acm_cols = d;
  return SPP_OK;
}

sppStatus sppReplayGatherAcm(sppReplayHandle h, const int64_t* idx, int B, float* x, float* y, void* stream) {
  SPP_REQUIRE(h && idx && x && y && B > 0, SPP_E_INVALID_ARG, "gather_acm: bad args");
  hipLaunchKernelGGL(k_replay_gather_acm, dim3(cdiv(B, kStageTile)), dim3(256), 0, S(stream), h->d, idx, B, x, y);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppPolicyAct(sppAgentHandle a, const float* obs, int E, const float* eps, const float* noise,
                       float act_noise, int mode, int denorm_out, float* target_out, float* env_out, void* stream) {
  SPP_REQUIRE(a && obs && E > 0 && target_out && env_out, SPP_E_INVALID_ARG, "policy_act: bad args");
  SPP_REQUIRE(mode >= 0 && mode <= 3, SPP_E_INVALID_ARG, "mode");
  SPP_REQUIRE((mode != 0 && mode != 3) || eps, SPP_E_INVALID_ARG, "modes 0 / 3 need eps");
  SPP_REQUIRE(mode != 3 || !a->ddpg, SPP_E_INVALID_ARG, "mode 3 (caller action) is a SAC_AcM-handle (AcM) mode");
  hipStream_t st = S(stream);
  sppStatus s = check_ready(a);
  if (s) return s;
  launch_pack(a, a->o_actor, (int)(a->pj_actor.size() + a->pj_acm.size()), st);
  SacArgs p = make_args(a, 32);
  ActArgs g{E, mode, denorm_out, act_noise, obs, eps, noise, target_out, env_out, a->plain ? 1 : 0};
  const int grid = std::max(1, std::min(cdiv(cdiv(E, 32), kWavesPerWG), a->num_cu));
  if (a->ddpg)
    hipLaunchKernelGGL(a->ks.dact, dim3(grid), dim3(256), 0, st, p, g, a->bz);
  else if (a->plain && a->ks.act_team && a->team_ok && cdiv(E, 32) <= a->num_cu)  // one tile per CU (sac_team.h)
    hipLaunchKernelGGL(a->ks.act_team, dim3(cdiv(E, 32)), dim3(64 * kTeamCritic), 0, st, p, g);
  else
    hipLaunchKernelGGL(a->ks.act, dim3(grid), dim3(256), 0, st, p, g);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppDebugDense(const float* x, const float* W, const float* b, float* y, int B, int K, int N, int act,
                        void* stream) {
  SPP_REQUIRE(x && W && y && B > 0 && K > 0 && K <= 256 && N > 0 && N <= 256, SPP_E_INVALID_ARG, "debug dense: bad");
  SPP_REQUIRE(K <= 224 || K == 256, SPP_E_INVALID_ARG, "debug dense: K in (224, 256) not supported");
  hipStream_t st = S(stream);
  const int NBI = blocks_of(K), NBO = blocks_of(N);
  const int ibm = NBI == 8 ? 1 : 0;
  float4* wf;
  PackJob* dj;
  SPP_CHECK_HIP(hipMalloc(&wf, sizeof(float4) * NBO * NBI * 256));
  SPP_CHECK_HIP(hipMalloc(&dj, sizeof(PackJob)));
  PackJob pj{W, nullptr, 1 << 30, K, 0, 0, nat(N), nat(K), NBO, NBI, ibm, wf};
  SPP_CHECK_HIP(hipMemcpy(dj, &pj, sizeof(pj), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_pack_matrix, dim3(16, 1), dim3(256), 0, st, (const PackJob*)dj);
  const dim3 grid(cdiv(B, 32));
  const int kq = regs_valid(K, 0) / 4;  // quads of block 0 that carry units
  if (NBI == 1 && kq < 4) {
    switch (kq) {
#define SPP_DD(n) case n: hipLaunchKernelGGL((k_debug_dense<1, 1, n>), grid, dim3(64), 0, st, (const float4*)wf, b, x, y, B, K, N, act); break;
      SPP_DD(1) SPP_DD(2) SPP_DD(3)
#undef SPP_DD
    }
  } else if (NBI < 8) {
    switch (NBI) {
#define SPP_DD(n) case n: hipLaunchKernelGGL((k_debug_dense<n, 1>), grid, dim3(64), 0, st, (const float4*)wf, b, x, y, B, K, N, act); break;
      SPP_DD(1) SPP_DD(2) SPP_DD(3) SPP_DD(4) SPP_DD(5) SPP_DD(6) SPP_DD(7)
#undef SPP_DD
    }
  } else {
    switch (NBO) {
#define SPP_DD(n) case n: hipLaunchKernelGGL((k_debug_dense<8, n>), grid, dim3(64), 0, st, (const float4*)wf, b, x, y, B, K, N, act); break;
      SPP_DD(1) SPP_DD(2) SPP_DD(3) SPP_DD(4) SPP_DD(5) SPP_DD(6) SPP_DD(7) SPP_DD(8)
#undef SPP_DD
    }
  }
  SPP_CHECK_HIP(hipGetLastError());
  SPP_CHECK_HIP(hipStreamSynchronize(st));
  hipFree(wf); hipFree(dj);
  return SPP_OK;
}

}  // extern "C"

// ================================================================== on-policy (A2C / PPO) nets
namespace spp {
struct OnpKernels {
  void (*value)(OnpArgs);
  void (*critic)(OnpArgs);
  void (*actor)(OnpArgs);
  void (*act)(OnpArgs);
};
template <int OB, int AOUT>
OnpKernels make_onp() {
  using C = OCfg<OB, AOUT>;
  return {k_onp_value<C>, k_onp_critic_grad<C>, k_onp_actor_grad<C>, k_onp_act<C>};
}
static bool find_onp(int ob, int aout, OnpKernels* k) {
  if (ob == 17 && aout == 17) { *k = make_onp<17, 17>(); return true; }  // SPP-PPO HalfCheetah
  if (ob == 11 && aout == 11) { *k = make_onp<11, 11>(); return true; }  // Hopper
  if (ob == 17 && aout == 6) { *k = make_onp<17, 6>(); return true; }    // vanilla PPO HalfCheetah
  if (ob == 3 && aout == 1) { *k = make_onp<3, 1>(); return true; }      // Pendulum (tests)
  return false;
}
static int64_t onp_actor_size(int ob, int aout) { return aout + 64LL * ob + 64 + 64 * 64 + 64 + aout * 64LL + aout; }
static int64_t onp_critic_size(int ob) { return 64LL * ob + 64 + 64 * 64 + 64 + 64 + 1; }
}  // namespace spp

struct sppOnPolicy {
  sppOnPolicyConfig cfg{};
  int device = 0, num_cu = 256;
  OnpKernels ks{};
  NetBufs net[2];  // 0 actor, 1 critic
  int64_t nsize[2] = {};
  int64_t steps[2] = {0, 0};
  DevArray<float> lim;
  DevArray<float4> pk;
  DevArray<PackJob> d_pj;
  int npj_actor = 0, npj_critic = 0;
  OnpNet actor{}, critic{};
  std::vector<TabSeg> tab;
  DevArray<float> scratch;
  float *XT = nullptr, *H1 = nullptr, *H2 = nullptr, *D1 = nullptr, *D2 = nullptr, *D3 = nullptr, *part = nullptr;
  int Bpmax = 0, pstride = 0;
  DwSet dw[2];  // 0 critic, 1 actor
  DevArray<AdamJob> d_adam;
  // persistent PPO actor epochs (sppOnpActorEpoch, sgd_mlp.hip HEAD 1): slabs + parameter buffer, {counter, flag}
  DevArray<float> sgd_slab;
  DevArray<int> sgd_sync;
  int sgd_max_wg = -1;
  int crit_max_wg = -1;  // co-resident persistent-critic workgroups (onp_critic_max_wg, cached)
  int wg_reserve = 0;    // CUs left to a persistent launch on another stream (sppOnpReserveWorkgroups)
};

static sppStatus onp_packs(sppOnPolicy* o) {
  const int ob = o->cfg.ob, aout = o->cfg.aout;
  SPP_REQUIRE(o->net[0].p && o->net[1].p, SPP_E_STATE, "on-policy nets not bound");
  std::vector<PackJob> jobs;
  std::vector<const float4**> slots;
  auto M = [&](const float* W, int ld, int trans, MapDesc out, MapDesc in, int NBO, int NBI, const float4** slot) {
    jobs.push_back(PackJob{W, nullptr, 1 << 30, ld, trans, 0, out, in, NBO, NBI, 0, nullptr});
    slots.push_back(slot);
  };
  o->tab.clear();
  int toff = 0;
  auto T = [&](const float* v, int n) {
    const int off = toff, tot = (int)round_up(n, 32);
    o->tab.push_back(TabSeg{v, n, tot, off, 0});
    toff += tot;
    return off;
  };
  {  // actor: log_scale, fc1, fc2, fc3 (basic_model.py:14-21)
    const float* P = o->net[0].p;
    const float *W1 = P + aout, *b1 = W1 + 64 * ob, *W2 = b1 + 64, *b2 = W2 + 64 * 64, *W3 = b2 + 64,
                *b3 = W3 + aout * 64;
    M(W1, ob, 0, nat(64), nat(ob), 2, blocks_of(ob), &o->actor.W1);
    M(W2, 64, 0, nat(64), nat(64), 2, 2, &o->actor.W2);
    M(W3, 64, 0, nat(aout), nat(64), blocks_of(aout), 2, &o->actor.W3);
    M(W3, 64, 1, nat(64), nat(aout), 2, blocks_of(aout), &o->actor.W3T);
    M(W2, 64, 1, nat(64), nat(64), 2, 2, &o->actor.W2T);
    o->actor.tb1 = T(b1, 64);
    o->actor.tb2 = T(b2, 64);
    o->actor.tb3 = T(b3, aout);
  }
  o->npj_actor = (int)jobs.size();
  {  // critic: fc1, fc2, fc3 (basic_model.py:62-70)
    const float* P = o->net[1].p;
    const float *W1 = P, *b1 = W1 + 64 * ob, *W2 = b1 + 64, *b2 = W2 + 64 * 64, *w3 = b2 + 64, *b3 = w3 + 64;
    M(W1, ob, 0, nat(64), nat(ob), 2, blocks_of(ob), &o->critic.W1);
    M(W2, 64, 0, nat(64), nat(64), 2, 2, &o->critic.W2);
    M(W2, 64, 1, nat(64), nat(64), 2, 2, &o->critic.W2T);
    o->critic.tb1 = T(b1, 64);
    o->critic.tb2 = T(b2, 64);
    o->critic.tb3 = T(w3, 64);
    o->critic.b3 = b3;
  }
  o->npj_critic = (int)jobs.size() - o->npj_actor;
  SPP_REQUIRE(toff <= 1024 && o->tab.size() <= 8, SPP_E_SHAPE, "on-policy LDS table too large");
  size_t nf4 = 0;
  for (auto& j : jobs) nf4 += (size_t)j.NBO * j.NBI * 256;
  o->pk.release();
  SPP_CHECK_HIP(o->pk.alloc(nf4));
  size_t of = 0;
  for (size_t i = 0; i < jobs.size(); ++i) {
    jobs[i].dst = o->pk.ptr + of;
    *slots[i] = jobs[i].dst;
    of += (size_t)jobs[i].NBO * jobs[i].NBI * 256;
  }
  o->d_pj.release();
  SPP_CHECK_HIP(o->d_pj.alloc(jobs.size()));
  SPP_CHECK_HIP(hipMemcpy(o->d_pj.ptr, jobs.data(), sizeof(PackJob) * jobs.size(), hipMemcpyHostToDevice));
  AdamJob aj[2] = {AdamJob{o->net[0].p, o->net[0].g, o->net[0].m, o->net[0].v, nullptr, o->net[0].n},
                   AdamJob{o->net[1].p, o->net[1].g, o->net[1].m, o->net[1].v, nullptr, o->net[1].n}};
  if (!o->d_adam.ptr) SPP_CHECK_HIP(o->d_adam.alloc(2));
  SPP_CHECK_HIP(hipMemcpy(o->d_adam.ptr, aj, sizeof(aj), hipMemcpyHostToDevice));
  o->dw[0].B = o->dw[1].B = -1;
  return SPP_OK;
}

static sppStatus onp_dw(sppOnPolicy* o, int which, int N) {
  const int Bp = (int)round_up(N, 32), ob = o->cfg.ob, aout = o->cfg.aout;
  std::vector<DwJob> jobs;
  auto J = [&](const float* A, int Nn, const float* X, int K, float* dW, float* db) {
    DwJob j{};
    j.A = A; j.N = Nn; j.X0 = X; j.K0 = K; j.dW = dW; j.db = db; j.Bp = Bp; j.nrow2 = Nn;
    j.slab_stride = round_up((int64_t)Nn * K + Nn, 4);
    jobs.push_back(j);
  };
  if (which == 0) {
    float* G = o->net[1].g;
    float *gW1 = G, *gb1 = gW1 + 64 * ob, *gW2 = gb1 + 64, *gb2 = gW2 + 64 * 64, *gw3 = gb2 + 64, *gb3 = gw3 + 64;
    J(o->D1, 64, o->XT, ob, gW1, gb1);
    J(o->D2, 64, o->H1, 64, gW2, gb2);
    J(o->D3, 1, o->H2, 64, gw3, gb3);
  } else {
    float* G = o->net[0].g;
    float *gW1 = G + aout, *gb1 = gW1 + 64 * ob, *gW2 = gb1 + 64, *gb2 = gW2 + 64 * 64, *gW3 = gb2 + 64,
          *gb3 = gW3 + aout * 64;
    J(o->D1, 64, o->XT, ob, gW1, gb1);
    J(o->D2, 64, o->H1, 64, gW2, gb2);
    J(o->D3, aout, o->H2, 64, gW3, gb3);
  }
  DwSet& D = o->dw[which];
  D.j0[0] = 0;
  D.nj[0] = (int)jobs.size();
  return finalize_dw(D, jobs, 1, Bp, N, o->num_cu);
}

static OnpArgs onp_args(sppOnPolicy* o, int N) {
  OnpArgs p{};
  p.N = N;
  p.Np = (int)round_up(N, 32);
  p.actor = o->actor;
  p.critic = o->critic;
  p.log_scale = o->net[0].p;
  p.lim = o->lim.ptr;
  p.eps_clip = o->cfg.ppo_epsilon;
  p.XT = o->XT; p.H1 = o->H1; p.H2 = o->H2; p.D1 = o->D1; p.D2 = o->D2; p.D3 = o->D3;
  p.part = o->part;
  p.pstride = o->pstride;
  p.nseg = (int)o->tab.size();
  for (int i = 0; i < p.nseg; ++i) p.seg[i] = o->tab[i];
  return p;
}

// net 0: repack the actor's weight images (the params may have changed since the last call), 1: the
// critic's; the other network's images are not touched.
static sppStatus onp_ready(sppOnPolicy* o, int N, hipStream_t st, int net) {
  SPP_REQUIRE(N > 0 && N <= o->cfg.max_batch, SPP_E_SHAPE, "batch %d outside (0, max_batch=%d]", N, o->cfg.max_batch);
  SPP_REQUIRE(o->lim.ptr, SPP_E_STATE, "actor limits not set");
  if (!o->pk.ptr) {
    sppStatus s = onp_packs(o);
    if (s) return s;
  }
  const PackJob* pj = (const PackJob*)o->d_pj.ptr + (net == 0 ? 0 : o->npj_actor);
  hipLaunchKernelGGL(k_pack_matrix, dim3(16, net == 0 ? o->npj_actor : o->npj_critic), dim3(256), 0, st, pj);
  return SPP_OK;
}

static int onp_grid(sppOnPolicy* o, int N) {
  return std::max(1, std::min(cdiv(cdiv(N, 32), 4), o->num_cu * 2));
}

extern "C" {

sppStatus sppOnpCreate(sppOnPolicyHandle* out, const sppOnPolicyConfig* cfg, int device) {
  SPP_REQUIRE(out && cfg && cfg->max_batch > 0, SPP_E_INVALID_ARG, "on-policy create: bad args");
  OnpKernels k;
  SPP_REQUIRE(find_onp(cfg->ob, cfg->aout, &k), SPP_E_SHAPE, "no on-policy instantiation for (ob=%d, aout=%d)", cfg->ob,
              cfg->aout);
  SPP_CHECK_HIP(hipSetDevice(device));
  auto o = std::make_unique<sppOnPolicy>();
  o->cfg = *cfg;
  o->device = device;
  o->ks = k;
  hipDeviceProp_t prop;
  SPP_CHECK_HIP(hipGetDeviceProperties(&prop, device));
  o->num_cu = prop.multiProcessorCount;
  o->nsize[0] = onp_actor_size(cfg->ob, cfg->aout);
  o->nsize[1] = onp_critic_size(cfg->ob);
  const int64_t Bp = round_up(cfg->max_batch, 32);
  o->Bpmax = (int)Bp;
  o->pstride = (int)round_up(3 + cfg->aout, 4);
  const int64_t rows = cfg->ob + 64 + 64 + 64 + 64 + std::max(cfg->aout, 1);
  const int64_t total = rows * Bp + (Bp / 32) * o->pstride + 64;
  hipError_t e = o->scratch.alloc(total);
  if (e != hipSuccess) {
    set_error("on-policy scratch alloc: %s", hipGetErrorString(e));
    return SPP_E_OOM;
  }
  SPP_CHECK_HIP(hipMemset(o->scratch.ptr, 0, sizeof(float) * total));
  float* b = o->scratch.ptr;
  o->XT = b; b += cfg->ob * Bp;
  o->H1 = b; b += 64 * Bp;
  o->H2 = b; b += 64 * Bp;
  o->D1 = b; b += 64 * Bp;
  o->D2 = b; b += 64 * Bp;
  o->D3 = b; b += std::max(cfg->aout, 1) * Bp;
  o->part = b;
  *out = o.release();
  return SPP_OK;
}

sppStatus sppOnpDestroy(sppOnPolicyHandle o) {
  if (!o) return SPP_OK;
  hipSetDevice(o->device);
  hipDeviceSynchronize();
  o->lim.release(); o->pk.release(); o->d_pj.release(); o->scratch.release(); o->d_adam.release();
  o->sgd_slab.release(); o->sgd_sync.release();
  for (auto& D : o->dw) D.release();
  delete o;
  return SPP_OK;
}

sppStatus sppOnpNetSize(sppOnPolicyHandle o, int net, int64_t* n) {
  SPP_REQUIRE(o && n && (net == 0 || net == 1), SPP_E_INVALID_ARG, "bad net id");
  *n = o->nsize[net];
  return SPP_OK;
}

sppStatus sppOnpBindNet(sppOnPolicyHandle o, int net, float* p, float* g, float* m, float* v) {
  SPP_REQUIRE(o && (net == 0 || net == 1) && p && g && m && v, SPP_E_INVALID_ARG, "on-policy bind: bad args");
  o->net[net] = NetBufs{p, g, m, v, o->nsize[net]};
  o->pk.release();
  return SPP_OK;
}

sppStatus sppOnpSetLimits(sppOnPolicyHandle o, const float* lim_host) {
  SPP_REQUIRE(o && lim_host, SPP_E_INVALID_ARG, "null");
  if (!o->lim.ptr) SPP_CHECK_HIP(o->lim.alloc(o->cfg.aout));
  SPP_CHECK_HIP(hipMemcpy(o->lim.ptr, lim_host, sizeof(float) * o->cfg.aout, hipMemcpyHostToDevice));
  return SPP_OK;
}

sppStatus sppOnpValue(sppOnPolicyHandle o, const float* x, int N, float* v, void* stream) {
  SPP_REQUIRE(o && x && v, SPP_E_INVALID_ARG, "value: null");
  hipStream_t st = S(stream);
  sppStatus s = onp_ready(o, N, st, 1);
  if (s) return s;
  OnpArgs p = onp_args(o, N);
  p.X = x;
  p.V = v;
  hipLaunchKernelGGL(o->ks.value, dim3(onp_grid(o, N)), dim3(256), 0, st, p);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppOnpCriticGrads(sppOnPolicyHandle o, const float* x, const float* q, int N, float* loss, void* stream) {
  SPP_REQUIRE(o && x && q, SPP_E_INVALID_ARG, "critic grads: null");
  hipStream_t st = S(stream);
  sppStatus s = onp_ready(o, N, st, 1);
  if (s) return s;
  if (o->dw[0].B != N && (s = onp_dw(o, 0, N))) return s;
  OnpArgs p = onp_args(o, N);
  p.X = x;
  p.Q = q;
  hipLaunchKernelGGL(o->ks.critic, dim3(onp_grid(o, N)), dim3(256), 0, st, p);
  SPP_CHECK_HIP(hipGetLastError());
  launch_dw_set(o->dw[0], 0, st);
  hipLaunchKernelGGL(k_onp_finish_critic, dim3(1), dim3(256), 0, st, (const float*)o->part, p.Np / 32, o->pstride, N,
                     loss);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppOnpCriticApply(sppOnPolicyHandle o, void* stream) {
  SPP_REQUIRE(o && o->d_adam.ptr, SPP_E_STATE, "on-policy handle not ready");
  o->steps[1] += 1;
  const double bc1 = 1.0 - std::pow(0.9, (double)o->steps[1]), bc2s = std::sqrt(1.0 - std::pow(0.999, (double)o->steps[1]));
  hipLaunchKernelGGL(k_adam, dim3(std::max(1, std::min(cdiv(o->net[1].n, 1024), 1024)), 1), dim3(256), 0, S(stream),
                     (const AdamJob*)(o->d_adam.ptr + 1), (float)(-(o->cfg.critic_lr / bc1)), (float)bc2s, 0.f);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppOnpActorGrads(sppOnPolicyHandle o, const float* x, const float* act, const float* lp_old,
                           const float* adv, const float* next_obs, int N, float* out4, void* stream) {
  SPP_REQUIRE(o && x && act && lp_old && adv && out4, SPP_E_INVALID_ARG, "actor grads: null");
  hipStream_t st = S(stream);
  sppStatus s = onp_ready(o, N, st, 0);
  if (s) return s;
  if (o->dw[1].B != N && (s = onp_dw(o, 1, N))) return s;
  OnpArgs p = onp_args(o, N);
  p.X = x; p.ACT = act; p.LP_OLD = lp_old; p.ADV = adv; p.NXT = next_obs;
  hipLaunchKernelGGL(o->ks.actor, dim3(onp_grid(o, N)), dim3(256), 0, st, p);
  SPP_CHECK_HIP(hipGetLastError());
  launch_dw_set(o->dw[1], 0, st);
  hipLaunchKernelGGL(k_onp_finish_actor, dim3(1), dim3(256), 0, st, (const float*)o->part, p.Np / 32, o->pstride, N,
                     o->cfg.aout, o->cfg.entropy_coef, (const float*)o->net[0].p, o->net[0].g, out4);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppOnpActorApply(sppOnPolicyHandle o, void* stream) {
  SPP_REQUIRE(o && o->d_adam.ptr, SPP_E_STATE, "on-policy handle not ready");
  o->steps[0] += 1;
  const double bc1 = 1.0 - std::pow(0.9, (double)o->steps[0]), bc2s = std::sqrt(1.0 - std::pow(0.999, (double)o->steps[0]));
  hipLaunchKernelGGL(k_adam, dim3(std::max(1, std::min(cdiv(o->net[0].n, 1024), 1024)), 1), dim3(256), 0, S(stream),
                     (const AdamJob*)o->d_adam.ptr, (float)(-(o->cfg.actor_lr / bc1)), (float)bc2s, 0.f);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

// co-resident workgroups of the multi-workgroup PPO actor epoch kernel (0: no instantiation for these dims)
static int onp_epoch_max_wg(sppOnPolicy* o) {
  if (o->sgd_max_wg >= 0) return o->sgd_max_wg;
  const int ob = o->cfg.ob, aout = o->cfg.aout;
  int n = 0;
  if (ob == 17 && aout == 17) n = mlp_sgd_max_wg<17, 64, 17, 1>(o->num_cu);
  else if (ob == 11 && aout == 11) n = mlp_sgd_max_wg<11, 64, 11, 1>(o->num_cu);
  o->sgd_max_wg = n;
  return n;
}

// slots of a kernel with `full` co-resident workgroups on the device that the reserved CUs take away: each
// reserved CU held a whole workgroup of the concurrent launch (k_mlp_sgd's LDS, > 80 KB for every
// instantiation, fits one per CU), so it removes this kernel's per-CU occupancy, not one slot
static int onp_reserved_slots(sppOnPolicy* o, int full) {
  return o->wg_reserve * std::max(1, cdiv(full, std::max(1, o->num_cu)));
}

int sppOnpActorEpochMaxBatch(sppOnPolicyHandle o) {
  if (!o) return 0;
  const int n = onp_epoch_max_wg(o) - onp_reserved_slots(o, onp_epoch_max_wg(o));
  return n > 0 ? kMlR * n : 0;
}

// gout: one step's reduced gradient into gout (the actor's bound gradient buffer) instead of Adam
static sppStatus onp_actor_run(sppOnPolicyHandle o, const float* x, const float* act, const float* lp_old,
                               const float* adv, const float* next_obs, const int64_t* idx, int nrows, int bs,
                               float* out4, float* gout, float gscale, void* stream) {
  SPP_REQUIRE(o && x && act && lp_old && adv && idx && out4 && nrows >= 0 && bs > 0, SPP_E_INVALID_ARG,
              "actor epoch: bad args");
  const int nsteps = cdiv(nrows, bs);
  SPP_REQUIRE(o->net[0].p && o->net[0].m && o->net[0].v && o->lim.ptr, SPP_E_STATE, "actor epoch: actor not bound");
  const int nwg = cdiv(bs, kMlR), maxwg = onp_epoch_max_wg(o) - onp_reserved_slots(o, onp_epoch_max_wg(o));
  SPP_REQUIRE(maxwg > 0, SPP_E_SHAPE, "actor epoch: no instantiation for ob=%d aout=%d", o->cfg.ob, o->cfg.aout);
  SPP_REQUIRE(nwg <= maxwg, SPP_E_SHAPE, "actor epoch: batch %d needs %d co-resident workgroups > %d", bs, nwg, maxwg);
  if (nsteps == 0) return SPP_OK;
  hipStream_t st = S(stream);
  MlpSgdArgs g{};
  g.x = x; g.y = act; g.nxt = next_obs ? next_obs : act; g.lp_old = lp_old; g.adv = adv; g.idx = idx;
  g.nsteps = nsteps; g.bs = bs; g.bsl = bs; g.bs_last = nrows - (nsteps - 1) * bs;
  const NetBufs& n = o->net[0];
  g.params = n.p; g.m = n.m; g.v = n.v; g.lr = o->cfg.actor_lr; g.step0 = o->steps[0];
  g.lim = o->lim.ptr; g.eps_clip = o->cfg.ppo_epsilon; g.ent_coef = o->cfg.entropy_coef; g.out = out4;
  g.spin = g_sgd_spin; g.gout = gout; g.gscale = gscale;
  if (nwg > 1) {
    g.bsl = cdiv(bs, nwg);
    sppStatus s = mlp_sgd_buffers(o->sgd_slab, o->sgd_sync, st);
    if (s) return s;
    g.slab = o->sgd_slab.ptr;
    g.pbuf = o->sgd_slab.ptr + (size_t)2 * kMlMaxWG * kMlSlabMax;
    g.ctr = sgd_ctr(o->sgd_sync);
    g.err = o->sgd_sync.ptr + 1;
  }
  const bool mw = nwg > 1;
#define SPP_EPOCH_LAUNCH(OB_)                                                                          \
  if (mw) hipLaunchKernelGGL((k_mlp_sgd<OB_, 64, OB_, 1, true>), dim3(nwg), dim3(kMlTH), 0, st, g);     \
  else hipLaunchKernelGGL((k_mlp_sgd<OB_, 64, OB_, 1, false>), dim3(1), dim3(kMlTH), 0, st, g)
  if (o->cfg.ob == 17) SPP_EPOCH_LAUNCH(17);
  else SPP_EPOCH_LAUNCH(11);
#undef SPP_EPOCH_LAUNCH
  if (!gout) o->steps[0] += nsteps;  // (a gradient-only launch takes no Adam step: sppOnpActorApply counts it)
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppOnpActorEpoch(sppOnPolicyHandle o, const float* x, const float* act, const float* lp_old, const float* adv,
                           const float* next_obs, const int64_t* idx, int nrows, int bs, float* out4, void* stream) {
  return onp_actor_run(o, x, act, lp_old, adv, next_obs, idx, nrows, bs, out4, nullptr, 1.f, stream);
}

sppStatus sppOnpActorStepGrads(sppOnPolicyHandle o, const float* x, const float* act, const float* lp_old,
                               const float* adv, const float* next_obs, const int64_t* idx, int N, float* out4,
                               float grad_scale, void* stream) {
  SPP_REQUIRE(o && o->net[0].g && N > 0, SPP_E_STATE, "actor step grads: actor not bound or empty step");
  if (!o->pk.ptr) {  // the handle's Adam jobs (sppOnpActorApply) and pack images, as the phase path sets them up
    sppStatus s = onp_packs(o);
    if (s) return s;
  }
  return onp_actor_run(o, x, act, lp_old, adv, next_obs, idx, N, N, out4, o->net[0].g, grad_scale, stream);
}

// persistent critic steps (HEAD 2): co-resident workgroups, passes of 64 rows per workgroup and step
constexpr int kCriticMaxPasses = 64;  // (the data-parallel PPO union batch: world x 32,768 rows)
// slots the critic grid always leaves free (a concurrent ACM grid of up to 64 workgroups: PPO_AcM), so that
// its row partition -- and with it the gradient's summation order -- is the same with or without one
constexpr int kCriticSideSlots = 64;

static int onp_critic_max_wg(sppOnPolicy* o) {
  if (o->crit_max_wg >= 0) return o->crit_max_wg;
  const int ob = o->cfg.ob;
  int n = 0;
  if (ob == 17) n = mlp_sgd_max_wg<17, 64, 1, 2>(o->num_cu);
  else if (ob == 11) n = mlp_sgd_max_wg<11, 64, 1, 2>(o->num_cu);
  o->crit_max_wg = n;
  return n;
}

static int onp_critic_budget(sppOnPolicy* o) {
  const int full = onp_critic_max_wg(o);
  const int res = onp_reserved_slots(o, full);
  return std::max(0, full > kCriticSideSlots ? full - std::max(res, kCriticSideSlots) : full - res);
}

int sppOnpCriticStepsMaxBatch(sppOnPolicyHandle o) {
  if (!o) return 0;
  const int b = onp_critic_budget(o);
  // one workgroup takes one 64-row pass per step (its single-workgroup form has no passes): batches of more
  // than one tile need >= 2 co-resident workgroups
  return b >= 2 ? kMlR * kCriticMaxPasses * b : (b == 1 ? kMlR : 0);
}

sppStatus sppOnpReserveWorkgroups(sppOnPolicyHandle o, int n) {
  SPP_REQUIRE(o && n >= 0, SPP_E_INVALID_ARG, "reserve workgroups: bad args");
  o->wg_reserve = n;
  return SPP_OK;
}

// gout: one step's reduced gradient into gout (the critic's bound gradient buffer) instead of Adam
static sppStatus onp_critic_run(sppOnPolicyHandle o, const float* x, const float* q, int N, int nsteps, float* loss_sum,
                                float* gout, float gscale, void* stream) {
  SPP_REQUIRE(o && x && q && loss_sum && N > 0 && nsteps >= 0, SPP_E_INVALID_ARG, "critic steps: bad args");
  SPP_REQUIRE(o->net[1].p && o->net[1].m && o->net[1].v && o->lim.ptr, SPP_E_STATE, "critic steps: critic not bound");
  const int maxwg = onp_critic_budget(o);
  SPP_REQUIRE(maxwg > 0, SPP_E_SHAPE, "critic steps: no instantiation for ob=%d (or every slot reserved)", o->cfg.ob);
  // fewest passes per workgroup the co-resident grid allows, then the fewest workgroups for that many passes;
  // more than one tile always runs the multi-workgroup form (G >= 2: the single-workgroup kernel makes one
  // 64-row pass per step)
  const int tiles = cdiv(N, kMlR);
  SPP_REQUIRE(tiles == 1 || maxwg >= 2, SPP_E_SHAPE, "critic steps: batch %d needs >= 2 co-resident workgroups", N);
  const int passes = tiles == 1 ? 1 : cdiv(tiles, maxwg), nwg = tiles == 1 ? 1 : std::max(2, cdiv(tiles, passes));
  SPP_REQUIRE(passes <= kCriticMaxPasses, SPP_E_SHAPE, "critic steps: batch %d > %d", N, kMlR * kCriticMaxPasses * maxwg);
  if (nsteps == 0) return SPP_OK;
  hipStream_t st = S(stream);
  MlpSgdArgs g{};
  g.x = x; g.y = q; g.nsteps = nsteps; g.bs = N; g.bsl = N; g.bs_last = N;
  const NetBufs& n = o->net[1];
  g.params = n.p; g.m = n.m; g.v = n.v; g.lr = o->cfg.critic_lr; g.step0 = o->steps[1];
  g.lim = o->lim.ptr; g.loss_sum = loss_sum; g.spin = g_sgd_spin; g.gout = gout; g.gscale = gscale;
  if (nwg > 1) {
    g.bsl = cdiv(N, nwg);
    sppStatus s = mlp_sgd_buffers(o->sgd_slab, o->sgd_sync, st);
    if (s) return s;
    g.slab = o->sgd_slab.ptr;
    g.pbuf = o->sgd_slab.ptr + (size_t)2 * kMlMaxWG * kMlSlabMax;
    g.ctr = sgd_ctr(o->sgd_sync);
    g.err = o->sgd_sync.ptr + 1;
  }
  const bool mw = nwg > 1;
#define SPP_CRITIC_LAUNCH(OB_)                                                                        \
  if (mw) hipLaunchKernelGGL((k_mlp_sgd<OB_, 64, 1, 2, true>), dim3(nwg), dim3(kMlTH), 0, st, g);     \
  else hipLaunchKernelGGL((k_mlp_sgd<OB_, 64, 1, 2, false>), dim3(1), dim3(kMlTH), 0, st, g)
  if (o->cfg.ob == 17) SPP_CRITIC_LAUNCH(17);
  else SPP_CRITIC_LAUNCH(11);
#undef SPP_CRITIC_LAUNCH
  if (!gout) o->steps[1] += nsteps;  // (a gradient-only launch takes no Adam step: sppOnpCriticApply counts it)
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

sppStatus sppOnpCriticSteps(sppOnPolicyHandle o, const float* x, const float* q, int N, int nsteps, float* loss_sum,
                            void* stream) {
  return onp_critic_run(o, x, q, N, nsteps, loss_sum, nullptr, 1.f, stream);
}

sppStatus sppOnpCriticStepGrads(sppOnPolicyHandle o, const float* x, const float* q, int N, float* loss, float grad_scale,
                                void* stream) {
  SPP_REQUIRE(o && o->net[1].g, SPP_E_STATE, "critic step grads: critic not bound");
  if (!o->pk.ptr) {  // the handle's Adam jobs (sppOnpCriticApply) and pack images, as the phase path sets them up
    sppStatus s = onp_packs(o);
    if (s) return s;
  }
  return onp_critic_run(o, x, q, N, 1, loss, o->net[1].g, grad_scale, stream);
}

sppStatus sppOnpSyncStatusAsync(sppOnPolicyHandle o, int* timed_out_pinned, void* stream) {
  SPP_REQUIRE(o && timed_out_pinned, SPP_E_INVALID_ARG, "onp sync status async: null");
  if (o->sgd_sync.ptr)
    SPP_CHECK_HIP(hipMemcpyAsync(timed_out_pinned, o->sgd_sync.ptr + 1, sizeof(int), hipMemcpyDeviceToHost, S(stream)));
  else
    *timed_out_pinned = 0;
  return SPP_OK;
}

sppStatus sppSetSgdSpinLimit(int polls) {
  g_sgd_spin = polls;  // < 0: every wait gives up at once (sgd_arrive_wait_wt)
  return SPP_OK;
}

sppStatus sppOnpActorEpochStatus(sppOnPolicyHandle o, int* timed_out) {
  SPP_REQUIRE(o && timed_out, SPP_E_INVALID_ARG, "actor epoch status: null");
  *timed_out = 0;
  if (o->sgd_sync.ptr) SPP_CHECK_HIP(hipMemcpy(timed_out, o->sgd_sync.ptr + 1, sizeof(int), hipMemcpyDeviceToHost));
  return SPP_OK;
}

sppStatus sppOnpAct(sppOnPolicyHandle o, const float* x, int N, const float* eps, float* act_out, float* logp_out,
                    void* stream) {
  SPP_REQUIRE(o && x && act_out, SPP_E_INVALID_ARG, "act: null");
  hipStream_t st = S(stream);
  sppStatus s = onp_ready(o, N, st, 0);
  if (s) return s;
  OnpArgs p = onp_args(o, N);
  p.X = x; p.EPS = eps; p.ACT_OUT = act_out; p.LP_OUT = logp_out;
  hipLaunchKernelGGL(o->ks.act, dim3(onp_grid(o, N)), dim3(256), 0, st, p);
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

// ---------------------------------------------------------------- RCCL exchange (§8e)
// librccl is resolved at run time (the one torch already loaded, if any), so the library has no
// link-time RCCL dependency and a C/C++ host can run data parallelism without torch.distributed.
namespace {
struct RcclUid {
  char internal[SPP_COMM_ID_BYTES];
};
struct Rccl {
  int (*get_uid)(RcclUid*) = nullptr;
  int (*init_rank)(void**, int, RcclUid, int) = nullptr;
  int (*destroy)(void*) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  int (*all_gather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  int (*group_start)() = nullptr;
  int (*group_end)() = nullptr;
  const char* (*err)(int) = nullptr;
  bool ok = false;
};
Rccl& rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r;
  tried = true;
  void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!lib) lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) lib = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) return r;
  r.get_uid = (int (*)(RcclUid*))dlsym(lib, "ncclGetUniqueId");
  r.init_rank = (int (*)(void**, int, RcclUid, int))dlsym(lib, "ncclCommInitRank");
  r.destroy = (int (*)(void*))dlsym(lib, "ncclCommDestroy");
  r.all_reduce = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(lib, "ncclAllReduce");
  r.all_gather = (int (*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(lib, "ncclAllGather");
  r.group_start = (int (*)())dlsym(lib, "ncclGroupStart");
  r.group_end = (int (*)())dlsym(lib, "ncclGroupEnd");
  r.err = (const char* (*)(int))dlsym(lib, "ncclGetErrorString");
  r.ok = r.get_uid && r.init_rank && r.destroy && r.all_reduce && r.all_gather && r.group_start && r.group_end && r.err;
  return r;
}
constexpr int kNcclFloat32 = 7, kNcclSum = 0;
}  // namespace

#define SPP_CHECK_RCCL(expr)                                                                   \
  do {                                                                                         \
    const int r_ = (expr);                                                                     \
    if (r_ != 0) {                                                                             \
      ::spp::set_error("%s:%d %s -> rccl %d (%s)", __FILE__, __LINE__, #expr, r_, rccl().err(r_)); \
      return SPP_E_RCCL;                                                                       \
    }                                                                                          \
  } while (0)

__global__ void k_scale(float* x, int64_t n, float s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= s;
}

sppStatus sppCommGetUniqueId(void* uid_out) {
  SPP_REQUIRE(uid_out, SPP_E_INVALID_ARG, "comm uid: null");
  SPP_REQUIRE(rccl().ok, SPP_E_RCCL, "librccl.so.1 not loadable");
  RcclUid u;
  SPP_CHECK_RCCL(rccl().get_uid(&u));
  memcpy(uid_out, &u, sizeof(u));
  return SPP_OK;
}

sppStatus sppCommInitRank(void** comm_out, int nranks, const void* uid, int rank, int device) {
  SPP_REQUIRE(comm_out && uid && nranks > 0 && rank >= 0 && rank < nranks, SPP_E_INVALID_ARG,
              "comm init: nranks %d rank %d", nranks, rank);
  SPP_REQUIRE(rccl().ok, SPP_E_RCCL, "librccl.so.1 not loadable");
  SPP_CHECK_HIP(hipSetDevice(device));
  RcclUid u;
  memcpy(&u, uid, sizeof(u));
  void* c = nullptr;
  SPP_CHECK_RCCL(rccl().init_rank(&c, nranks, u, rank));
  *comm_out = c;
  return SPP_OK;
}

sppStatus sppCommDestroy(void* comm) {
  SPP_REQUIRE(comm, SPP_E_INVALID_ARG, "comm destroy: null");
  SPP_REQUIRE(rccl().ok, SPP_E_RCCL, "librccl.so.1 not loadable");
  SPP_CHECK_RCCL(rccl().destroy(comm));
  return SPP_OK;
}

// In-place sum of a device buffer over the communicator (the obs-statistics exchange of C hosts).
sppStatus sppCommAllReduceSum(void* comm, void* buf, int64_t count, int dtype, void* stream) {
  SPP_REQUIRE(comm && buf && count >= 0 && dtype >= 0 && dtype <= 4, SPP_E_INVALID_ARG,
              "comm allreduce sum: dtype %d count %lld", dtype, (long long)count);
  SPP_REQUIRE(rccl().ok, SPP_E_RCCL, "librccl.so.1 not loadable");
  // ncclFloat32 7, ncclFloat64 8, ncclInt32 2, ncclInt64 4, ncclUint32 3
  static const int kType[5] = {7, 8, 2, 4, 3};
  if (count == 0) return SPP_OK;
  SPP_CHECK_RCCL(rccl().all_reduce(buf, buf, (size_t)count, kType[dtype], kNcclSum, comm, S(stream)));
  return SPP_OK;
}

// Rank-major all-gather of `bytes` per rank (the one-pass statistics' sample exchange); in place when
// send == recv + rank * bytes.
sppStatus sppCommAllGather(void* comm, const void* send, void* recv, int64_t bytes, void* stream) {
  SPP_REQUIRE(comm && send && recv && bytes >= 0, SPP_E_INVALID_ARG, "comm allgather: bad args");
  SPP_REQUIRE(rccl().ok, SPP_E_RCCL, "librccl.so.1 not loadable");
  if (bytes == 0) return SPP_OK;
  SPP_CHECK_RCCL(rccl().all_gather(send, recv, (size_t)bytes, 0 /* ncclInt8 */, comm, S(stream)));
  return SPP_OK;
}

// In-place average of one exchange bucket over the communicator (ncclSum, then x 1/world: the same
// arithmetic as spprl.dp.make_allreduce), stream-ordered between *Grads and *Apply.
sppStatus sppAllReduceGrads(sppAgentHandle h, int bucket, int world, void* rccl_comm, void* stream) {
  SPP_REQUIRE(h && rccl_comm && world > 0 && bucket >= SPP_BUCKET_CRITIC && bucket <= SPP_BUCKET_ALL,
              SPP_E_INVALID_ARG, "allreduce grads: bucket %d world %d", bucket, world);
  SPP_REQUIRE(rccl().ok, SPP_E_RCCL, "librccl.so.1 not loadable");
  hipStream_t st = S(stream);
  std::vector<std::pair<float*, int64_t>> bufs;
  auto add = [&](int net) {
    if (h->net[net].g && h->nsize[net] > 0) bufs.push_back({h->net[net].g, h->nsize[net]});
  };
  const bool all = bucket == SPP_BUCKET_ALL;
  if (all || bucket == SPP_BUCKET_CRITIC) {
    add(SPP_NET_CRITIC1);
    if (!h->ddpg) add(SPP_NET_CRITIC2);
  }
  if (all || bucket == SPP_BUCKET_ACTOR) {
    add(SPP_NET_ACTOR);
    if (!h->ddpg) bufs.push_back({h->alpha_grad, 1});
  }
  if ((all || bucket == SPP_BUCKET_ACM) && !h->plain) add(SPP_NET_ACM);
  SPP_REQUIRE(!bufs.empty(), SPP_E_STATE, "allreduce grads: no gradient buffer bound for bucket %d", bucket);
  SPP_CHECK_RCCL(rccl().group_start());
  for (auto& b : bufs) {
    const int r = rccl().all_reduce(b.first, b.first, (size_t)b.second, kNcclFloat32, kNcclSum, rccl_comm, st);
    if (r != 0) {
      rccl().group_end();
      set_error("ncclAllReduce -> rccl %d (%s)", r, rccl().err(r));
      return SPP_E_RCCL;
    }
  }
  SPP_CHECK_RCCL(rccl().group_end());
  if (world > 1) {
    const float inv = 1.0f / (float)world;
    for (auto& b : bufs)
      hipLaunchKernelGGL(k_scale, dim3(std::max(1, std::min(cdiv(b.second, 256), 1024))), dim3(256), 0, st, b.first,
                         b.second, inv);
  }
  SPP_CHECK_HIP(hipGetLastError());
  return SPP_OK;
}

}  // extern "C"

extern "C" sppStatus sppDebugReadProf(unsigned long long* out64, int reset) {
#ifdef SPP_PROF
  SPP_REQUIRE(out64, SPP_E_INVALID_ARG, "null");
  SPP_CHECK_HIP(hipDeviceSynchronize());
  SPP_CHECK_HIP(hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_tprof), sizeof(unsigned long long) * 64));
  if (reset) {
    unsigned long long z[64] = {};
    SPP_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_tprof), z, sizeof(z)));
  }
  return SPP_OK;
#else
  (void)out64;
  (void)reset;
  set_error("region profiling is only compiled into profiling builds (build.py --prof)");
  return SPP_E_STATE;
#endif
}
