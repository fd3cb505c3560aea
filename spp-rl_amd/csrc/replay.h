#pragma once
#include "common.h"

namespace spp {

// The HBM replay ring (rltoolkit/buffer/replay_buffer.py: MetaReplayBuffer's obs-index ring + the
// BufferAcMOffPolicy timestep arrays).  Observations are stored once per obs slot, row-major.  Everything
// else a timestep holds is ONE 64-B-aligned record of rw 32-bit words, so a sampled transition reads one
// record segment and two obs rows instead of seven scattered arrays (8-B obs / next indices, 4-B reward,
// 1-B done, the action and ACM rows, each touching its own 64-B line):
//   word 0  obs slot            word 1  next-obs slot        word 2  reward (fp32 bits)
//   word 3  done (bit 0) | end (bit 8)
//   words 4 .. 4 + ac - 1            the ACM (env) action  (within the first 64 B for ac <= 12)
//   words 4 + ac .. 4 + ac + aout - 1 the actor output the buffer stores as "action"
// obs_idx keeps the obs slot of every timestep as its own array too: the obs statistics read every live
// row through it in order (replay_buffer.py:83-96), where a contiguous index stream is the right layout.
struct ReplayDev {
  float* obs;        // [cap][ob]
  int64_t* obs_idx;  // [cap]
  uint32_t* rec;     // [cap][rw]
  int64_t cap;
  int ob, aout, ac;
  int rw;            // record words: 4 + ac + aout rounded up to 16 (a multiple of 64 B)
  const int* acm_cols;  // AcMTrainer.acm_ob_idx (acm.py:94-99, 260-264): the ob columns of acm_cat, or null
};
constexpr int kRecAcm = 4;  // first ACM word
__host__ __device__ inline int rec_words(int aout, int ac) { return (kRecAcm + ac + aout + 15) / 16 * 16; }
__host__ __device__ inline int rec_act(const ReplayDev& r) { return kRecAcm + r.ac; }  // first action word

}  // namespace spp
