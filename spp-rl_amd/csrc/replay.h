#pragma once
#include "common.h"

namespace spp {

struct ReplayDev {
  float* obs;
  int64_t* obs_idx;
  int64_t* next_idx;
  float* act;
  float* acm;
  float* rew;
  uint8_t* done;
  uint8_t* end;
  int64_t cap;
  int ob, aout, ac;
};

}  // namespace spp
