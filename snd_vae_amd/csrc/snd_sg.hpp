#pragma once
#include "snd_common.hpp"

namespace snd {
// SND_SGJOINT graph latent over the spanning-tree copies (model.py:177,180):
//   zbar[b] = (1/S) sum_s z[b S + s]          (fixed order over s)
//   dz[b S + s] = dzbar[b] / S
int launch_sg_mean(const float* z, float* zbar, int B, int S, int L, hipStream_t s);
int launch_sg_spread(const float* dzbar, float* dz, int B, int S, int L, hipStream_t s);
}  // namespace snd
