// Decode-side kernels for snd_generate (eval / reconstruction / sampling,
// main.py:358-469, model.py:163-169): the predicted adjacency of the inner-
// product decoder.  Not on the training path: one fp32 FMA chain per logit
// (k ascending), so the sign agrees with an fp32 evaluation of J J^T.
#include "snd_decode.hpp"

namespace snd {

constexpr int kGaT = 64;    // output tile (rows and columns)
constexpr int kGaK = 16;    // k chunk staged in LDS

__global__ void __launch_bounds__(256) gen_adj_kernel(GenAdjArgs a) {
  __shared__ float sa[kGaK][kGaT + 4];
  __shared__ float sb[kGaK][kGaT + 4];
  const int g = blockIdx.z, r0 = blockIdx.y * kGaT, c0 = blockIdx.x * kGaT;
  const float* J = a.j + (long long)g * a.n * a.ldj;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[i][q] = 0.f;
  for (int k0 = 0; k0 < a.d; k0 += kGaK) {
    for (int e = threadIdx.x; e < kGaT * kGaK; e += 256) {
      const int rr = e / kGaK, kk = e % kGaK, k = k0 + kk;
      const int ra = r0 + rr, cb = c0 + rr;
      sa[kk][rr] = (ra < a.n && k < a.d) ? J[(long long)ra * a.ldj + k] : 0.f;
      sb[kk][rr] = (cb < a.n && k < a.d) ? J[(long long)cb * a.ldj + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kGaK; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { av[i] = sa[kk][ty * 4 + i]; bv[i] = sb[kk][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] = fmaf(av[i], bv[q], acc[i][q]);
    }
    __syncthreads();
  }
  const bool vec = (a.n & 3) == 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = r0 + ty * 4 + i;
    if (row >= a.n) continue;
    unsigned char* o = a.out + ((long long)g * a.n + row) * a.n;
    const int col = c0 + tx * 4;
    unsigned int bits = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned int v = (col + q != row && acc[i][q] > 0.f) ? 1u : 0u;
      bits |= v << (8 * q);
    }
    if (vec && col + 3 < a.n) {
      *reinterpret_cast<unsigned int*>(o + col) = bits;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (col + q < a.n) o[col + q] = (unsigned char)((bits >> (8 * q)) & 1u);
    }
  }
}

int launch_gen_adj(const GenAdjArgs& a, hipStream_t s) {
  SND_CHECK_ARG(a.j && a.out && a.n > 0 && a.ngraphs > 0 && a.d > 0 && a.ldj >= a.d,
                "gen_adj: bad arguments");
  const int t = (a.n + kGaT - 1) / kGaT;
  hipLaunchKernelGGL(gen_adj_kernel, dim3(t, t, a.ngraphs), dim3(256), 0, s, a);
  SND_LAUNCH_CHECK("gen_adj_kernel");
  return 0;
}

}  // namespace snd
