// Packed bf16 weight images (snd_fast.hpp PackDesc): one 16-byte chunk of an image,
// shared by pack_kernel (snd_fast.hip) and the fused encoder front (snd_head.hip).
#pragma once
#include "snd_fast.hpp"

namespace snd {

// 16-byte chunk XOR of a [row][kp] bf16 image read by ds_read_b128 with lane
// row = l & 15, chunk = 4 ks + (l >> 4) (conflict-free; as the zz^T images).
__host__ __device__ __forceinline__ int img_swz(int row, int kp) {
  return kp >= 128 ? (row & 15) : (kp == 64 ? ((row >> 1) & 7) : 0);
}

// physical chunk i of image d: dst[t][n][8 c .. 8 c + 7] = W values of logical chunk c ^ swz
// chunk i's 8 values (fp32) and its store; pack_chunk = both, back to back
__device__ __forceinline__ void pack_chunk_vals(const PackDesc& d, int i, float (&vals)[8]) {
  const int kc = d.kp >> 3;
  const int c = i % kc, tn = i / kc;
  const int n = tn % d.np, t = tn / d.np;
  const int lc = c ^ img_swz(n, d.kp);          // logical chunk stored at physical chunk c
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * lc + j;
    float val = 0.f;
    for (int si = 0; si < d.nsrc; ++si) {
      const PackSrc& s = d.s[si];
      if (s.mode == 2) {                  // identity over [a0, a1)
        if (k == n && k >= s.a0 && k < s.a1) val = 1.f;
        continue;
      }
      int aa, bb, tt;
      if (s.mode == 0) { bb = n - s.n_off + s.b0; aa = k - s.k_off + s.a0; tt = t; }
      else { aa = n - s.n_off + s.a0; bb = k - s.k_off + s.b0; tt = d.T - 1 - t; }
      if (aa >= s.a0 && aa < s.a1 && bb >= s.b0 && bb < s.b1)
        val = s.w[((long long)tt * s.A + aa) * s.B + bb];
    }
    vals[j] = val;
  }
}
__device__ __forceinline__ void pack_chunk_store(const PackDesc& d, int i, const float (&vals)[8]) {
  const int kc = d.kp >> 3;
  const int c = i % kc, tn = i / kc;
  const int n = tn % d.np, t = tn / d.np;
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)vals[j];
  *reinterpret_cast<bf16x8*>(d.dst + ((long long)(t * d.np + n) * d.kp + 8 * c)) = v;
}
__device__ __forceinline__ void pack_chunk(const PackDesc& d, int i) {
  float vals[8];
  pack_chunk_vals(d, i, vals);
  pack_chunk_store(d, i, vals);
}

__host__ __device__ __forceinline__ int pack_chunks(const PackDesc& d) { return d.T * d.np * (d.kp >> 3); }

}  // namespace snd
