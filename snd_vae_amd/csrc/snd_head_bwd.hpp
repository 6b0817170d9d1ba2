// The fused backward head's tile body and the LDS helpers it shares with head_fwd_kernel
// (snd_head.hip) and the fused decoder-backward + backward-head kernel (snd_dec.hip).
#pragma once
#include "snd_head.hpp"
#include "snd_gather.hpp"

namespace snd {
namespace hbk {

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

__device__ __forceinline__ void hglds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds, 16, 0, 0);
}
// 16-byte chunk XOR of a [row][kp] bf16 image (snd_fast.hip swz: conflict-free b128 reads)
__host__ __device__ __forceinline__ int hswz(int row, int kp) {
  return kp == 128 ? (row & 15) : (kp == 64 ? ((row >> 1) & 7) : 0);
}

// LDS-DMA a packed [np][kp] bf16 weight image (whole 1 KB pieces)
__device__ __forceinline__ void stage_img(const __bf16* src, int bytes, char* dst, int nw) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const char* g = reinterpret_cast<const char*>(src) + lane * 16;
  for (int j = w; j < (bytes >> 10); j += nw) hglds16(g + (j << 10), dst + (j << 10));
}

// out^T = W^T x^T over one tap (the row engine's MFMA loop, snd_fast.hip rowconv_kernel):
// lane (li, lg) of wave (rb, nb0) ends with row 16 rb + li, columns 16 (nb0 + i) + 4 lg ..+3
template <int NBH>
__device__ __forceinline__ void img_gemm(const __bf16* xs, const __bf16* ws, int kp, int np, int rb,
                                         int nb0, int li, int lg, f32x4 (&acc)[NBH]) {
  const int nbc = np >> 4;
#pragma unroll
  for (int i = 0; i < NBH; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int xrow = 16 * rb + li;
  const __bf16* xrp = xs + xrow * kp;
  const int xsw = hswz(xrow, kp), wsw = hswz(li, kp);
  const __bf16* wrp = ws + li * kp;
  const int kcs = kp >> 5;
  for (int ks = 0; ks < kcs; ++ks) {
    const int ch = 4 * ks + lg;
    const bf16x8 bx = *reinterpret_cast<const bf16x8*>(xrp + ((ch ^ xsw) << 3));
#pragma unroll
    for (int i = 0; i < NBH; ++i) {
      if (nb0 + i < nbc) {
        const bf16x8 aw = *reinterpret_cast<const bf16x8*>(wrp + 16 * (nb0 + i) * kp + ((ch ^ wsw) << 3));
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, bx, acc[i], 0, 0, 0);
      }
    }
  }
}

// bf16x4 at (row, column n0) of a [row][kp] image (n0 % 4 == 0)
__device__ __forceinline__ bf16x4* img_at4(__bf16* img, int row, int n0, int kp) {
  return reinterpret_cast<bf16x4*>(img + row * kp + (((n0 >> 3) ^ hswz(row, kp)) << 3) + (n0 & 4));
}

// ---------------------------------------------------------------- backward head
// LDS of head_bwd_kernel (bytes): Wms^T image | Wh^T image | d[mu | s] image | dh image |
// per-wave bias sums of d[mu | s]
// Rows per backward-head tile (kHeadBwdRows, snd_head.hpp): 128 rows x 1024 threads
struct BwdLay {
  int w1, w2, m, h, red, total;
  __host__ __device__ BwdLay(int kp1, int np1, int kp2, int np2, int L, int hr = kHeadBwdRows) {
    w1 = 0;
    w2 = np1 * kp1 * 2;
    m = w2 + np2 * kp2 * 2;
    h = m + hr * kp1 * 2;
    red = h + hr * kp2 * 2;
    total = red + (hr / 8) * 2 * L * 4;
  }
};
constexpr int kBwdStaticLds = ((kHeadBwdRows / 16) * 4 * 128 + (kHeadBwdRows / 16) * 128 + 5 * 128) * 4 +
                              (kHeadBwdRows / 8) * 12;

__device__ __forceinline__ float shfl_rows8(float v) {   // sum over the 8 rows a wave holds per sub
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// the tile of workgroup b: XCD-aware (a graph's tiles on one XCD, as the gather kernels'
// row blocks: consecutive workgroups go to consecutive XCDs)
__device__ __forceinline__ int head_tile_xcd(const HeadBwdArgs& a, int HR, int b) {
  int t = b;
  if (a.ngraphs % 8 == 0 && a.npg % HR == 0 && a.ngraphs > 0) {
    const int tpg = a.npg / HR, x = t & 7, sq = t >> 3;
    const int gi = sq / tpg;
    t = (x + 8 * gi) * tpg + (sq - gi * tpg);
  }
  return t;
}

// NQ: 64-column chunks of z per lane (L <= 64: 1); NB1 / NB2: column blocks per wave half
// One backward-head tile (rows [t HR, t HR + HR)) on the calling workgroup (HR * 8
// threads): the body of head_bwd_kernel, and the tail of dec_bwd_head_kernel (snd_dec.hip),
// which runs it on the decoder's tile right after the decoder's backward chain.  smem: the
// dynamic LDS (BwdLay); cps / cpb / colp / sl / stp: the per-tile partial scratch (static
// in head_bwd_kernel, carved from the dynamic LDS past the decoder's use in the fused one).
template <int HR, int NQ, int NB1, int NB2>
__device__ __forceinline__ void head_bwd_tile(const HeadBwdArgs& a, const int t, char* smem,
                                              float (*cps)[4][128], float (*cpb)[128], float (*colp)[128],
                                              double* sl, unsigned* stp) {
  constexpr int HT = HR * 8, HW = HT / 64, NRB = HR / 16;   // threads, waves, 16-row blocks
  const BwdLay lay(a.kp1, a.np1, a.kp2, a.np2, a.L, HR);
  __bf16* w1s = reinterpret_cast<__bf16*>(smem + lay.w1);
  __bf16* w2s = reinterpret_cast<__bf16*>(smem + lay.w2);
  __bf16* ms_img = reinterpret_cast<__bf16*>(smem + lay.m);
  __bf16* dh_img = reinterpret_cast<__bf16*>(smem + lay.h);
  float* bred = reinterpret_cast<float*>(smem + lay.red);
  const int L = a.L, L2 = 2 * L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = t * HR;

  stage_img(a.wmsb_img, a.np1 * a.kp1 * 2, reinterpret_cast<char*>(w1s), HW);
  stage_img(a.whb_img, a.np2 * a.kp2 * 2, reinterpret_cast<char*>(w2s), HW);
  // the dh image's columns [gh, kp2) are the zero k-padding the row engine stages
  for (int i = tid; i < HR * a.kp2 / 8; i += HT) reinterpret_cast<uint4*>(dh_img)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int n = tid; n < 128; n += HT) {   // rowconv RC_ENC1 column parameters
    const bool cv = n < a.W;
    colp[1][n] = cv ? a.ge[n] * kBnC : 0.f;
    colp[3][n] = (cv && n < a.h1) ? a.g1[n] * kBnC : 0.f;
    colp[4][n] = (cv && n < a.h1) ? a.b1[n] : 0.f;
  }

  // ---- 1. per-edge terms of row rs (edge_bf16_kernel) + reparameterisation backward
  {
    const int rs = tid >> 3, sub = tid & 7;
    const int r = r0 + rs;
    const bool rv = r < a.R;
    const int nch = L >> 3;
    bool qv[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) qv[q] = sub + 8 * q < nch;
    float lossr = 0.f;
    unsigned tp = 0;
    // z_i stays packed (bf16 pairs, widened per use): the gather holds 64 VGPRs in flight
    u32x4 zi[NQ];
    float ej[NQ][8];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      zi[q] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 8; ++j) ej[q][j] = 0.f;
    }
    if (rv)
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        if (qv[q]) zi[q] = *reinterpret_cast<const u32x4*>(a.zb + (long long)r * L + 64 * q + 8 * sub);
    const float pw = a.pos_weight;
    if (rv && !(kdbg(a.dbg) & 1)) {
      const __amdgpu_buffer_rsrc_t rsd = rows_rsrc(a.zb, (long long)a.R * L * 2);
      gather_rows16<NQ>(a.colidx, a.rowptr[r], a.rowptr[r + 1], rsd, 2u * L, sub,
                        [&](int, const u32x4 (&v)[NQ], bool valid) {
        float zj[NQ][8], dot = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const unsigned wv = v[q][p];
            zj[q][2 * p] = qv[q] ? __uint_as_float(wv << 16) : 0.f;
            zj[q][2 * p + 1] = qv[q] ? __uint_as_float(wv & 0xFFFF0000u) : 0.f;
          }
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          if (qv[q]) dot = dot8_bf16(zi[q], v[q], dot);   // as edge_bf16_kernel
        const float Lij = row8_sum(dot);
        if (!valid) return;
        float coef;
        edge_ce_terms(Lij, pw, coef, lossr);
        lossr -= pw * Lij;
        tp += Lij > 0.f ? 1u : 0u;
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j) ej[q][j] += coef * zj[q][j];
      });
    }
    if (sub != 0 || !rv) { lossr = 0.f; tp = 0; }   // the row's 8 lanes hold the same sums
    // dz = adj_scale (dJd + ej) + dz_dec; dmu = dz + kl mu; dlogstd = dz eps e^s + kl (e^2s - 1)
    float dm[NQ][8], dl[NQ][8];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { dm[q][j] = 0.f; dl[q][j] = 0.f; }
      const int c0 = 64 * q + 8 * sub;
      if (rv && qv[q]) {
        const float* msr = a.ms + (long long)r * L2;
        const long long ie = (long long)r * L + c0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 mu = *reinterpret_cast<const float4*>(msr + c0 + 4 * h);
          const float4 ls = *reinterpret_cast<const float4*>(msr + L + c0 + 4 * h);
          const float4 ep = *reinterpret_cast<const float4*>(a.eps + ie + 4 * h);
          float4 dj = *reinterpret_cast<const float4*>(a.dJd + ie + 4 * h);
          for (int sx = 0; sx < a.nextra; ++sx) {   // zzt_split_sum_kernel's order
            const float4 e = *reinterpret_cast<const float4*>(a.dJd_extra + (long long)sx * a.R * L + ie + 4 * h);
            dj.x += e.x; dj.y += e.y; dj.z += e.z; dj.w += e.w;
          }
          const float4 dd = *reinterpret_cast<const float4*>(a.dz_dec + ie + 4 * h);
          const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, l4[4] = {ls.x, ls.y, ls.z, ls.w};
          const float e4[4] = {ep.x, ep.y, ep.z, ep.w}, j4[4] = {dj.x, dj.y, dj.z, dj.w};
          const float d4[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
          for (int u = 0; u < 4; ++u)
            reparam_bwd_elem(m4[u], l4[u], e4[u], j4[u], ej[q][4 * h + u], d4[u], a.adj_scale, a.kl_scale,
                             dm[q][4 * h + u], dl[q][4 * h + u]);
        }
      }
      if (qv[q]) {
        bf16x8 om, os;
#pragma unroll
        for (int j = 0; j < 8; ++j) { om[j] = (__bf16)dm[q][j]; os[j] = (__bf16)dl[q][j]; }
        const int cm = c0 >> 3, cs = (L + c0) >> 3;
        *reinterpret_cast<bf16x8*>(ms_img + rs * a.kp1 + ((cm ^ hswz(rs, a.kp1)) << 3)) = om;
        *reinterpret_cast<bf16x8*>(ms_img + rs * a.kp1 + ((cs ^ hswz(rs, a.kp1)) << 3)) = os;
        if (rv && !(kdbg(a.dbg) & 8)) {
          *reinterpret_cast<bf16x8*>(a.dms + (long long)r * L2 + c0) = om;
          *reinterpret_cast<bf16x8*>(a.dms + (long long)r * L2 + L + c0) = os;
        }
        // bias gradient of the [mu | s] head: the wave's 8 rows of this lane's columns
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float sm = shfl_rows8(dm[q][j]), ss = shfl_rows8(dl[q][j]);
          if (lane < 8) { bred[w * L2 + c0 + j] = sm; bred[w * L2 + L + c0 + j] = ss; }
        }
      }
    }
    const double lw = wave_sum_d((double)lossr);
    const unsigned tw = wave_sum_u(tp);
    if (lane == 0) { sl[w] = lw; stp[w] = tw; }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): weight images landed
  __syncthreads();
  if (tid < L2) {
    float v = 0.f;
    for (int k = 0; k < HW; ++k) v += bred[k * L2 + tid];
    a.bms_part[(long long)t * L2 + tid] = v;
  }
  if (tid == 0) {
    double tl = 0.0, tt = 0.0;
    for (int k = 0; k < HW; ++k) { tl += sl[k]; tt += (double)stp[k]; }
    a.edge_part[2 * t] = tl;
    a.edge_part[2 * t + 1] = tt;
  }

  // ---- 2. dh = d[mu | s] Wms^T (row engine RC_LIN, no bias) + its column sums
  const int li = lane & 15, lg = lane >> 4, rb = w % NRB, half = w / NRB;
  const int row = 16 * rb + li, r = r0 + row;
  const bool vrow = r < a.R;
  {
    f32x4 acc1[NB1];
    img_gemm<NB1>(ms_img, w1s, a.kp1, a.np1, rb, NB1 * half, li, lg, acc1);
#pragma unroll
    for (int i = 0; i < NB1; ++i) {
      const int nb = NB1 * half + i;
      if (nb >= (a.np1 >> 4)) continue;
      const int n0 = 16 * nb + 4 * lg;
      const bool cv = vrow && n0 < a.gh;
      float qs[4];
      bf16x4 v4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float o = acc1[i][e] + 0.f;   // the row engine adds a zero bias (-0 becomes +0)
        qs[e] = cv ? o : 0.f;
        v4[e] = (__bf16)o;
      }
      if (n0 < a.gh) *img_at4(dh_img, row, n0, a.kp2) = v4;
      if (cv && !(kdbg(a.dbg) & 8)) *reinterpret_cast<bf16x4*>(a.dh + (long long)r * a.gh + n0) = v4;
#pragma unroll
      for (int e = 0; e < 4; ++e) qs[e] = row16_sum(qs[e]);
      if (li == 0) *reinterpret_cast<float4*>(&cpb[rb][n0]) = make_float4(qs[0], qs[1], qs[2], qs[3]);
    }
  }
  // ENC1 epilogue operands: P1 for the B1 part, X for the feature part
  f32x4 ypf[NB2];
  unsigned cvm[NB2];
#pragma unroll
  for (int i = 0; i < NB2; ++i) {
    ypf[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    cvm[i] = 0u;
    const int nb = NB2 * half + i;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = 16 * nb + 4 * lg + e;
      if (nb < (a.np2 >> 4) && n < a.W) {
        cvm[i] |= 1u << e;
        if (vrow) ypf[i][e] = n < a.h1 ? a.p1[(long long)r * a.h1 + n] : a.x[(long long)r * a.ldx + (n - a.h1)];
      }
    }
  }
  __syncthreads();
  if (tid < a.gh) {
    float v = 0.f;
#pragma unroll
    for (int b = 0; b < NRB; ++b) v += cpb[b][tid];
    a.bh_part[(long long)t * a.gh + tid] = v;
  }

  // ---- 3. dG = dh Wh^T -> BNe / BN1 / lrelu backward (row engine RC_ENC1) -> dP1
  {
    f32x4 acc2[NB2];
    img_gemm<NB2>(dh_img, w2s, a.kp2, a.np2, rb, NB2 * half, li, lg, acc2);
#pragma unroll
    for (int i = 0; i < NB2; ++i) {
      const int nb = NB2 * half + i;
      if (nb >= (a.np2 >> 4)) continue;
      const int n0 = 16 * nb + 4 * lg;
      const unsigned cm = vrow ? cvm[i] : 0u;
      unsigned sm = cm;
      float o[4], qs[4][4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + e;
        const bool ok = cm >> e & 1u;
        const float dg = ok ? acc2[i][e] : 0.f;
        const bool bpart = n < a.h1;
        const float pv = ypf[i][e];
        const float a1 = lrelu(pv);
        const float x2 = bpart ? a1 * colp[3][n] + colp[4][n] : pv;
        qs[0][e] = dg * x2;
        qs[1][e] = dg;
        const float dh2 = dg * colp[1][n];
        o[e] = 0.f;
        qs[2][e] = 0.f;
        qs[3][e] = 0.f;
        if (bpart) {
          qs[2][e] = dh2 * a1;
          qs[3][e] = dh2;
          o[e] = dh2 * colp[3][n] * lrelu_grad(pv);
        } else {
          sm &= ~(1u << e);
        }
      }
      if (!(kdbg(a.dbg) & 8)) {
        __bf16* op = a.dp1 + (long long)r * a.h1 + n0;
        if (sm == 15u) {
          bf16x4 v4;
#pragma unroll
          for (int e = 0; e < 4; ++e) v4[e] = (__bf16)o[e];
          *reinterpret_cast<bf16x4*>(op) = v4;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) if (sm >> e & 1u) op[e] = (__bf16)o[e];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = row16_sum(qs[q][e]);
        if (li == 0) *reinterpret_cast<float4*>(&cps[rb][q][n0]) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < 4 * a.W; i += HT) {
    const int q = i / a.W, n = i - q * a.W;
    float v = 0.f;
#pragma unroll
    for (int b = 0; b < NRB; ++b) v += cps[b][q][n];
    a.enc1_part[(long long)t * 4 * a.W + i] = v;
  }
}


}  // namespace hbk
}  // namespace snd
