// Graph-latent (T-ref) heads and decoder projection on MI355X (gfx950).
//
// model.py:113-115 applies linear() to tf.reshape(g, [B, -1]): a [B, N*W] x
// [N*W, g_hidden] product whose weight (27.4 M floats at N=4096, W=67) dwarfs
// every activation, and model_joint.py:97 ('d_sg_lin1') projects z [B, L] to
// [B, N*node_h] through a [L, N*node_h] weight (26.2 M floats).  With B <= 8
// graphs per GPU these are weight streams: ~8 FMA per weight element, so each
// kernel is bound by reading (and, backward, writing) its weight once from HBM.
// The layouts keep every weight access a coalesced float4 stream:
//
//   head fwd   thread = (row slot, column quad); rows stride by the slots,
//              G[b, k] broadcast from LDS; split-K partial slab per block.
//   head bwd   two Wh rows per wave instruction (32 lanes x column quads):
//              dWh[k, :] = sum_b G[b, k] dh[b, :] written from registers,
//              dG[b, k] = dh[b, :] . Wh[k, :] reduced over the 32 lanes (DPP).
//   proj fwd   thread = column quad, z broadcast from LDS, 20 loads in flight.
//   proj bwd   thread = column quad holding dJ[:, quad]; wave w owns latent
//              rows l = w (mod 4): dWp written, dz wave-reduced per l (DPP).
//
// Reductions are fixed-order (no float atomics): results are bitwise
// reproducible like the rest of the step.
#include "snd_tref.hpp"

#include <algorithm>

namespace snd {
namespace {

constexpr int B8 = kTrefMaxB;

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ void fma4(float4& acc, float s, const float4& w) {
  acc.x = fmaf(s, w.x, acc.x);
  acc.y = fmaf(s, w.y, acc.y);
  acc.z = fmaf(s, w.z, acc.z);
  acc.w = fmaf(s, w.w, acc.w);
}
__device__ __forceinline__ float dot4(const float4& a, const float4& b) {
  return fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
}

// element (b, k) of flat(G): fp32 [B, K] or the fast encoder's bf16 node rows
template <typename A>
__device__ __forceinline__ float g_at(const A& a, int b, long long k) {
  if (a.gb) {
    const long long n = k / a.W;
    return (float)a.gb[((long long)b * a.npg + n) * a.ldg + (k - n * a.W)];
  }
  return a.g[(long long)b * a.K + k];
}

__device__ __forceinline__ float4 ld_nt(const float* p) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st_nt(float* p, const float4& x) {
  const f32x4 v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}

// fused TF1 Adam on 4 consecutive elements; g is the (complete) gradient.  Every Adam
// kernel divides by v_rcp_f32 of v_sqrt_f32 (1 ulp each) instead of the IEEE div / sqrt
// sequences (~15 VALU per element): the update moves by a few ulp of itself, ~1e-10
// of a parameter; the fused streams are partly VALU-bound (C4 step 0.6277 -> 0.6173 ms)
__device__ __forceinline__ float adam_lrt(const AdamFuse& f) {
  const int t = *f.step + 1;
  return (float)((double)f.lr * sqrt(1.0 - pow((double)f.b2, t)) / (1.0 - pow((double)f.b1, t)));
}
// m, v, p: the moments and parameters as already loaded (issued with the weight loads,
// so a row's update does not wait a memory round trip of its own)
__device__ __forceinline__ void adam4(const AdamFuse& f, float lrt, long long i, const float4& g,
                                      float4 p, float4 m, float4 v) {
  adam_elem(p.x, m.x, v.x, g.x, f.b1, f.b2, f.eps, lrt);
  adam_elem(p.y, m.y, v.y, g.y, f.b1, f.b2, f.eps, lrt);
  adam_elem(p.z, m.z, v.z, g.z, f.b1, f.b2, f.eps, lrt);
  adam_elem(p.w, m.w, v.w, g.w, f.b1, f.b2, f.eps, lrt);
  // streamed once per step: non-temporal stores (no L2 / Infinity Cache allocation)
  st_nt(f.m + i, m);
  st_nt(f.v + i, v);
  st_nt(f.p + i, p);
}

// ------------------------------------------------------------------ head fwd
constexpr int HF_T = 256;

__global__ void __launch_bounds__(HF_T) tref_head_fwd_kernel(TrefHeadFwdArgs a, int rpb) {
  extern __shared__ float sm[];
  const int TPR = a.gh >> 2, RPI = HF_T / TPR;
  const int t = threadIdx.x, q = t % TPR, r = t / TPR;
  const long long k0 = (long long)blockIdx.x * rpb;
  const int nk = (int)std::min<long long>(rpb, a.K - k0);
  // G[b, k0 .. k0+nk) -> gs[kk][8] (coalesced per graph)
  for (int b = 0; b < B8; ++b)
    for (int kk = t; kk < nk; kk += HF_T)
      sm[kk * B8 + b] = b < a.B ? g_at(a, b, k0 + kk) : 0.f;
  __syncthreads();
  float4 acc[B8];
#pragma unroll
  for (int b = 0; b < B8; ++b) acc[b] = f4(0.f);
  if (r < RPI) {
    const float* wrow = a.wh + (k0 + r) * a.gh + 4 * q;
    const long long wstep = (long long)RPI * a.gh;
    int kk = r;
    for (; kk + 7 * RPI < nk; kk += 8 * RPI) {
      float4 w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = *reinterpret_cast<const float4*>(wrow + u * wstep);
      wrow += 8 * wstep;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 g0 = *reinterpret_cast<const float4*>(sm + (kk + u * RPI) * B8);
        const float4 g1 = *reinterpret_cast<const float4*>(sm + (kk + u * RPI) * B8 + 4);
        fma4(acc[0], g0.x, w[u]); fma4(acc[1], g0.y, w[u]);
        fma4(acc[2], g0.z, w[u]); fma4(acc[3], g0.w, w[u]);
        fma4(acc[4], g1.x, w[u]); fma4(acc[5], g1.y, w[u]);
        fma4(acc[6], g1.z, w[u]); fma4(acc[7], g1.w, w[u]);
      }
    }
    // the last < 8 rows: all loads issued before the first FMA (one memory round trip)
    float4 w[7];
#pragma unroll
    for (int u = 0; u < 7; ++u)
      w[u] = kk + u * RPI < nk ? *reinterpret_cast<const float4*>(wrow + u * wstep) : f4(0.f);
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      if (kk + u * RPI >= nk) break;
      const float4 g0 = *reinterpret_cast<const float4*>(sm + (kk + u * RPI) * B8);
      const float4 g1 = *reinterpret_cast<const float4*>(sm + (kk + u * RPI) * B8 + 4);
      fma4(acc[0], g0.x, w[u]); fma4(acc[1], g0.y, w[u]); fma4(acc[2], g0.z, w[u]); fma4(acc[3], g0.w, w[u]);
      fma4(acc[4], g1.x, w[u]); fma4(acc[5], g1.y, w[u]); fma4(acc[6], g1.z, w[u]); fma4(acc[7], g1.w, w[u]);
    }
  }
  __syncthreads();
  // reduce the row slots: red[r][b][gh]
  if (r < RPI)
#pragma unroll
    for (int b = 0; b < B8; ++b)
      *reinterpret_cast<float4*>(sm + (r * B8 + b) * a.gh + 4 * q) = acc[b];
  __syncthreads();
  const int outs = a.B * a.gh;
  for (int o = t; o < outs; o += HF_T) {
    float s = 0.f;
    for (int rr = 0; rr < RPI; ++rr) s += sm[rr * B8 * a.gh + o];
    if (blockIdx.x == 0) s += a.bh[o % a.gh];
    a.slab[(long long)blockIdx.x * outs + o] = s;
  }
}

int head_fwd_rpb(long long K, int gh) {
  const int RPI = HF_T / (gh / 4);
  long long rpb = round_up(cdiv(K, 1024), RPI);
  rpb = std::max<long long>(rpb, 4LL * RPI);
  return (int)std::min<long long>(rpb, 1024);
}

// ------------------------------------------------------------------ head bwd
// Two rows of Wh per wave instruction: lanes 32h + q (h = row of the pair, q =
// column quad, q < gh/4 active).  dWh is written straight from registers; the
// per-row dot products dG[b, k] = dh[b, :] . Wh[k, :] are reduced over the 32
// lanes of the half with DPP (row16) + one xor-16 swizzle, and parked in LDS so
// dG leaves the block as coalesced rows.
// (rows per block, row pairs / rows in flight: other values measured flat or worse, round 3)
constexpr int HB_T = 256, HB_RPB = 256;

__global__ void __launch_bounds__(HB_T) tref_head_bwd_kernel(TrefHeadBwdArgs a) {
  __shared__ float gs[HB_RPB * B8];      // G[b, k0 + kk] as [kk][8]
  __shared__ float dgs[2][B8 * HB_RPB];  // dG[b, k0 + kk] as [b][kk]: the two 16-lane halves' sums
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int h = lane >> 5, q = lane & 31;
  const int TPR = a.gh >> 2;
  const bool qa = q < TPR;
  const long long k0 = (long long)blockIdx.x * HB_RPB;
  const int nk = (int)std::min<long long>(HB_RPB, a.K - k0);
  for (int b = 0; b < B8; ++b)
    for (int kk = t; kk < nk; kk += HB_T)
      gs[kk * B8 + b] = b < a.B ? g_at(a, b, k0 + kk) : 0.f;
  float4 dh[B8];
#pragma unroll
  for (int b = 0; b < B8; ++b)
    dh[b] = (qa && b < a.B) ? *reinterpret_cast<const float4*>(a.dh + b * a.gh + 4 * q) : f4(0.f);
  __syncthreads();
  const bool fused = a.adam.p != nullptr;
  const float lrt = fused ? adam_lrt(a.adam) : 0.f;
  constexpr int U = 4;                   // row pairs in flight per wave
  const int r0 = 2 * wv + h;             // row slot of this lane; 8 rows per block pass
  for (int base = 0; base < nk; base += 8 * U) {
    float4 w[U], am[U], av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = base + 8 * u + r0;
      const bool ld = qa && kk < nk;
      const long long i = (k0 + (ld ? kk : 0)) * a.gh + 4 * q;
      w[u] = ld ? ld_nt(a.wh + i) : f4(0.f);
      am[u] = av[u] = f4(0.f);
      if (fused && ld) {
        am[u] = ld_nt(a.adam.m + i);
        av[u] = ld_nt(a.adam.v + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = base + 8 * u + r0;
      const bool rv = kk < nk;
      const int kc = rv ? kk : 0;
      const float4 g0 = *reinterpret_cast<const float4*>(gs + kc * B8);
      const float4 g1 = *reinterpret_cast<const float4*>(gs + kc * B8 + 4);
      const float gb[B8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      float4 dw = f4(0.f);
#pragma unroll
      for (int b = 0; b < B8; ++b) fma4(dw, gb[b], dh[b]);
      if (qa && rv) {
        if (fused) adam4(a.adam, lrt, (k0 + kk) * a.gh + 4 * q, dw, w[u], am[u], av[u]);
        else *reinterpret_cast<float4*>(a.dwh + (k0 + kk) * a.gh + 4 * q) = dw;
      }
      // all lanes active: inactive quads hold 0.  Each 16-lane half parks its sum; the
      // halves are added at the store (same order as a cross-half swizzle, no LDS permute)
      float p[B8];
#pragma unroll
      for (int b = 0; b < B8; ++b) p[b] = row16_sum(dot4(dh[b], w[u]));
      if ((q & 15) == 0 && rv)
#pragma unroll
        for (int b = 0; b < B8; ++b) dgs[q >> 4][b * HB_RPB + kk] = p[b];
    }
  }
  __syncthreads();
  for (int b = 0; b < a.B; ++b)
    for (int kk = t; kk < nk; kk += HB_T) {
      const long long k = k0 + kk;
      const float v = dgs[0][b * HB_RPB + kk] + dgs[1][b * HB_RPB + kk];
      if (a.dgb) {
        const long long n = k / a.W;
        a.dgb[((long long)b * a.npg + n) * a.ldg + (k - n * a.W)] = (__bf16)v;
      } else {
        a.dg[(long long)b * a.K + k] = v;
      }
    }
}

// ------------------------------------------------------------------ proj fwd
// Block = 64 column quads x 4 waves; wave w sums latent rows [w L / 4, (w + 1) L / 4)
// (one wave per SIMD was too few loads in flight), wave 0 adds the other waves'
// partials in wave order and stores: J = b_p + ((S_0 + S_1) + S_2) + S_3.
constexpr int PF_W = 4;
__global__ void __launch_bounds__(64 * PF_W) tref_proj_fwd_kernel(TrefProjFwdArgs a) {
  __shared__ float zs[128 * B8];          // [l][8]
  __shared__ float4 part[PF_W - 1][B8][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < a.L * B8; i += 64 * PF_W) {
    const int l = i >> 3, b = i & 7;
    zs[i] = b < a.B ? a.z[b * a.L + l] : 0.f;
  }
  __syncthreads();
  const long long c4 = 4LL * ((long long)blockIdx.x * 64 + lane);
  const bool live = c4 < a.Cp;            // a dead lane still reaches the barrier
  float4 acc[B8];
#pragma unroll
  for (int b = 0; b < B8; ++b) acc[b] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* wcol = a.wp + (live ? c4 : 0);
  const int l1 = (w + 1) * a.L / PF_W;
  int l = w * a.L / PF_W;
  constexpr int U = 10;
  for (; l + U - 1 < l1; l += U) {
    float4 wv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) wv[u] = *reinterpret_cast<const float4*>(wcol + (long long)(l + u) * a.Cp);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float4 z0 = *reinterpret_cast<const float4*>(zs + (l + u) * B8);
      const float4 z1 = *reinterpret_cast<const float4*>(zs + (l + u) * B8 + 4);
      fma4(acc[0], z0.x, wv[u]); fma4(acc[1], z0.y, wv[u]); fma4(acc[2], z0.z, wv[u]);
      fma4(acc[3], z0.w, wv[u]); fma4(acc[4], z1.x, wv[u]); fma4(acc[5], z1.y, wv[u]);
      fma4(acc[6], z1.z, wv[u]); fma4(acc[7], z1.w, wv[u]);
    }
  }
  {   // the last < U rows: all loads issued before the first FMA
    float4 wr[U - 1];
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      wr[u] = l + u < l1 ? *reinterpret_cast<const float4*>(wcol + (long long)(l + u) * a.Cp) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < U - 1; ++u) {
      if (l + u >= l1) break;
      const float4 z0 = *reinterpret_cast<const float4*>(zs + (l + u) * B8);
      const float4 z1 = *reinterpret_cast<const float4*>(zs + (l + u) * B8 + 4);
      fma4(acc[0], z0.x, wr[u]); fma4(acc[1], z0.y, wr[u]); fma4(acc[2], z0.z, wr[u]); fma4(acc[3], z0.w, wr[u]);
      fma4(acc[4], z1.x, wr[u]); fma4(acc[5], z1.y, wr[u]); fma4(acc[6], z1.z, wr[u]); fma4(acc[7], z1.w, wr[u]);
    }
  }
  if (w > 0)
#pragma unroll
    for (int b = 0; b < B8; ++b) part[w - 1][b][lane] = acc[b];
  __syncthreads();
  if (w > 0 || !live) return;
  const float4 bias = *reinterpret_cast<const float4*>(a.bp + c4);
#pragma unroll
  for (int b = 0; b < B8; ++b) {
    float4 s = acc[b];
#pragma unroll
    for (int v = 0; v < PF_W - 1; ++v) {
      const float4 o = part[v][b][lane];
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    s.x += bias.x; s.y += bias.y; s.z += bias.z; s.w += bias.w;
    if (b < a.B) *reinterpret_cast<float4*>(a.j + (long long)b * a.Cp + c4) = s;
  }
}

// ------------------------------------------------------------------ proj bwd
// Block = 64 column quads (256 columns) x 4 waves; wave w owns latent rows
// l = w (mod 4).  Every lane keeps dJ[b, its quad] in registers (combined from the
// three producers on load), streams Wp[l, quad] in and dWp[l, quad] out, and the
// 8 dot products per l are wave-reduced with DPP; lane 0 parks them in LDS, and
// the block writes one [B][L] dz partial.
constexpr int PB_T = 256, PB_W = PB_T / 64;

__global__ void __launch_bounds__(PB_T) tref_proj_bwd_kernel(TrefProjBwdArgs a) {
  __shared__ float zs[128 * B8];         // z as [l][8]
  __shared__ float red[4][128 * B8];     // dz partials as [16-lane row][l][8]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int i = t; i < a.L * B8; i += PB_T) {
    const int l = i >> 3, b = i & 7;
    zs[i] = b < a.B ? a.z[b * a.L + l] : 0.f;
  }
  const long long c4 = 4LL * ((long long)blockIdx.x * 64 + lane);
  const bool cv = c4 < a.Cp;
  float4 d[B8];
#pragma unroll
  for (int b = 0; b < B8; ++b) {
    d[b] = f4(0.f);
    if (cv && b < a.B) {
      const long long i = (long long)b * a.Cp + c4;
      const float4 x = *reinterpret_cast<const float4*>(a.dz_dec + i);
      const float4 y = *reinterpret_cast<const float4*>(a.dJd + i);
      const float4 z = *reinterpret_cast<const float4*>(a.ej + i);
      d[b] = make_float4(fmaf(a.adj_scale, y.x + z.x, x.x), fmaf(a.adj_scale, y.y + z.y, x.y),
                         fmaf(a.adj_scale, y.z + z.z, x.z), fmaf(a.adj_scale, y.w + z.w, x.w));
    }
  }
  if (wv == 0 && cv) {
    float4 s = d[0];
#pragma unroll
    for (int b = 1; b < B8; ++b) { s.x += d[b].x; s.y += d[b].y; s.z += d[b].z; s.w += d[b].w; }
    if (a.adam_b.p)
      adam4(a.adam_b, adam_lrt(a.adam_b), c4, s, ld_nt(a.adam_b.p + c4), ld_nt(a.adam_b.m + c4),
            ld_nt(a.adam_b.v + c4));
    else
      *reinterpret_cast<float4*>(a.dbp + c4) = s;
  }
  __syncthreads();
  const bool fused = a.adam.p != nullptr;
  const float lrt = fused ? adam_lrt(a.adam) : 0.f;
  constexpr int U = 5;                   // weight rows in flight per thread
  for (int l0 = wv; l0 < a.L; l0 += PB_W * U) {
    float4 w[U], am[U], av[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int l = l0 + PB_W * u;
      const bool ld = cv && l < a.L;
      const long long i = (long long)(ld ? l : 0) * a.Cp + (cv ? c4 : 0);
      w[u] = ld ? ld_nt(a.wp + i) : f4(0.f);
      am[u] = av[u] = f4(0.f);
      if (fused && ld) {
        am[u] = ld_nt(a.adam.m + i);
        av[u] = ld_nt(a.adam.v + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int l = l0 + PB_W * u;
      if (l >= a.L) break;                       // wave-uniform
      const float4 z0 = *reinterpret_cast<const float4*>(zs + l * B8);
      const float4 z1 = *reinterpret_cast<const float4*>(zs + l * B8 + 4);
      float4 dw = f4(0.f);
      fma4(dw, z0.x, d[0]); fma4(dw, z0.y, d[1]); fma4(dw, z0.z, d[2]); fma4(dw, z0.w, d[3]);
      fma4(dw, z1.x, d[4]); fma4(dw, z1.y, d[5]); fma4(dw, z1.z, d[6]); fma4(dw, z1.w, d[7]);
      if (cv) {
        if (fused) adam4(a.adam, lrt, (long long)l * a.Cp + c4, dw, w[u], am[u], av[u]);
        else *reinterpret_cast<float4*>(a.dwp + (long long)l * a.Cp + c4) = dw;
      }
#pragma unroll
      for (int b = 0; b < B8; ++b) {   // each 16-lane row parks its sum (no LDS permutes)
        const float p = row16_sum(dot4(d[b], w[u]));
        if ((lane & 15) == 0) red[lane >> 4][l * B8 + b] = p;
      }
    }
  }
  __syncthreads();
  for (int i = t; i < a.L * a.B; i += PB_T) {
    const int b = i / a.L, l = i - b * a.L;
    const int j = l * B8 + b;   // (R0 + R1) + (R2 + R3): the order of the xor-16 / xor-32 swizzles
    a.slab[(long long)blockIdx.x * a.B * a.L + i] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
  }
}

// ------------------------------------------------------------------ Adam (float4)
__global__ void __launch_bounds__(256) adam_vec_kernel(float4* p, const float4* g, float4* m,
                                                       float4* v, long long n4, float lr, float b1,
                                                       float b2, float eps, float gscale,
                                                       const int* step) {
  // the first element's loads go out before the bias-correction arithmetic (f64 pow)
  // so its memory round trip overlaps it (small buffers: one element per thread)
  const long long i0 = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long st = (long long)gridDim.x * 256;
  float4 gi, mi, vi, pi;
  if (i0 < n4) { gi = g[i0]; mi = m[i0]; vi = v[i0]; pi = p[i0]; }
  const int t = *step;
  const double lr_t = (double)lr * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t));
  const float lrt = (float)lr_t;
  for (long long i = i0; i < n4; i += st) {
    if (i != i0) { gi = g[i]; mi = m[i]; vi = v[i]; pi = p[i]; }
    adam_elem(pi.x, mi.x, vi.x, __fmul_rn(gi.x, gscale), b1, b2, eps, lrt);
    adam_elem(pi.y, mi.y, vi.y, __fmul_rn(gi.y, gscale), b1, b2, eps, lrt);
    adam_elem(pi.z, mi.z, vi.z, __fmul_rn(gi.z, gscale), b1, b2, eps, lrt);
    adam_elem(pi.w, mi.w, vi.w, __fmul_rn(gi.w, gscale), b1, b2, eps, lrt);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

// several disjoint float4 ranges of the same flat buffers in one launch (the blocks an
// in-step fused update leaves: C4 has three); same arithmetic as adam_vec_kernel
struct AdamRanges {
  long long off4[kAdamMaxRanges], start4[kAdamMaxRanges + 1];
  int n;
};
__global__ void __launch_bounds__(256) adam_ranges_kernel(float4* p, const float4* g, float4* m, float4* v,
                                                          AdamRanges rg, float lr, float b1, float b2,
                                                          float eps, float gscale, const int* step) {
  const long long tot = rg.start4[rg.n];
  const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
  long long i = -1;
  if (j < tot) {
    int r = 0;
    while (r + 1 < rg.n && j >= rg.start4[r + 1]) ++r;
    i = rg.off4[r] + (j - rg.start4[r]);
  }
  float4 gi, mi, vi, pi;
  if (i >= 0) { gi = g[i]; mi = m[i]; vi = v[i]; pi = p[i]; }
  const int t = *step;
  const double lr_t = (double)lr * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t));
  const float lrt = (float)lr_t;
  if (i < 0) return;
  adam_elem(pi.x, mi.x, vi.x, __fmul_rn(gi.x, gscale), b1, b2, eps, lrt);
  adam_elem(pi.y, mi.y, vi.y, __fmul_rn(gi.y, gscale), b1, b2, eps, lrt);
  adam_elem(pi.z, mi.z, vi.z, __fmul_rn(gi.z, gscale), b1, b2, eps, lrt);
  adam_elem(pi.w, mi.w, vi.w, __fmul_rn(gi.w, gscale), b1, b2, eps, lrt);
  m[i] = mi;
  v[i] = vi;
  p[i] = pi;
}

}  // namespace

int launch_adam_ranges(float* p, const float* g, float* m, float* v, const long long* off,
                       const long long* cnt, int n, float lr, float b1, float b2, float eps, float gscale,
                       const int* step, hipStream_t s) {
  SND_CHECK_ARG(n >= 1 && n <= kAdamMaxRanges, "adam_ranges: 1..%d ranges", kAdamMaxRanges);
  SND_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                "adam_ranges: 16-byte aligned buffers");
  AdamRanges rg{};
  rg.n = n;
  long long acc = 0;
  for (int k = 0; k < n; ++k) {
    SND_CHECK_ARG(off[k] >= 0 && cnt[k] >= 0 && off[k] % 4 == 0 && cnt[k] % 4 == 0,
                  "adam_ranges: offsets and counts must be multiples of 4");
    rg.off4[k] = off[k] / 4;
    rg.start4[k] = acc;
    acc += cnt[k] / 4;
  }
  rg.start4[n] = acc;
  if (acc == 0) return 0;
  hipLaunchKernelGGL(adam_ranges_kernel, dim3((unsigned)cdiv(acc, 256)), dim3(256), 0, s,
                     reinterpret_cast<float4*>(p), reinterpret_cast<const float4*>(g),
                     reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v), rg, lr, b1, b2, eps, gscale,
                     step);
  SND_LAUNCH_CHECK("adam_ranges_kernel");
  return 0;
}

int tref_head_fwd_blocks(long long K, int gh) { return cdiv(K, head_fwd_rpb(K, gh)); }

int launch_tref_head_fwd(const TrefHeadFwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(a.B >= 1 && a.B <= B8 && a.gh % 4 == 0 && a.gh >= 4 && a.gh <= 128 && a.K > 0,
                "tref_head_fwd: B in 1..8, g_hidden %% 4 in 4..128");
  SND_CHECK_ARG((a.g || (a.gb && a.W > 0 && a.npg > 0 && a.ldg >= a.W && (long long)a.W * a.npg == a.K)) &&
                    a.wh && a.bh && a.slab, "tref_head_fwd: null operand / bf16 G geometry");
  const int rpb = head_fwd_rpb(a.K, a.gh);
  const int RPI = HF_T / (a.gh / 4);
  const size_t lds = sizeof(float) * std::max<size_t>((size_t)rpb * B8, (size_t)RPI * B8 * a.gh);
  hipLaunchKernelGGL(tref_head_fwd_kernel, dim3(tref_head_fwd_blocks(a.K, a.gh)), dim3(HF_T), lds, s, a,
                     rpb);
  SND_LAUNCH_CHECK("tref_head_fwd_kernel");
  return 0;
}

int launch_tref_head_bwd(const TrefHeadBwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(a.B >= 1 && a.B <= B8 && a.gh % 4 == 0 && a.gh >= 4 && a.gh <= 128 && a.K > 0,
                "tref_head_bwd: B in 1..8, g_hidden %% 4 in 4..128");
  SND_CHECK_ARG((a.g || (a.gb && a.W > 0 && a.npg > 0 && a.ldg >= a.W && (long long)a.W * a.npg == a.K)) &&
                    a.wh && a.dh && (a.dwh || a.adam.p) && (a.dg || (a.dgb && a.gb)),
                "tref_head_bwd: null operand / bf16 G geometry");
  SND_CHECK_ARG(!a.adam.p || (a.adam.m && a.adam.v && a.adam.step && a.adam.p == a.wh),
                "tref_head_bwd: fused Adam needs m, v, step and p == wh");
  hipLaunchKernelGGL(tref_head_bwd_kernel, dim3(cdiv(a.K, HB_RPB)), dim3(HB_T), 0, s, a);
  SND_LAUNCH_CHECK("tref_head_bwd_kernel");
  return 0;
}

int launch_tref_proj_fwd(const TrefProjFwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(a.B >= 1 && a.B <= B8 && a.L >= 1 && a.L <= 128 && a.Cp % 4 == 0 && a.Cp > 0,
                "tref_proj_fwd: B in 1..8, L <= 128, Cp %% 4");
  SND_CHECK_ARG(a.z && a.wp && a.bp && a.j, "tref_proj_fwd: null operand");
  hipLaunchKernelGGL(tref_proj_fwd_kernel, dim3(cdiv(a.Cp / 4, 64)), dim3(64 * PF_W), 0, s, a);
  SND_LAUNCH_CHECK("tref_proj_fwd_kernel");
  return 0;
}

int tref_proj_bwd_blocks(long long Cp) { return cdiv(Cp, 256); }

int launch_tref_proj_bwd(const TrefProjBwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(a.B >= 1 && a.B <= B8 && a.L >= 1 && a.L <= 128 && a.Cp % 4 == 0 && a.Cp > 0,
                "tref_proj_bwd: B in 1..8, L <= 128, Cp %% 4");
  SND_CHECK_ARG(a.z && a.wp && a.dz_dec && a.dJd && a.ej && (a.dwp || a.adam.p) && (a.dbp || a.adam_b.p) &&
                    a.slab, "tref_proj_bwd: null operand");
  SND_CHECK_ARG(!a.adam.p || (a.adam.m && a.adam.v && a.adam.step && a.adam.p == a.wp),
                "tref_proj_bwd: fused Adam needs m, v, step and p == wp");
  SND_CHECK_ARG(!a.adam_b.p || (a.adam_b.m && a.adam_b.v && a.adam_b.step),
                "tref_proj_bwd: fused bias Adam needs m, v, step");
  hipLaunchKernelGGL(tref_proj_bwd_kernel, dim3(tref_proj_bwd_blocks(a.Cp)), dim3(PB_T), 0, s, a);
  SND_LAUNCH_CHECK("tref_proj_bwd_kernel");
  return 0;
}

int launch_adam_vec(float* p, const float* g, float* m, float* v, long long n, float lr, float b1,
                    float b2, float eps, float gscale, const int* step, hipStream_t s) {
  SND_CHECK_ARG(n % 4 == 0 && ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                "adam_vec: n %% 4 and 16-byte aligned buffers");
  if (n == 0) return 0;
  const long long n4 = n / 4;
  const int blocks = (int)std::min<long long>(cdiv(n4, 256), 8192);
  hipLaunchKernelGGL(adam_vec_kernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<float4*>(p),
                     reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(m),
                     reinterpret_cast<float4*>(v), n4, lr, b1, b2, eps, gscale, step);
  SND_LAUNCH_CHECK("adam_vec_kernel");
  return 0;
}

}  // namespace snd
