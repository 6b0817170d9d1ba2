// Fused encoder heads of the node-latent bf16 fast path.
//
// head_fwd_kernel replaces four launches of the step's forward (the GraphConvolution 1
// SpMM with its epilogue, the two head linears on the row engine, reparam_prep) with
// one: a workgroup owns 128 rows of one graph and
//   1. gathers A XW1 for its rows (the spmm_bf16_kernel engine: 8 lanes per row,
//      16 neighbours in flight, fp32 sums in colidx order) and applies the
//      GraphConvolution 1 epilogue (layers.py:122-123, model.py:107-112): P1 (fp32)
//      and G = BNe([BN1(lrelu(P1)) | X]) leave for the backward pass, G also lands in
//      LDS as the [row][k] image the row engine would have staged from HBM;
//   2. h = G Wh + bh (model.py:113) on v_mfma_f32_16x16x32_bf16 from that image and
//      the packed weight image (LDS-DMA'd during the gather), bf16 h to HBM (the Wms
//      weight gradient reads it) and to LDS;
//   3. [mu | s] = h Wms + bms (model.py:114-115), fp32 to HBM; the s half crosses to
//      the mu waves through LDS;
//   4. z = mu + eps e^s (model.py:159), the KL partials (optimizer.py:193), bf16 z and
//      the zz^T staging images (z sqrt(log2 e), its transpose, per-64-row column sums).
// Every product and epilogue is the unfused kernels' own arithmetic in the same order:
// P1, G, h, [mu | s], z, eps, the staging images and the column sums equal theirs bit
// for bit (tests/test_gpu_step.py); only the KL partials group their rows differently.
#include "snd_head.hpp"
#include "snd_gather.hpp"
#include "snd_pack.hpp"

#include <algorithm>

namespace snd {
namespace {

// HR rows of one graph per workgroup, 8 lanes per row in the gather: HR * 8 threads.
// 64-row tiles (8 waves, ~73 KB LDS at C2) put two workgroups on a CU, so one's
// gather latency overlaps the other's GEMMs and stores (the 128-row variant, one per CU,
// measured slower and was removed in round 5).
constexpr int kHeadRows = 64;
constexpr int HWMAX = 16;
constexpr float kSqrtLog2e = 1.2011224087864498f;
__device__ __forceinline__ int cdiv_dev(int a, int b) { return (a + b - 1) / b; }

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

__device__ __forceinline__ void hglds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds, 16, 0, 0);
}
// 16-byte chunk XOR of a [row][kp] bf16 image (snd_fast.hip swz: conflict-free b128 reads)
__host__ __device__ __forceinline__ int hswz(int row, int kp) {
  return kp == 128 ? (row & 15) : (kp == 64 ? ((row >> 1) & 7) : 0);
}

// LDS layout (bytes) of head_fwd_kernel, shared by host and device.  The [mu | s]
// exchange (fp32 2 x [HR][L + 4]) reuses the weight, G and h images, dead after step 3.
struct FwdLay {
  int w2, w1, g, h, zt, total, sx_end;
  __host__ __device__ FwdLay(int HR, int kp1, int np1, int kp2, int np2, int L) {
    w2 = 0;
    w1 = np2 * kp2 * 2;
    g = w1 + np1 * kp1 * 2;
    h = g + HR * kp1 * 2;
    zt = h + HR * kp2 * 2;
    total = zt + HR * (L + 1) * 4;
    sx_end = 2 * HR * (L + 4) * 4;
  }
};
constexpr int kHeadStaticLds = 2 * 128 * 4 + 2 * HWMAX * 8;
constexpr int kHeadDynLds = 160 * 1024 - kHeadStaticLds - 512;

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

template <int HR, int NB1, int NB2>
__global__ void __launch_bounds__(HR * 8) head_fwd_kernel(HeadFwdArgs a) {
  constexpr int HT = HR * 8, HW = HT / 64, NRB = HR / 16;   // threads, waves, 16-row blocks
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float cb1[128], cb2[128];   // bh, bms per physical column
  __shared__ double klw[2 * HWMAX];
  const FwdLay lay(HR, a.kp1, a.np1, a.kp2, a.np2, a.L);
  __bf16* w2s = reinterpret_cast<__bf16*>(smem + lay.w2);
  __bf16* w1s = reinterpret_cast<__bf16*>(smem + lay.w1);
  __bf16* gs = reinterpret_cast<__bf16*>(smem + lay.g);
  __bf16* hs = reinterpret_cast<__bf16*>(smem + lay.h);
  float* mx = reinterpret_cast<float*>(smem);                        // [HR][L + 4] mu, then
  float* sx = reinterpret_cast<float*>(smem + HR * (a.L + 4) * 4);   // s: over the dead images
  float* zt = reinterpret_cast<float*>(smem + lay.zt);
  const int L = a.L, sxs = L + 4, zts = L + 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tpg = a.npad / HR;
  // XCD-aware tile order (as head_bwd and the gather kernels): blocks b and b + 8 share an
  // XCD, so graph g's tiles go to block group g % 8 and its gathered XW1 rows stay in one L2
  // (natural order spread every graph over all 8 L2s: 32 MB fetched per launch)
  int tb = blockIdx.x;
  if (a.ngraphs % 8 == 0 && a.ngraphs > 0) {
    const int x = tb & 7, sq = tb >> 3;
    const int g8 = sq / tpg;
    tb = (x + 8 * g8) * tpg + (sq - g8 * tpg);
  }
  const int gi = tb / tpg, lt = tb - gi * tpg;
  const int lr0 = lt * HR;                          // first row of the tile in its graph
  const long long gr0 = (long long)gi * a.npg;      // the graph's first global row

  // ---- weight images in flight during the gather; biases; zero h image (pad columns)
  stage_img(a.wh_img, a.np1 * a.kp1 * 2, reinterpret_cast<char*>(w1s), HW);
  stage_img(a.wms_img, a.np2 * a.kp2 * 2, reinterpret_cast<char*>(w2s), HW);
  for (int i = tid; i < 128; i += HT) {
    cb1[i] = i < a.gh ? a.bh[i] : 0.f;
    cb2[i] = i < 2 * L ? a.bms[i] : 0.f;
  }
  for (int i = tid; i < HR * a.kp2 / 8; i += HT) reinterpret_cast<uint4*>(hs)[i] = make_uint4(0u, 0u, 0u, 0u);

  // ---- 1. P1 = A XW1 for row rs (8 lanes), GraphConvolution 1 epilogue
  const int rs = tid >> 3, sub = tid & 7;
  const int lr = lr0 + rs;
  const bool rv = lr < a.npg;
  const long long r = gr0 + lr;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (rv && !(kdbg(a.dbg) & 1)) {
    const __amdgpu_buffer_rsrc_t rsd = rows_rsrc(a.xw1, (long long)a.R * a.h1 * 2);
    gather_rows16<1>(a.colidx, a.rowptr[r], a.rowptr[r + 1], rsd, 2u * a.h1, sub,
                     [&](int, const u32x4 (&v)[1], bool) { acc8v(acc, v[0]); });
  }
  const int nch = a.h1 >> 3, kc1 = a.kp1 >> 3;
  uint4 gdat = make_uint4(0u, 0u, 0u, 0u), gxv = make_uint4(0u, 0u, 0u, 0u);
  if (sub < nch) {
    float gv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * sub + j;
      const float b1 = lrelu(acc[j]) * (a.g1[c] * kBnC) + a.b1[c];     // H2[:, :h1]
      gv[j] = b1 * (a.ge[c] * kBnC) + a.be[c];                          // encoder_g BN
    }
    gdat = to_bf16x8(gv);
  }
  // the concat-X chunk (model.py:109) is chunk nch: lane nch's first or lane nch-8's second
  const int xo = (sub == nch) ? 0 : (sub + 8 == nch ? 1 : -1);
  if (xo >= 0 && rv) {
    float gv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = a.h1 + j;
      gv[j] = j < a.f ? a.x[r * a.ldx + j] * (a.ge[c] * kBnC) + a.be[c] : 0.f;
    }
    gxv = to_bf16x8(gv);
  }
  {
    // chunk sub: data, the X chunk or zeros; chunk sub + 8: the X chunk or zeros
    // (component selects: a select of whole vectors goes through scratch)
    const bool d0 = sub < nch, x0 = xo == 0, x1 = xo == 1;
    const uint4 v0 = make_uint4(d0 ? gdat.x : (x0 ? gxv.x : 0u), d0 ? gdat.y : (x0 ? gxv.y : 0u),
                                d0 ? gdat.z : (x0 ? gxv.z : 0u), d0 ? gdat.w : (x0 ? gxv.w : 0u));
    const uint4 v1 = make_uint4(x1 ? gxv.x : 0u, x1 ? gxv.y : 0u, x1 ? gxv.z : 0u, x1 ? gxv.w : 0u);
    if (sub < kc1) *reinterpret_cast<uint4*>(gs + rs * a.kp1 + ((sub ^ hswz(rs, a.kp1)) << 3)) = v0;
    if (sub + 8 < kc1) *reinterpret_cast<uint4*>(gs + rs * a.kp1 + (((sub + 8) ^ hswz(rs, a.kp1)) << 3)) = v1;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): weight images landed (gathers consumed)
  __syncthreads();
  // P1 and G leave for the backward pass while the heads run
  if (rv && !(kdbg(a.dbg) & 8)) {
    if (sub < nch) {
      float* pp = a.p1 + r * a.h1 + 8 * sub;
      *reinterpret_cast<float4*>(pp) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(pp + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      *reinterpret_cast<uint4*>(a.g + r * a.ldg + 8 * sub) = gdat;
    }
    if (xo >= 0) *reinterpret_cast<uint4*>(a.g + r * a.ldg + a.h1) = gxv;
  }

  // ---- 2. h = G Wh + bh
  const int li = lane & 15, lg = lane >> 4, rb = w % NRB, half = w / NRB;
  const int row = 16 * rb + li, lrw = lr0 + row;
  const bool vrow = lrw < a.npg;
  const long long rr = gr0 + lrw;
  {
    f32x4 acc1[NB1];
    if (kdbg(a.dbg) & 16) { for (int i = 0; i < NB1; ++i) acc1[i] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    else img_gemm<NB1>(gs, w1s, a.kp1, a.np1, rb, NB1 * half, li, lg, acc1);
#pragma unroll
    for (int i = 0; i < NB1; ++i) {
      const int n0 = 16 * (NB1 * half + i) + 4 * lg;
      if (n0 >= a.gh) continue;
      bf16x4 v4;
#pragma unroll
      for (int e = 0; e < 4; ++e) v4[e] = (__bf16)(acc1[i][e] + cb1[n0 + e]);
      *img_at4(hs, row, n0, a.kp2) = v4;
      if (vrow && !(kdbg(a.dbg) & 8)) *reinterpret_cast<bf16x4*>(a.hh + rr * a.gh + n0) = v4;
    }
  }
  __syncthreads();

  // ---- 3. [mu | s] = h Wms + bms; both halves go to LDS (the weight and h images are dead)
  {
    f32x4 acc2[NB2];
    if (kdbg(a.dbg) & 16) { for (int i = 0; i < NB2; ++i) acc2[i] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    else img_gemm<NB2>(hs, w2s, a.kp2, a.np2, rb, NB2 * half, li, lg, acc2);
    float o[NB2][4];
#pragma unroll
    for (int i = 0; i < NB2; ++i) {
      const int n0 = 16 * (NB2 * half + i) + 4 * lg;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[i][e] = acc2[i][e] + cb2[n0 + e];
      if (vrow && !(kdbg(a.dbg) & 8))
        *reinterpret_cast<float4*>(a.ms + rr * (2 * L) + n0) = make_float4(o[i][0], o[i][1], o[i][2], o[i][3]);
    }
    __syncthreads();   // every wave is past its MFMA reads of the Wms and h images
#pragma unroll
    for (int i = 0; i < NB2; ++i) {
      const int n0 = 16 * (NB2 * half + i) + 4 * lg;   // half 0: mu columns, half 1: s columns
      *reinterpret_cast<float4*>((half ? sx : mx) + row * sxs + (n0 - half * L)) =
          make_float4(o[i][0], o[i][1], o[i][2], o[i][3]);
    }
  }
  __syncthreads();

  // ---- 4. z = mu + eps e^s, KL, bf16 z, z sqrt(log2 e) rows, z into LDS for the transpose;
  // every wave takes rows x Philox quads of the tile
  {
    const unsigned off = a.step ? (unsigned)(*a.step) : 0u;
    if (a.stepn && blockIdx.x == 0 && tid == 0) *a.stepn = (int)off + 1;
    const int nq = L >> 2;
    double kl[HR / 64];
#pragma unroll
    for (int h = 0; h < HR / 64; ++h) kl[h] = 0.0;
    for (int it = (kdbg(a.dbg) & 32) ? HR * nq : tid; it < HR * nq; it += HT) {
      const int zr = it / nq, c = 4 * (it - zr * nq);
      const int zl = lr0 + zr;
      float z4[4] = {0.f, 0.f, 0.f, 0.f};
      if (zl < a.npg) {
        const long long ie = (gr0 + zl) * L + c;
        const float4 m4 = *reinterpret_cast<const float4*>(mx + zr * sxs + c);
        const float4 s4 = *reinterpret_cast<const float4*>(sx + zr * sxs + c);
        const float4 ep = a.eps_in ? *reinterpret_cast<const float4*>(a.eps_in + ie)
                                   : philox_normal4(a.seed, off, (a.eps_base + (unsigned long long)ie) >> 2);
        const float mu[4] = {m4.x, m4.y, m4.z, m4.w}, s[4] = {s4.x, s4.y, s4.z, s4.w};
        const float e[4] = {ep.x, ep.y, ep.z, ep.w};
        double kq = 0.0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float es = __expf(s[t]);
          z4[t] = mu[t] + e[t] * es;                                          // model.py:159
          kq += (double)kl_elem(s[t], mu[t]);        // optimizer.py:193
        }
#pragma unroll
        for (int h = 0; h < HR / 64; ++h) kl[h] += (zr >> 6) == h ? kq : 0.0;
        if (!(kdbg(a.dbg) & 8)) {
          *reinterpret_cast<float4*>(a.z + ie) = make_float4(z4[0], z4[1], z4[2], z4[3]);
          *reinterpret_cast<float4*>(a.eps_out + ie) = ep;
          bf16x4 zb;
#pragma unroll
          for (int t = 0; t < 4; ++t) zb[t] = (__bf16)z4[t];
          *reinterpret_cast<bf16x4*>(a.zb + ie) = zb;
        }
      }
      bf16x4 jb;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        jb[t] = (__bf16)(z4[t] * kSqrtLog2e);
        zt[zr * zts + c + t] = z4[t];
      }
      *reinterpret_cast<bf16x4*>(a.jrow + ((long long)gi * a.npad + zl) * L + c) = jb;
    }
#pragma unroll
    for (int h = 0; h < HR / 64; ++h) {
      const double v = wave_sum_d(kl[h]);
      if (lane == 0) klw[h * HWMAX + w] = v;
    }
  }
  __syncthreads();
  // per-64-row column sums of the stored K-role values (reparam_prep order)
  for (int i = (kdbg(a.dbg) & 64) ? HT * HR : tid; i < (HR / 64) * L; i += HT) {
    const int h = i / L, c = i - h * L;
    float cs = 0.f;
    for (int q0 = 0; q0 < 64; q0 += 16) {   // 16 reads in flight, the sum in row order
      float t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = zt[(64 * h + q0 + u) * zts + c];
#pragma unroll
      for (int u = 0; u < 16; ++u) cs += (float)(__bf16)(t[u] * kSqrtLog2e);
    }
    a.colpart[((long long)gi * (a.npad / 64) + (HR / 64) * lt + h) * L + c] = cs;
  }
  // z^T image: 4 consecutive rows per lane
  for (int idx = (kdbg(a.dbg) & 64) ? HT * HR : tid; idx < (HR / 4) * L; idx += HT) {
    const int c = idx / (HR / 4), r4 = 4 * (idx % (HR / 4));
    bf16x4 t;
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = (__bf16)zt[(r4 + u) * zts + c];
    *reinterpret_cast<bf16x4*>(a.jt + ((long long)gi * L + c) * a.npad + lr0 + r4) = t;
  }
  if (tid < HR / 64) {   // the 64-row block's partial: every wave's share, in wave order
    double v = 0.0;
    for (int k = 0; k < HW; ++k) v += klw[tid * HWMAX + k];
    a.kl_part[(long long)gi * (a.npad / 64) + (HR / 64) * lt + tid] = v;
  }
}

template <int HR, int NB1, int NB2>
int head_fwd_launch(const HeadFwdArgs& a, hipStream_t s) {
  const size_t lds = (size_t)FwdLay(HR, a.kp1, a.np1, a.kp2, a.np2, a.L).total;
  hipLaunchKernelGGL((head_fwd_kernel<HR, NB1, NB2>), dim3(a.ngraphs * (a.npad / HR)), dim3(HR * 8), lds, s, a);
  SND_LAUNCH_CHECK("head_fwd_kernel");
  return 0;
}
template <int HR>
int head_fwd_dispatch(const HeadFwdArgs& a, hipStream_t s) {
  const int nb1 = (a.np1 / 16 + 1) / 2, nb2 = a.np2 / 32;
  if (nb1 == 1) return nb2 == 2 ? head_fwd_launch<HR, 1, 2>(a, s) : head_fwd_launch<HR, 1, 4>(a, s);
  return nb2 == 2 ? head_fwd_launch<HR, 2, 2>(a, s) : head_fwd_launch<HR, 2, 4>(a, s);
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

// NQ: 64-column chunks of z per lane (L <= 64: 1); NB1 / NB2: column blocks per wave half
template <int HR, int NQ, int NB1, int NB2>
__global__ void __launch_bounds__(HR * 8) head_bwd_kernel(HeadBwdArgs a) {
  constexpr int HT = HR * 8, HW = HT / 64, NRB = HR / 16;   // threads, waves, 16-row blocks
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ __attribute__((aligned(16))) float cps[NRB][4][128];   // ENC1 column partials per 16-row block
  __shared__ __attribute__((aligned(16))) float cpb[NRB][128];      // dh column partials per 16-row block
  __shared__ float colp[5][128];                                     // ENC1 per-column parameters
  __shared__ double sl[HW];
  __shared__ unsigned stp[HW];
  const BwdLay lay(a.kp1, a.np1, a.kp2, a.np2, a.L, HR);
  __bf16* w1s = reinterpret_cast<__bf16*>(smem + lay.w1);
  __bf16* w2s = reinterpret_cast<__bf16*>(smem + lay.w2);
  __bf16* ms_img = reinterpret_cast<__bf16*>(smem + lay.m);
  __bf16* dh_img = reinterpret_cast<__bf16*>(smem + lay.h);
  float* bred = reinterpret_cast<float*>(smem + lay.red);
  const int L = a.L, L2 = 2 * L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // tile: XCD-aware (a graph's tiles on one XCD, as the gather kernels' row blocks)
  int t = blockIdx.x;
  if (a.ngraphs % 8 == 0 && a.npg % HR == 0 && a.ngraphs > 0) {
    const int tpg = a.npg / HR, x = t & 7, sq = t >> 3;
    const int gi = sq / tpg;
    t = (x + 8 * gi) * tpg + (sq - gi * tpg);
  }
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

template <int NQ, int NB1, int NB2>
int head_bwd_launch(const HeadBwdArgs& a, hipStream_t s) {
  const int hr = head_bwd_rows(a.R);
  const size_t lds = (size_t)BwdLay(a.kp1, a.np1, a.kp2, a.np2, a.L, hr).total;
  if (hr == kHeadBwdTinyRows)
    hipLaunchKernelGGL((head_bwd_kernel<kHeadBwdTinyRows, NQ, NB1, NB2>), dim3(head_tiles(a.R)),
                       dim3(kHeadBwdTinyRows * 8), lds, s, a);
  else if (hr == 64)
    hipLaunchKernelGGL((head_bwd_kernel<64, NQ, NB1, NB2>), dim3(head_tiles(a.R)), dim3(64 * 8), lds, s, a);
  else
    hipLaunchKernelGGL((head_bwd_kernel<kHeadBwdRows, NQ, NB1, NB2>), dim3(head_tiles(a.R)),
                       dim3(kHeadBwdRows * 8), lds, s, a);
  SND_LAUNCH_CHECK("head_bwd_kernel");
  return 0;
}

// ---------------------------------------------------------------- encoder front
// One 128-row tile per workgroup: AX by the gcn0 gather (8 lanes per row, the fp32
// features of the neighbours), H1 = [BN0(lrelu(AX W0)) | X] to HBM (the W1 weight
// gradient and the backward read it) and into LDS, then XW1 = H1 W1 on MFMA with the
// W1 image built in LDS from the fp32 weights (pack_kernel's image, bit for bit).
// Workgroups past the tiles build the step's packed weight images (pack_chunk).
template <int NB>
__global__ void __launch_bounds__(1024) enc_front_kernel(FrontArgs a) {
  const int tid = threadIdx.x;
  const int ntiles = cdiv_dev(a.R, 128);
  if ((int)blockIdx.x >= ntiles) {
    const int pb = blockIdx.x - ntiles;
    int s = 0;
    while (s + 1 < a.npack && pb >= a.pack_wg[s + 1]) ++s;
    s = __builtin_amdgcn_readfirstlane(s);
    const PackDesc& d = a.pack[s];
    const int i = (pb - a.pack_wg[s]) * 1024 + tid;
    if (i < pack_chunks(d)) pack_chunk(d, i);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float sp[6][128];     // W0 rows (f <= 4), gamma0 * c, beta0
  __bf16* wimg = reinterpret_cast<__bf16*>(smem);
  __bf16* himg = reinterpret_cast<__bf16*>(smem + a.np1 * a.kp1 * 2);
  const int r0 = blockIdx.x * 128;
  const int K1 = a.h0 + a.f;
  for (int i = tid; i < a.h0; i += 1024) {
#pragma unroll
    for (int q = 0; q < 4; ++q) sp[q][i] = q < a.f ? a.w0[q * a.h0 + i] : 0.f;
    sp[4][i] = a.g0[i] * kBnC;
    sp[5][i] = a.b0[i];
  }
  __syncthreads();   // sp[] (read by the H1 math below)
  // W1 image [np1][kp1]: element (n, k) = W1[k][n] (pack mode 0).  Its loads are issued
  // before the A X gather and written to LDS after it, so their latency overlaps the
  // gather's dependent rowptr -> colidx -> x chain instead of preceding it (np1 * kp1 / 8
  // <= 1024 chunks: one per thread at the C2 widths, loops otherwise)
  const int kc = a.kp1 >> 3;
  const bool w1one = a.np1 * kc <= 1024;
  float w1v[8];
  if (w1one && tid < a.np1 * kc) {
    const int c = tid % kc, n = tid / kc;
    const int lc = c ^ img_swz(n, a.kp1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * lc + j;
      w1v[j] = (k < K1 && n < a.n1) ? a.w1[k * a.n1 + n] : 0.f;
    }
  }
  // ---- AX for row rs (gcn0_kernel: two neighbours in flight per lane)
  const int rs = tid >> 3, sub = tid & 7;
  const int r = r0 + rs;
  const bool rv = r < a.R;
  float ax[4] = {0.f, 0.f, 0.f, 0.f};
  if (rv) {
    const int s = a.rowptr[r], e = a.rowptr[r + 1];
    int k = s + sub;
    for (; k + 8 < e; k += 16) {
      const int c0 = a.colidx[k], c1 = a.colidx[k + 8];
      float v0[4], v1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v0[j] = j < a.f ? a.x[(long long)c0 * a.ldx + j] : 0.f;
        v1[j] = j < a.f ? a.x[(long long)c1 * a.ldx + j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) ax[j] += v0[j] + v1[j];
    }
    if (k < e) {
      const int c0 = a.colidx[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) ax[j] += j < a.f ? a.x[(long long)c0 * a.ldx + j] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) ax[j] = row8_sum(ax[j]);
  // ---- H1 = [BN0(lrelu(AX W0)) | X]: lane sub owns chunk sub; the X chunk is chunk h0 / 8
  const int nch = a.h0 >> 3, kc1 = a.kp1 >> 3;
  uint4 hd = make_uint4(0u, 0u, 0u, 0u), hx = make_uint4(0u, 0u, 0u, 0u);
  if (sub < nch) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 8 * sub + j;
      float p = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) p += ax[q] * sp[q][col];
      o[j] = lrelu(p) * sp[4][col] + sp[5][col];
    }
    hd = to_bf16x8(o);
  }
  const int xo = (sub == nch) ? 0 : (sub + 8 == nch ? 1 : -1);
  if (xo >= 0 && rv) {
    float xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = j < a.f ? a.x[(long long)r * a.ldx + j] : 0.f;
    hx = to_bf16x8(xv);
  }
  {
    const bool d0 = sub < nch, x0 = xo == 0, x1 = xo == 1;
    const uint4 v0 = make_uint4(d0 ? hd.x : (x0 ? hx.x : 0u), d0 ? hd.y : (x0 ? hx.y : 0u),
                                d0 ? hd.z : (x0 ? hx.z : 0u), d0 ? hd.w : (x0 ? hx.w : 0u));
    const uint4 v1 = make_uint4(x1 ? hx.x : 0u, x1 ? hx.y : 0u, x1 ? hx.z : 0u, x1 ? hx.w : 0u);
    if (sub < kc1) *reinterpret_cast<uint4*>(himg + rs * a.kp1 + ((sub ^ hswz(rs, a.kp1)) << 3)) = v0;
    if (sub + 8 < kc1) *reinterpret_cast<uint4*>(himg + rs * a.kp1 + (((sub + 8) ^ hswz(rs, a.kp1)) << 3)) = v1;
  }
  if (w1one) {
    if (tid < a.np1 * kc) {
      const int c = tid % kc, n = tid / kc;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__bf16)w1v[j];
      *reinterpret_cast<bf16x8*>(wimg + n * a.kp1 + 8 * c) = v;
    }
  } else {
    for (int i = tid; i < a.np1 * kc; i += 1024) {
      const int c = i % kc, n = i / kc;
      const int lc = c ^ img_swz(n, a.kp1);
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * lc + j;
        v[j] = (__bf16)((k < K1 && n < a.n1) ? a.w1[k * a.n1 + n] : 0.f);
      }
      *reinterpret_cast<bf16x8*>(wimg + n * a.kp1 + 8 * c) = v;
    }
  }
  if (rv && !(kdbg(a.dbg) & 8)) {
    if (sub < nch) *reinterpret_cast<uint4*>(a.h1 + (long long)r * a.ldh1 + 8 * sub) = hd;
    if (xo >= 0) *reinterpret_cast<uint4*>(a.h1 + (long long)r * a.ldh1 + a.h0) = hx;
    if (sub == 0) {
      *reinterpret_cast<float4*>(a.ax + (long long)r * 4) = make_float4(ax[0], ax[1], ax[2], ax[3]);
      const float axp[8] = {ax[0], ax[1], ax[2], ax[3], 0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<uint4*>(a.axb + (long long)r * 8) = to_bf16x8(axp);
    }
  }
  __syncthreads();
  // ---- XW1 = H1 W1 (row engine RC_LIN, no bias)
  const int lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lg = lane >> 4, rb = w & 7, half = w >> 3;
  const int row = 16 * rb + li, rr = r0 + row;
  f32x4 acc[NB];
  img_gemm<NB>(himg, wimg, a.kp1, a.np1, rb, NB * half, li, lg, acc);
  if (rr >= a.R || (kdbg(a.dbg) & 8)) return;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n0 = 16 * (NB * half + i) + 4 * lg;
    if (n0 >= a.n1) continue;
    bf16x4 v4;
#pragma unroll
    for (int e = 0; e < 4; ++e) v4[e] = (__bf16)(acc[i][e] + 0.f);   // the row engine's zero bias
    *reinterpret_cast<bf16x4*>(a.xw1 + (long long)rr * a.n1 + n0) = v4;
  }
}

}  // namespace

bool front_supported(int f, int h0, int n1, int kp1, int np1) {
  return f >= 1 && f <= 4 && h0 % 8 == 0 && h0 >= 8 && h0 <= 64 && h0 + 8 <= kp1 && n1 % 16 == 0 &&
         np1 == n1 && np1 <= 128 && (kp1 == 32 || kp1 == 64 || kp1 == 128) &&
         (np1 + 128) * kp1 * 2 + 6 * 128 * 4 <= 160 * 1024;
}

int launch_front(FrontArgs& a, const PackDesc* pack, int npack, hipStream_t s) {
  if (a.R <= 0) return 0;
  SND_CHECK_ARG(front_supported(a.f, a.h0, a.n1, a.kp1, a.np1), "front: unsupported widths (f %d h0 %d n1 %d)",
                a.f, a.h0, a.n1);
  SND_CHECK_ARG(npack >= 0 && npack <= kMaxPack, "front: at most %d packed images", kMaxPack);
  SND_CHECK_ARG(a.rowptr && (a.colidx || a.R == 0) && a.x && a.w0 && a.g0 && a.b0 && a.h1 && a.ax && a.axb &&
                    a.w1 && a.xw1 && a.ldh1 % 8 == 0 && a.ldh1 >= a.h0 + 8,
                "front: operands");
  a.npack = npack;
  int wg = 0;
  for (int i = 0; i < npack; ++i) {
    const PackDesc& x = pack[i];
    SND_CHECK_ARG((x.kp == 32 || x.kp == 64 || x.kp == 128) && x.np % 16 == 0 && x.np > 0 && x.T >= 1 &&
                      x.nsrc >= 1 && x.nsrc <= 2,
                  "front: bad pack descriptor %d", i);
    a.pack[i] = x;
    a.pack_wg[i] = wg;
    wg += cdiv(pack_chunks(x), 1024);
  }
  a.pack_wg[npack] = wg;
  SND_TRY(head_init_attributes());
  const size_t lds = (size_t)(a.np1 + 128) * a.kp1 * 2;
  const dim3 grid(cdiv(a.R, 128) + wg);
  switch ((a.np1 / 16 + 1) / 2) {
    case 1: hipLaunchKernelGGL((enc_front_kernel<1>), grid, dim3(1024), lds, s, a); break;
    case 2: hipLaunchKernelGGL((enc_front_kernel<2>), grid, dim3(1024), lds, s, a); break;
    case 3: hipLaunchKernelGGL((enc_front_kernel<3>), grid, dim3(1024), lds, s, a); break;
    default: hipLaunchKernelGGL((enc_front_kernel<4>), grid, dim3(1024), lds, s, a); break;
  }
  SND_LAUNCH_CHECK("enc_front_kernel");
  return 0;
}

int head_bwd_rows(int R) {
  if (cdiv(R, kHeadBwdRows) >= kHeadBwdSmall) return kHeadBwdRows;
  return cdiv(R, 64) < kHeadBwdTiny ? kHeadBwdTinyRows : 64;
}
int head_tiles(int R) { return cdiv(R, head_bwd_rows(R)); }

bool head_bwd_supported(int L, int gh, int W, int h1, int kp1, int np1, int kp2, int np2) {
  if ((L != 16 && L != 32 && L != 64) || kp1 != 2 * L) return false;
  if (gh % 16 || gh < 16 || np1 != gh || np1 > 64 || gh > kp2 || (kp2 != 32 && kp2 != 64 && kp2 != 128)) return false;
  if (W > 128 || np2 != (int)round_up(W, 16) || h1 % 4 || h1 > W) return false;
  return BwdLay(kp1, np1, kp2, np2, L).total + kBwdStaticLds <= 160 * 1024;
}

int launch_head_bwd(const HeadBwdArgs& a, hipStream_t s) {
  if (a.R <= 0) return 0;
  SND_CHECK_ARG(head_bwd_supported(a.L, a.gh, a.W, a.h1, a.kp1, a.np1, a.kp2, a.np2),
                "head_bwd: unsupported widths (L %d gh %d W %d h1 %d)", a.L, a.gh, a.W, a.h1);
  SND_CHECK_ARG((long long)a.R * a.L * 2 < (1ll << 31), "head_bwd: rows x L beyond the 2 GB buffer range");
  SND_CHECK_ARG(a.rowptr && (a.colidx || a.R == 0) && a.zb && a.edge_part && a.ms && a.eps && a.dz_dec &&
                    a.dJd && a.dms && a.bms_part && a.wmsb_img && a.dh && a.bh_part && a.whb_img && a.ge &&
                    a.g1 && a.b1 && a.p1 && a.x && a.dp1 && a.enc1_part,
                "head_bwd: null operand");
  SND_TRY(head_init_attributes());
  const int nb1 = (a.np1 / 16 + 1) / 2, nb2 = (a.np2 / 16 + 1) / 2;
#define SND_HB(B1)                                   \
  switch (nb2) {                                     \
    case 1: return head_bwd_launch<1, B1, 1>(a, s);  \
    case 2: return head_bwd_launch<1, B1, 2>(a, s);  \
    case 3: return head_bwd_launch<1, B1, 3>(a, s);  \
    default: return head_bwd_launch<1, B1, 4>(a, s); \
  }
  if (nb1 == 1) { SND_HB(1) } else { SND_HB(2) }
#undef SND_HB
}

bool head_fwd_supported(int h1, int f, int gh, int L, int kp1, int np1, int kp2, int np2) {
  if (h1 % 8 || h1 < 8 || h1 > 64 || f < 1 || f > 8) return false;
  if ((kp1 != 32 && kp1 != 64 && kp1 != 128) || (kp2 != 32 && kp2 != 64 && kp2 != 128)) return false;
  if (h1 + 8 > kp1 || gh % 16 || gh < 16 || np1 != gh || np1 > 64 || gh > kp2) return false;
  if ((L != 32 && L != 64) || np2 != 2 * L) return false;
  const FwdLay l64(64, kp1, np1, kp2, np2, L), l128(128, kp1, np1, kp2, np2, L);
  return l128.total <= kHeadDynLds && l64.sx_end <= l64.zt && l128.sx_end <= l128.zt;
}

int launch_head_fwd(const HeadFwdArgs& a, hipStream_t s) {
  if (a.R <= 0) return 0;
  SND_CHECK_ARG(head_fwd_supported(a.h1, a.f, a.gh, a.L, a.kp1, a.np1, a.kp2, a.np2),
                "head_fwd: unsupported widths (h1 %d f %d gh %d L %d)", a.h1, a.f, a.gh, a.L);
  SND_CHECK_ARG(a.npad % 128 == 0 && a.npad >= a.npg && (long long)a.npg * a.ngraphs == a.R,
                "head_fwd: npad %% 128, R = ngraphs x npg");
  SND_CHECK_ARG(a.ldg % 8 == 0 && a.ldg >= a.h1 + 8, "head_fwd: ldg");
  SND_CHECK_ARG((long long)a.R * a.h1 * 2 < (1ll << 31), "head_fwd: rows x h1 beyond the 2 GB buffer range");
  SND_CHECK_ARG(a.rowptr && (a.colidx || a.R == 0) && a.xw1 && a.g1 && a.b1 && a.x && a.ge && a.be && a.p1 &&
                    a.g && a.wh_img && a.bh && a.hh && a.wms_img && a.bms && a.ms && a.z && a.eps_out &&
                    a.zb && a.jrow && a.jt && a.colpart && a.kl_part,
                "head_fwd: null operand");
  SND_TRY(head_init_attributes());
  return head_fwd_dispatch<kHeadRows>(a, s);
}

static int head_init_attributes_once() {
  const void* ks[] = {reinterpret_cast<const void*>(head_fwd_kernel<64, 1, 2>),
                      reinterpret_cast<const void*>(head_fwd_kernel<64, 1, 4>),
                      reinterpret_cast<const void*>(head_fwd_kernel<64, 2, 2>),
                      reinterpret_cast<const void*>(head_fwd_kernel<64, 2, 4>)};
  const void* kb[] = {reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 1, 1>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 1, 2>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 1, 3>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 1, 4>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 2, 1>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 2, 2>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 2, 3>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdRows, 1, 2, 4>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 1, 1>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 1, 2>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 1, 3>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 1, 4>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 2, 1>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 2, 2>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 2, 3>),
                      reinterpret_cast<const void*>(head_bwd_kernel<64, 1, 2, 4>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 1, 1>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 1, 2>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 1, 3>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 1, 4>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 2, 1>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 2, 2>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 2, 3>),
                      reinterpret_cast<const void*>(head_bwd_kernel<kHeadBwdTinyRows, 1, 2, 4>)};
  const void* kf[] = {reinterpret_cast<const void*>(enc_front_kernel<1>),
                      reinterpret_cast<const void*>(enc_front_kernel<2>),
                      reinterpret_cast<const void*>(enc_front_kernel<3>),
                      reinterpret_cast<const void*>(enc_front_kernel<4>)};
  for (const void* k : kf) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 6 * 128 * 4) !=
        hipSuccess) {
      set_error("head: hipFuncSetAttribute failed");
      return SND_ERR_HIP;
    }
  }
  for (const void* k : kb) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - kBwdStaticLds) !=
        hipSuccess) {
      set_error("head: hipFuncSetAttribute failed");
      return SND_ERR_HIP;
    }
  }
  for (const void* k : ks) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kHeadDynLds) != hipSuccess) {
      set_error("head: hipFuncSetAttribute failed");
      return SND_ERR_HIP;
    }
  }
  return 0;
}

// once per process, thread-safe (a function-local static's initialiser runs exactly once)
int head_init_attributes() {
  static const int rc = head_init_attributes_once();
  return rc;
}

}  // namespace snd
