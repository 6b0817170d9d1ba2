// Fused bf16 decoder of the train step: two launches instead of seven.
//
//   dec_fwd_kernel  conv1 -> conv2 -> conv3 (k=5 SAME + bias + frozen BN + lrelu,
//                   model_joint.py:112-118,129-140), then the sigmoid heads, their
//                   MSE and the head backward (model_joint.py:121,144;
//                   optimizer.py:149,153)
//   dec_bwd_kernel  conv3^T -> BN/lrelu backward -> conv2^T -> BN/lrelu backward
//                   -> conv1^T = d cost / dJ of the decoders
//
// One workgroup owns a tile of 128 rows of one graph.  A k=5 conv needs two
// halo rows on each side, so a chain of c convs recomputes 2c halo rows per
// side instead of round-tripping every intermediate through HBM: the forward
// stages J rows [r0 - 6, r0 + 134), computes conv1 on [r0 - 4, r0 + 132),
// conv2 on [r0 - 2, r0 + 130) and conv3 on the own rows, each layer's bf16
// output staying in LDS as the next layer's MFMA operand (the [row][k] image
// the row engine of snd_fast.hip reads, 16-byte chunks XOR-swizzled).  Rows
// outside the tile's graph are written as zeros: TF SAME padding per graph.
// Only what the backward pass and the weight gradients need leaves the chip:
// Y1/Y2 (fp32 BN inputs), U1/U2 (bf16 wgrad operands), dY3 / dY2n (bf16).
// The backward chain recomputes its halos the same way (dY3 rows +-6).
//
// The arithmetic is the row engine's (same MFMA order over taps and k chunks,
// same epilogues): every activation and data gradient equals the unfused
// path's bit for bit; only the column partial sums are added in another order.
#include "snd_dec.hpp"

#include <algorithm>

namespace snd {
namespace {

// Workgroups: 16 waves per tile (128-, 64- or 32-row tiles, one workgroup per CU).  With
// J 128 wide (C5) the conv1 / conv1^T weight images (143-164 KB) do not fit the LDS
// whole: the kernels then stream every conv's weights through two one-tap LDS buffers
// (STR, conv_phase_str) on 64-row tiles.  (The same streaming on 8-wave 64-row tiles,
// two workgroups per CU at C2, measured slower than the whole images: DESIGN §6.)
constexpr int DT = 1024;                  // 16 waves
constexpr int NW = DT / 64;
// dynamic LDS of both kernels (their static LDS -- column parameters, head partials -- stays
// below 160 KB - kDynLds)
constexpr int kDynLds = 148 * 1024;

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

__device__ __forceinline__ void dglds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds_base, 16, 0, 0);
}
// chunk swizzle of a [row][kp] bf16 image (snd_fast.hip swz)
__host__ __device__ __forceinline__ int dswz(int row, int kp) {
  return kp == 128 ? (row & 15) : (kp == 64 ? ((row >> 1) & 7) : 0);
}
__host__ __device__ __forceinline__ int lkc_of(int kp) { return kp == 128 ? 4 : (kp == 64 ? 3 : 2); }
__host__ __device__ __forceinline__ int img_bytes(int rows, int kp) {
  return ((rows * kp * 2) + 1023) & ~1023;
}
__host__ __device__ __forceinline__ int rup(int a, int b) { return (a + b - 1) / b * b; }
__host__ __device__ constexpr int head_nq(int cin, int cout) { return cin * cout + cout + 3 * cin; }
// head reduction scratch (aliases the weight image once the convs are done): per head
// [NQ][TR + 1] floats (odd row stride: conflict-free both ways) + TR doubles of squared
// errors per head
__host__ __device__ constexpr int head_scr_bytes(int TR) {
  return (head_nq(10, 2) + head_nq(20, 1)) * (TR + 1) * 4 + 2 * TR * 8;
}

// rows of the input image of a k=5 phase whose output window has n_out rows
__host__ __device__ __forceinline__ int in_rows(int n_out) { return rup(n_out, 16) + 4; }

// ---- LDS layouts (bytes), shared by host (launch size) and device
// (TR: the tile's own rows, kDecRows or kDecRowsSmall)
// bytes of one tap of a packed [tap][np][kp] image (a multiple of 1 KB: np % 16, kp >= 32)
__host__ __device__ __forceinline__ int tap_bytes(const DecImg& im) { return im.np * im.kp * 2; }

// str: the streamed layout -- two one-tap weight buffers instead of the whole image
struct FwdLay {
  int w, a, b, c, total;        // offsets: weights | A: J -> U2 | B: U1 -> U3,Y3 | C: Y2n
  int ldY2n, tapb;              // tapb: one tap buffer (str)
  __host__ __device__ FwdLay(const DecChainFwdArgs& p, int TR, bool str = false) {
    tapb = max(max(tap_bytes(p.k1), tap_bytes(p.k2)), tap_bytes(p.k3));
    const int wimg = str ? 2 * tapb : max(max(p.k1.np * p.k1.kp, p.k2.np * p.k2.kp), p.k3.np * p.k3.kp) * 5 * 2;
    const int wb = max(wimg, (head_scr_bytes(TR) + 1023) & ~1023);
    const int kp_u2 = p.m2.phys() <= 32 ? 32 : (p.m2.phys() <= 64 ? 64 : 128);
    const int ja = img_bytes(in_rows(TR + 8), p.k1.kp);
    const int ua = img_bytes(in_rows(TR), kp_u2);
    const int u1 = img_bytes(in_rows(TR + 4), p.k2.kp);
    const int u3 = 2 * TR * 16 * 4;
    ldY2n = rup(max(p.m2.b, 1), 4);
    w = 0; a = wb; b = a + max(ja, ua); c = b + max(u1, u3);
    total = c + TR * ldY2n * 4;
  }
};
struct BwdLay {
  int w, d3, d2, d1, cps, total, tapb;
  __host__ __device__ BwdLay(const DecChainBwdArgs& p, int TR, bool str = false) {
    tapb = max(max(tap_bytes(p.k3t), tap_bytes(p.k2t)), tap_bytes(p.k1t));
    const int wb = str ? 2 * tapb : max(max(p.k3t.np * p.k3t.kp, p.k2t.np * p.k2t.kp), p.k1t.np * p.k1t.kp) * 5 * 2;
    const int nw = NW;   // the kernels' waves (slots per column group)
    w = 0;
    d3 = wb;
    d2 = d3 + img_bytes(in_rows(TR + 8), p.k3t.kp);
    d1 = d2 + img_bytes(in_rows(TR + 4), p.k2t.kp);
    cps = d1 + img_bytes(in_rows(TR), p.k1t.kp);
    // per-wave column partial slots: (waves / ncg) slots x 3 x np, max over the two BN phases
    const int c1 = (nw / ((p.k2t.np / 16 + 1) / 2)) * 3 * p.k2t.np;
    const int c2 = (nw / (p.k3t.np / 16)) * 3 * p.k3t.np;
    total = cps + max(c1, c2) * 4;
  }
};

// tile -> own rows [r0, rend) of graph [glo, ghi)
struct Tile { int r0, rend, glo, ghi; };
template <int TR>
__device__ __forceinline__ Tile tile_of(int t, int npg) {
  const int tpg = (npg + TR - 1) / TR;
  const int g = t / tpg, lt = t - g * tpg;
  Tile x;
  x.glo = g * npg; x.ghi = x.glo + npg;
  x.r0 = x.glo + lt * TR; x.rend = min(x.r0 + TR, x.ghi);
  return x;
}

// LDS-DMA a bf16 [R][ld] window of rows [wr0, wr0 + nrows) into a [row][kp] image;
// rows outside [glo, ghi) or at/after nvalid, and chunks at col >= K, read zeros.
template <int NWV = NW>
__device__ __forceinline__ void stage_window(const __bf16* src, int ld, int K, int wr0, int nrows,
                                             int nvalid, int glo, int ghi, int kp, char* img,
                                             const void* zero) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lk = lkc_of(kp), kc = 1 << lk;
  const int npc = ((nrows << lk) + 63) >> 6;
  for (int j = w; j < npc; j += NWV) {
    const int q = (j << 6) + lane;
    const int row = q >> lk, pc = q & (kc - 1);
    const int c = pc ^ dswz(row, kp);
    const int gr = wr0 + row;
    const bool v = row < nvalid && gr >= glo && gr < ghi && 8 * c < K;
    const void* g = v ? (const void*)(src + (long long)gr * ld + 8 * c) : zero;
    dglds16(g, img + (j << 10));
  }
}
__device__ __forceinline__ void stage_weights(const DecImg& im, char* dst, int dbg) {
  if (dbg & 1) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int npc = (5 * im.np * im.kp * 2) >> 10;
  const char* g = reinterpret_cast<const char*>(im.w) + lane * 16;
  for (int j = w; j < npc; j += NW) dglds16(g + (j << 10), dst + (j << 10));
}
// The weight DMA of a LATER phase, issued from inline asm: the compiler does not track it,
// so the current phase's ds_reads do not wait for it (with the builtin it drains vmcnt(0)
// before the next LDS read).  The caller owns the wait: wait_dma() before the image is read.
__device__ __forceinline__ void dglds16_async(const void* g, void* lds_base) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lptr_t)lds_base);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
}
__device__ __forceinline__ void stage_weights_async(const DecImg& im, char* dst, int dbg) {
  if (dbg & 1) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int npc = (5 * im.np * im.kp * 2) >> 10;
  const char* g = reinterpret_cast<const char*>(im.w) + lane * 16;
  for (int j = w; j < npc; j += NW) dglds16_async(g + (j << 10), dst + (j << 10));
}
// tap t of a packed image into a one-tap buffer (STR; untracked DMA, as above)
template <int NWV>
__device__ __forceinline__ void stage_tap_async(const DecImg& im, int t, char* dst, int dbg) {
  if (dbg & 1) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int npc = tap_bytes(im) >> 10;
  const char* g = reinterpret_cast<const char*>(im.w) + (long long)t * tap_bytes(im) + lane * 16;
  for (int j = w; j < npc; j += NWV) dglds16_async(g + (j << 10), dst + (j << 10));
}
__host__ __device__ __forceinline__ int wimg_bytes(const DecImg& im) { return 5 * im.np * im.kp * 2; }
__device__ __forceinline__ void wait_dma() {
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  __syncthreads();
}

// 4 bf16 of row `row`, columns n0 .. n0 + 3 (n0 % 4 == 0) of a [row][kp] image
__device__ __forceinline__ __bf16* img_at(__bf16* img, int row, int kp, int n0) {
  return img + row * kp + ((((n0 >> 3) ^ dswz(row, kp)) << 3) | (n0 & 4));
}

// One k=5 phase: out^T = W^T x^T on v_mfma_f32_16x16x32_bf16 (the row engine's
// operand roles and order).  Output window rows o in [0, n_out) read image rows
// o .. o + 4.  Waves are assigned column group cg = w % ncg and row blocks
// k, k + wpc, ... (k = w / ncg); PRE(orow, nb0, yp) loads epilogue operands before
// the MFMAs, EPI(orow, nb0, acc, yp) consumes a finished 16-row x NBH-block item.
// KCS = kpw / 32 k-chunks per tap as a compile-time count: the tap x chunk loop
// unrolls whole, so the operand reads of later chunks are issued ahead of the
// MFMAs of earlier ones (a runtime count left one LDS round trip per chunk exposed)
template <int NBH, int KCS, class Pre, class Epi>
__device__ __forceinline__ void conv_phase_t(const __bf16* xs, int kpx, const __bf16* ws, int kpw, int np,
                                             int n_out, Pre&& pre, Epi&& epi, int dbg) {
  // the wave index through readfirstlane: the row-block loop and the column-block choice
  // are then scalar, and the MFMAs straight-line code (a per-lane view of w made every
  // MFMA an exec-masked branch with its operand read right before it)
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int nrb = (n_out + 15) >> 4, nbc = np >> 4;
  const int ncg = (nbc + NBH - 1) / NBH, wpc = NW / ncg;
  const int cg = w % ncg, k0 = w / ncg;
  if (k0 >= wpc) return;
  const int nb0 = cg * NBH;
  // callers pass the RUNTIME bits (a.dbg, not kdbg(a.dbg)): the scalar branch around the
  // MFMA block bounds the scheduling region.  With the bit folded to a constant the
  // compiler hoisted the epilogue operands over the MFMAs and dec_bwd_kernel spilled
  // 72 VGPRs (22.6 -> 49.1 us, the round-4 C2 regression; tools/gpu_bisect.sh)
  const bool mm = !(dbg & 4);
  const int kcs = KCS ? KCS : kpw >> 5;
  const int wsw = dswz(li, kpw);
  // a column group's blocks past the image (np not a multiple of 16 NBH) repeat its last
  // block: the MFMA runs unconditionally and the epilogue drops the columns >= np
  int wb[NBH];
#pragma unroll
  for (int i = 0; i < NBH; ++i) wb[i] = 16 * min(nb0 + i, nbc - 1) * kpw;
  // the epilogue operands of a wave's NEXT row block are loaded before this block's MFMAs
  // (round 5: one HBM round trip per row-block pass was exposed in the backward phases)
  f32x4 ypn[NBH];
  if (k0 < nrb) pre(16 * k0 + li, nb0, ypn);
  for (int rb = k0; rb < nrb; rb += wpc) {
    f32x4 yp[NBH];
#pragma unroll
    for (int i = 0; i < NBH; ++i) yp[i] = ypn[i];
    if (rb + wpc < nrb) pre(16 * (rb + wpc) + li, nb0, ypn);
    f32x4 acc[NBH];
#pragma unroll
    for (int i = 0; i < NBH; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (mm) {
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        const int xrow = 16 * rb + li + t;
        const __bf16* xrp = xs + xrow * kpx;
        const int xsw = dswz(xrow, kpx);
        const __bf16* wrp = ws + (t * np + li) * kpw;
        auto chunk = [&](int ks) {
          const int ch = 4 * ks + lg;
          const bf16x8 bx = *reinterpret_cast<const bf16x8*>(xrp + ((ch ^ xsw) << 3));
#pragma unroll
          for (int i = 0; i < NBH; ++i) {
            const bf16x8 aw = *reinterpret_cast<const bf16x8*>(wrp + wb[i] + ((ch ^ wsw) << 3));
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, bx, acc[i], 0, 0, 0);
          }
        };
        if constexpr (KCS == 0) {
          for (int ks = 0; ks < kcs; ++ks) chunk(ks);
        } else {
#pragma unroll
          for (int ks = 0; ks < KCS; ++ks) chunk(ks);
        }
      }
    }
    epi(16 * rb + li, nb0, acc, yp);
  }
}
// KX: the chunk count the call site expects (the C2 decoder widths); the phase runs
// the unrolled instantiation when kpw / 32 == KX and the runtime loop otherwise (KX 0:
// always the runtime loop).  One unrolled instantiation per call site keeps the
// backward chain within 128 VGPRs.
template <int NBH, int KX, class Pre, class Epi>
__device__ __forceinline__ void conv_phase(const __bf16* xs, int kpx, const __bf16* ws, int kpw, int np,
                                           int n_out, Pre&& pre, Epi&& epi, int dbg = 0) {
  if (KX > 0 && kpw == 32 * KX) conv_phase_t<NBH, KX>(xs, kpx, ws, kpw, np, n_out, pre, epi, dbg);
  else conv_phase_t<NBH, 0>(xs, kpx, ws, kpw, np, n_out, pre, epi, dbg);
}

// The same phase with streamed weights (STR): the weights arrive one tap at a time through two LDS
// buffers (the kernel's taps form one sequence, tap g in buffer g & 1; g0 = this phase's
// first).  Tap t opens with vmcnt(0) + barrier (tap t is in, every wave has finished tap
// t - 1), then DMAs the sequence's next tap -- tap t + 1, or the next phase's tap 0 --
// into the buffer tap t - 1 used, and runs tap t over ALL the wave's row blocks (their
// accumulators live across the taps).  Per output the MFMA order is conv_phase_t's (taps
// outer, k chunks inner): bitwise the same sums.  Every wave reaches every barrier.
// MAXRB: the most row blocks a wave owns (checked on the host, dec_fused_supported); KCS: the
// k chunks per tap the call site expects (unrolled when kp == 32 KCS, a runtime loop else).
template <int NBH, int KCS, int NWV, int MAXRB, class Pre, class Epi>
__device__ __forceinline__ void conv_phase_str(const __bf16* xs, int kpx, const DecImg& im, char* wb0, char* wb1,
                                               int g0, const DecImg* next, int n_out, Pre&& pre, Epi&& epi,
                                               int dbg) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, lg = lane >> 4;
  const int kpw = im.kp, np = im.np;
  const int nrb = (n_out + 15) >> 4, nbc = np >> 4;
  const int ncg = (nbc + NBH - 1) / NBH, wpc = NWV / ncg;
  const int cg = w % ncg, k0 = w / ncg;
  const bool act = k0 < wpc;
  const int nb0 = cg * NBH;
  const bool mm = !(dbg & 4);
  const int wsw = dswz(li, kpw);
  int wb[NBH];
#pragma unroll
  for (int i = 0; i < NBH; ++i) wb[i] = 16 * min(nb0 + i, nbc - 1) * kpw;
  f32x4 acc[MAXRB][NBH], yp[MAXRB][NBH];
#pragma unroll
  for (int j = 0; j < MAXRB; ++j)
#pragma unroll
    for (int i = 0; i < NBH; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): tap t has landed
    __syncthreads();
    if (t < 4) stage_tap_async<NWV>(im, t + 1, ((g0 + t + 1) & 1) ? wb1 : wb0, dbg);
    else if (next) stage_tap_async<NWV>(*next, 0, ((g0 + 5) & 1) ? wb1 : wb0, dbg);
    if (t == 0 && act) {   // epilogue operands: in flight under the taps
#pragma unroll
      for (int j = 0; j < MAXRB; ++j)
        if (k0 + j * wpc < nrb) pre(16 * (k0 + j * wpc) + li, nb0, yp[j]);
    }
    if (act && mm) {
      const __bf16* wrp = reinterpret_cast<const __bf16*>(((g0 + t) & 1) ? wb1 : wb0) + li * kpw;
#pragma unroll
      for (int j = 0; j < MAXRB; ++j) {
        const int rb = k0 + j * wpc;
        if (rb >= nrb) break;
        const int xrow = 16 * rb + li + t;
        const __bf16* xrp = xs + xrow * kpx;
        const int xsw = dswz(xrow, kpx);
        auto chunk = [&](int ks) {
          const int ch = 4 * ks + lg;
          const bf16x8 bx = *reinterpret_cast<const bf16x8*>(xrp + ((ch ^ xsw) << 3));
#pragma unroll
          for (int i = 0; i < NBH; ++i) {
            const bf16x8 aw = *reinterpret_cast<const bf16x8*>(wrp + wb[i] + ((ch ^ wsw) << 3));
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, bx, acc[j][i], 0, 0, 0);
          }
        };
        if (KCS > 0 && kpw == 32 * KCS) {   // the call site's expected width: unrolled
#pragma unroll
          for (int ks = 0; ks < KCS; ++ks) chunk(ks);
        } else {
          for (int ks = 0; ks < (kpw >> 5); ++ks) chunk(ks);
        }
      }
    }
  }
  if (!act) return;
#pragma unroll
  for (int j = 0; j < MAXRB; ++j) {
    const int rb = k0 + j * wpc;
    if (rb >= nrb) break;
    epi(16 * rb + li, nb0, acc[j], yp[j]);
  }
}

// per-column parameters of a (possibly split) layout, physical column n
__device__ __forceinline__ float colpar(const ColMap& m, int n, const float* A, const float* Bv) {
  if (!m.valid(n) || !A) return 0.f;
  if (n < m.a || !Bv) return A[n < m.a ? n : m.logical(n)];
  return Bv[n - m.offb];
}

// ------------------------------------------------------------------ heads
// One thread per own row (model_joint.py:121,144; optimizer.py:149,153): as
// heads_fast_kernel's head_rows, with the inputs read from LDS.  Partial sums
// {dW, db, sum dt*y, sum dt, sum dy} reduced over the tile in fixed order.
template <int CIN, int COUT, int SCR>
__device__ __forceinline__ void head_tile(int hi, int orow, bool rv, long long gr, const float (&u)[CIN],
                                          const float (&yv)[CIN], const float* hp, const float (&tg)[COUT],
                                          float count, float* yhat, __bf16* dyp, float* scr,
                                          double* sscr) {
  // hp (LDS, loaded at kernel start): W [CIN][COUT] | b [COUT] at 20 | gamma at 24 | beta at 24 + CIN
  float wv[CIN][COUT], bv[COUT], gk[CIN], bk[CIN];
#pragma unroll
  for (int k = 0; k < CIN; ++k) {
#pragma unroll
    for (int o = 0; o < COUT; ++o) wv[k][o] = hp[k * COUT + o];
    gk[k] = hp[24 + k] * kBnC;
    bk[k] = hp[24 + CIN + k];
  }
#pragma unroll
  for (int o = 0; o < COUT; ++o) bv[o] = hp[20 + o];
  float dp[COUT];
  double sse = 0.0;
#pragma unroll
  for (int o = 0; o < COUT; ++o) {
    float zo = bv[o];
#pragma unroll
    for (int k = 0; k < CIN; ++k) zo += u[k] * wv[k][o];
    const float yh = 1.f / (1.f + __expf(-zo));
    const float diff = yh - tg[o];
    if (rv) {
      if (yhat) yhat[gr * COUT + o] = yh;
      sse += (double)diff * diff;
    }
    dp[o] = rv ? 2.f * diff / count * yh * (1.f - yh) : 0.f;
  }
  float dt[CIN], dyv[CIN];
#pragma unroll
  for (int k = 0; k < CIN; ++k) {
    float du = 0.f;
#pragma unroll
    for (int o = 0; o < COUT; ++o) du += dp[o] * wv[k][o];
    dt[k] = du * lrelu_grad(yv[k] * gk[k] + bk[k]);
    dyv[k] = dt[k] * gk[k];
  }
  if (rv) {
#pragma unroll
    for (int c = 0; c < CIN / 4; ++c) {
      bf16x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (__bf16)dyv[4 * c + j];
      *reinterpret_cast<bf16x4*>(dyp + 4 * c) = v;
    }
#pragma unroll
    for (int k = (CIN / 4) * 4; k < CIN; ++k) dyp[k] = (__bf16)dyv[k];
  }
  // per-row quantities {dW, db, sum dt*y, sum dt, sum dy} and the squared error into
  // q-major scratch (odd row stride SCR: conflict-free both ways); the caller sums rows
  float* sc = scr + orow;
#pragma unroll
  for (int k = 0; k < CIN; ++k)
#pragma unroll
    for (int o = 0; o < COUT; ++o) sc[(k * COUT + o) * SCR] = u[k] * dp[o];
#pragma unroll
  for (int o = 0; o < COUT; ++o) sc[(CIN * COUT + o) * SCR] = dp[o];
  constexpr int QB = CIN * COUT + COUT;
#pragma unroll
  for (int k = 0; k < CIN; ++k) {
    sc[(QB + k) * SCR] = dt[k] * yv[k];
    sc[(QB + CIN + k) * SCR] = dt[k];
    sc[(QB + 2 * CIN + k) * SCR] = dyv[k];
  }
  sscr[orow] = sse;
  (void)hi; (void)gr;
}

// ------------------------------------------------------------------ forward
// NWV waves per workgroup (<= 128 VGPRs at 4 waves per SIMD); STR: weights streamed by tap
template <int TR, int NWV = NW, bool STR = false>
__global__ void __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(4, 4)))
dec_fwd_kernel(DecChainFwdArgs a) {
  constexpr int DTK = 64 * NWV;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ __attribute__((aligned(16))) float cp1[3][128], cp2[3][128], cp3[3][16];
  __shared__ float hp[2][64];   // head parameters (head_tile layout)
  const FwdLay L(a, TR, STR);
  const Tile tl = tile_of<TR>(blockIdx.x, a.npg);
  const int tid = threadIdx.x, lane = tid & 63, lg = lane >> 4;
  __bf16* wimg = reinterpret_cast<__bf16*>(smem + L.w);
  __bf16* jimg = reinterpret_cast<__bf16*>(smem + L.a);
  __bf16* u2img = jimg;                                   // A: J, then U2
  __bf16* u1img = reinterpret_cast<__bf16*>(smem + L.b);
  float* u3 = reinterpret_cast<float*>(smem + L.b);       // B: U1, then U3 | Y3
  float* y3 = u3 + TR * 16;
  float* y2n = reinterpret_cast<float*>(smem + L.c);
  const int kpu2 = a.m2.phys() <= 32 ? 32 : (a.m2.phys() <= 64 ? 64 : 128);
  const int own = tl.rend - tl.r0;
  // measurement only (debug bit 1 << 21): s_memrealtime at the phase boundaries, written by
  // thread 0 over the tile's head partials at the end (results wrong); tools/dec_stamps.py
  const bool stamp = kdbg(a.dbg) & (1 << 21);
  unsigned long long ts[9] = {};
  if (stamp) ts[0] = __builtin_amdgcn_s_memrealtime();

  // Zero what an MFMA reads against zero weights but nobody writes: the U1 image's
  // pad columns [k1.np, k2.kp) (conv2's last k-chunk; uninitialised LDS may hold NaN,
  // and NaN * 0 is NaN).  Everything else a valid output reads is written first: the
  // J window by its DMA (zeros outside the graph), U1 / U2 / U3 / Y3 / Y2n by the
  // epilogues; rows past a window only feed discarded output rows, and U2's pad
  // columns hold finite stale J values against zero weights.  (Zeroing the whole
  // 148 KB measured 1.6 us of the launch.)
  if (kdbg(a.dbg) & (1 << 23)) {   // test only: NaN in every activation byte first (worst-case stale LDS)
    for (int i = tid * 16; i < L.total - L.a; i += DTK * 16)
      *reinterpret_cast<uint4*>(smem + L.a + i) = make_uint4(~0u, ~0u, ~0u, ~0u);
    __syncthreads();
  }
  if (!(kdbg(a.dbg) & 32)) {   // (kp - np) / 4 <= 4 groups of 4 columns per row: no division
    const int kpo = a.k2.kp, npc = (kpo - a.k1.np) >> 2, nr = in_rows(TR + 4);
    for (int i = tid; i < nr * 4; i += DTK) {
      const int row = i >> 2, q = i & 3;
      if (q < npc) *reinterpret_cast<bf16x4*>(img_at(u1img, row, kpo, a.k1.np + 4 * q)) = bf16x4{};
    }
  }
  __syncthreads();
  // J window [r0 - 6, r0 + own + 6) and the conv1 weights
  if (!(kdbg(a.dbg) & 16))
    stage_window<NWV>(a.zb, a.ldz, a.dj, tl.r0 - 6, in_rows(TR + 8), own + 12, tl.glo, tl.ghi, a.k1.kp,
                      reinterpret_cast<char*>(jimg), a.zero);
  // tap buffers of the dual tiles (the weight region, two halves)
  char* tb0 = reinterpret_cast<char*>(wimg);
  char* tb1 = tb0 + L.tapb;
  if constexpr (STR) stage_tap_async<NWV>(a.k1, 0, tb0, kdbg(a.dbg));
  else stage_weights(a.k1, reinterpret_cast<char*>(wimg), kdbg(a.dbg));
  // head parameters and the tile's targets, fetched now so their latency hides under the convs
  constexpr int HPT = DTK == 1024 ? 512 : DTK - 128;   // threads [HPT, HPT + 128)
  static_assert(DTK - 128 >= 2 * TR || DTK == 1024, "dec_fwd: head parameter threads overlap the targets'");
  if (tid >= HPT && tid < HPT + 128) {
    const int i = tid - HPT, hh = i >> 6, j = i & 63;
    const int cin = hh ? 20 : 10, cout = hh ? 1 : 2;
    const float* w = hh ? a.wn : a.ws;
    const float* b = hh ? a.bn : a.bs;
    const float* g = hh ? a.g2n : a.g3;
    const float* be = hh ? a.be2n : a.be3;
    float v = 0.f;
    if (j < cin * cout) v = w[j];
    else if (j >= 20 && j < 20 + cout) v = b[j - 20];
    else if (j >= 24 && j < 24 + cin) v = g[j - 24];
    else if (j >= 24 + cin && j < 24 + 2 * cin) v = be[j - 24 - cin];
    hp[hh][j] = v;
  }
  float tg[2] = {0.f, 0.f};
  if (tid < 2 * TR) {
    const int orow = tid % TR;
    const long long gr = tl.r0 + orow;
    if (orow < own) {
      if (tid < TR) { tg[0] = a.s_truth[gr * 2]; tg[1] = a.s_truth[gr * 2 + 1]; }
      else tg[0] = a.x_truth[gr];
    }
  }
  if (tid < 128) {
    const int n = tid;
    cp1[0][n] = colpar(a.m1, n, a.b1, nullptr);
    cp1[1][n] = colpar(a.m1, n, a.g1, nullptr) * kBnC;
    cp1[2][n] = colpar(a.m1, n, a.be1, nullptr);
    cp2[0][n] = colpar(a.m2, n, a.b2s, a.b2n);
    cp2[1][n] = colpar(a.m2, n, a.g2s, a.g2n) * kBnC;
    cp2[2][n] = colpar(a.m2, n, a.be2s, a.be2n);
    if (n < 16) {
      const ColMap m3{a.s3, 0, a.s3};
      cp3[0][n] = colpar(m3, n, a.b3, nullptr);
      cp3[1][n] = colpar(m3, n, a.g3, nullptr) * kBnC;
      cp3[2][n] = colpar(m3, n, a.be3, nullptr);
    }
  }
  wait_dma();
  if (stamp) ts[1] = __builtin_amdgcn_s_memrealtime();

  auto nopre = [](int, int, auto&) {};
  // ---- conv1: window [r0 - 4, r0 + own + 4) -> U1 image (bf16), Y1 / U1 own rows to HBM
  {
    // Columns outside the split layout (the [s | n] gap, the pad to np) need no mask:
    // their packed weights and column parameters are zero, so y = +0 and lrelu(BN(y)) = +0
    // there, which is what the zero-filled Y1 / U1 pads and the image already hold; every
    // column group is a whole float4 inside np = ld1.  Only rows outside the graph (TF
    // SAME padding) are zeroed.
    const int wr0 = tl.r0 - 4, n_out = own + 8, kpo = a.k2.kp, nbc = a.k1.np >> 4;
    auto epi1 = [&](int orow, int nb0, f32x4 (&acc)[2], f32x4 (&)[2]) {
      if (orow >= n_out) return;
      const int gr = wr0 + orow;
      const bool ing = gr >= tl.glo && gr < tl.ghi, mine = gr >= tl.r0 && gr < tl.rend;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (nb0 + i >= nbc) continue;
        const int n0 = 16 * (nb0 + i) + 4 * lg;
        const f32x4 b = *reinterpret_cast<const f32x4*>(&cp1[0][n0]);
        const f32x4 g = *reinterpret_cast<const f32x4*>(&cp1[1][n0]);
        const f32x4 be = *reinterpret_cast<const f32x4*>(&cp1[2][n0]);
        f32x4 yv;
        bf16x4 ub;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          yv[e] = acc[i][e] + b[e];
          ub[e] = (__bf16)(ing ? lrelu(yv[e] * g[e] + be[e]) : 0.f);
        }
        *reinterpret_cast<bf16x4*>(img_at(u1img, orow, kpo, n0)) = ub;
        if (mine && !(kdbg(a.dbg) & 8)) {
          *reinterpret_cast<f32x4*>(a.y1 + (long long)gr * a.ldy1 + n0) = yv;
          *reinterpret_cast<bf16x4*>(a.u1 + (long long)gr * a.ldy1 + n0) = ub;
        }
      }
    };
    if constexpr (STR) conv_phase_str<2, 2, NWV, 3>(jimg, a.k1.kp, a.k1, tb0, tb1, 0, &a.k2, n_out, nopre, epi1, a.dbg);
    else conv_phase<2, 2>(jimg, a.k1.kp, wimg, a.k1.kp, a.k1.np, n_out, nopre, epi1, a.dbg);
  }
  __syncthreads();
  if (stamp) ts[2] = __builtin_amdgcn_s_memrealtime();
  // conv3's image at the tail of the weight region when it fits beside conv2's: its DMA
  // runs under conv2 (round 5; the dual tiles stream every tap instead)
  const int k3o = (L.a - L.w) - wimg_bytes(a.k3);
  const bool pre3 = !STR && wimg_bytes(a.k2) <= k3o && (k3o & 1023) == 0;
  __bf16* wimg3 = pre3 ? wimg + k3o / 2 : wimg;
  if constexpr (!STR) {
    stage_weights(a.k2, reinterpret_cast<char*>(wimg), kdbg(a.dbg));
    wait_dma();
    if (pre3) stage_weights_async(a.k3, reinterpret_cast<char*>(wimg3), kdbg(a.dbg));
  }
  if (stamp) ts[3] = __builtin_amdgcn_s_memrealtime();
  // ---- conv2: window [r0 - 2, r0 + own + 2) -> U2 image; Y2 / U2 own rows; Y2n own rows in LDS
  {
    // as conv1: no column masks (zero weights and parameters outside the layout)
    const int wr0 = tl.r0 - 2, n_out = own + 4, nbc = a.k2.np >> 4;
    const int nlo = a.m2.b ? a.m2.offb : 1 << 30, nhi = a.m2.offb + a.m2.b;
    auto epi2 = [&](int orow, int nb0, f32x4 (&acc)[2], f32x4 (&)[2]) {
      if (orow >= n_out) return;
      const int gr = wr0 + orow;
      const bool ing = gr >= tl.glo && gr < tl.ghi, mine = gr >= tl.r0 && gr < tl.rend;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (nb0 + i >= nbc) continue;
        const int n0 = 16 * (nb0 + i) + 4 * lg;
        const f32x4 b = *reinterpret_cast<const f32x4*>(&cp2[0][n0]);
        const f32x4 g = *reinterpret_cast<const f32x4*>(&cp2[1][n0]);
        const f32x4 be = *reinterpret_cast<const f32x4*>(&cp2[2][n0]);
        f32x4 yv;
        bf16x4 ub;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          yv[e] = acc[i][e] + b[e];
          ub[e] = (__bf16)(ing ? lrelu(yv[e] * g[e] + be[e]) : 0.f);
        }
        *reinterpret_cast<bf16x4*>(img_at(u2img, orow, kpu2, n0)) = ub;
        if (mine && !(kdbg(a.dbg) & 8)) {
          *reinterpret_cast<f32x4*>(a.y2 + (long long)gr * a.ldy2 + n0) = yv;
          *reinterpret_cast<bf16x4*>(a.u2 + (long long)gr * a.ldy2 + n0) = ub;
          if (n0 >= nlo && n0 < nhi)   // the n branch's columns: whole float4 groups (b % 4 == 0)
            *reinterpret_cast<f32x4*>(&y2n[(gr - tl.r0) * L.ldY2n + (n0 - a.m2.offb)]) = yv;
        }
      }
    };
    if constexpr (STR) conv_phase_str<2, 4, NWV, 2>(u1img, a.k2.kp, a.k2, tb0, tb1, 5, &a.k3, n_out, nopre, epi2, a.dbg);
    else conv_phase<2, 4>(u1img, a.k2.kp, wimg, a.k2.kp, a.k2.np, n_out, nopre, epi2, a.dbg);
  }
  __syncthreads();
  if (stamp) ts[4] = __builtin_amdgcn_s_memrealtime();
  if constexpr (!STR) {
    if (!pre3) stage_weights(a.k3, reinterpret_cast<char*>(wimg3), kdbg(a.dbg));
    wait_dma();
  }
  if (stamp) ts[5] = __builtin_amdgcn_s_memrealtime();
  // ---- conv3 (s branch): own rows -> U3, Y3 (fp32, LDS; the spatial head's input)
  {
    const int n_out = own;
    auto epi3 = [&](int orow, int nb0, f32x4 (&acc)[1], f32x4 (&)[1]) {
      if (orow >= n_out) return;
      const int n0 = 16 * nb0 + 4 * lg;
      float yv[4], o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {   // columns >= s3: zero weights and parameters, y = o = +0
        const int n = n0 + e;
        yv[e] = acc[0][e] + cp3[0][n];
        o[e] = lrelu(yv[e] * cp3[1][n] + cp3[2][n]);
      }
      *reinterpret_cast<float4*>(u3 + orow * 16 + n0) = make_float4(o[0], o[1], o[2], o[3]);
      *reinterpret_cast<float4*>(y3 + orow * 16 + n0) = make_float4(yv[0], yv[1], yv[2], yv[3]);
    };
    if constexpr (STR) conv_phase_str<1, 2, NWV, 1>(u2img, kpu2, a.k3, tb0, tb1, 10, nullptr, n_out, nopre, epi3, a.dbg);
    else conv_phase<1, 2>(u2img, kpu2, wimg3, a.k3.kp, a.k3.np, n_out, nopre, epi3, a.dbg);
  }
  __syncthreads();
  if (stamp) ts[6] = __builtin_amdgcn_s_memrealtime();
  // ---- heads: spatial (s3 -> sd) on threads [0, TR), node (n2 -> nf) on [TR, 2 TR); the
  // per-row partial quantities go to scratch over the (now idle) weight image
  const int t = blockIdx.x;
  constexpr int NQS = head_nq(10, 2), NQN = head_nq(20, 1);
  float* scr = reinterpret_cast<float*>(smem + L.w);
  constexpr int SCR = TR + 1;   // scratch row stride (words)
  double* sscr = reinterpret_cast<double*>(smem + L.w + (NQS + NQN) * SCR * 4);
  if (!(kdbg(a.dbg) & 2)) {
    if (tid < 2 * TR) {
      const int hi = tid / TR, orow = tid % TR;
      const bool rv = orow < own;
      const long long gr = tl.r0 + orow;
      if (hi == 0) {
        float u[10], yv[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) { u[k] = rv ? u3[orow * 16 + k] : 0.f; yv[k] = rv ? y3[orow * 16 + k] : 0.f; }
        const float t2[2] = {tg[0], tg[1]};
        head_tile<10, 2, SCR>(0, orow, rv, gr, u, yv, hp[0], t2, a.cnt_s, a.shat, a.dy3 + gr * a.lddy3, scr, sscr);
      } else {
        float u[20], yv[20];
#pragma unroll
        for (int k = 0; k < 20; ++k) {   // U2n: window row orow + 2 of the U2 image (bf16)
          const int n = a.m2.offb + k;
          u[k] = rv ? (float)img_at(u2img, orow + 2, kpu2, n & ~3)[n & 3] : 0.f;
          yv[k] = rv ? y2n[orow * L.ldY2n + k] : 0.f;
        }
        const float t1[1] = {tg[0]};
        head_tile<20, 1, SCR>(1, orow, rv, gr, u, yv, hp[1], t1, a.cnt_n, a.xhat, a.dy2 + gr * a.lddy2 + a.m2.offb,
                              scr + NQS * SCR, sscr + TR);
      }
    }
    __syncthreads();
    if (stamp) ts[7] = __builtin_amdgcn_s_memrealtime();
    // tile partials: each quantity summed over the TR rows in order
    if (tid < NQS + NQN) {
      const float* src = scr + tid * SCR;
      float v = 0.f;
#pragma unroll 32
      for (int r = 0; r < TR; ++r) v += src[r];
      if (tid < NQS) a.phs[(long long)t * NQS + tid] = v;
      else a.phn[(long long)t * NQN + tid - NQS] = v;
    } else if (tid >= 256 && tid < 258) {
      const double* src = sscr + TR * (tid - 256);
      double v = 0.0;
#pragma unroll 32
      for (int r = 0; r < TR; ++r) v += src[r];
      (tid == 256 ? a.sse_s : a.sse_n)[t] = v;
    }
  }
  if (stamp) {
    __syncthreads();
    if (tid == 0) {
      ts[8] = __builtin_amdgcn_s_memrealtime();
      unsigned* o = reinterpret_cast<unsigned*>(a.phs + (long long)t * NQS);
      for (int k = 0; k < 9; ++k) o[k] = (unsigned)ts[k];
    }
  }
}

// ------------------------------------------------------------------ backward
template <int NBH>
__device__ __forceinline__ void colpart_flush(float (&q)[3][NBH][4], float* slots, int np, int nb0, int nbc,
                                              int slot) {
  const int lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int i = 0; i < NBH; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = row16_sum(q[k][i][e]);
        const int n = 16 * (nb0 + i) + 4 * lg + e;
        if (li == 0 && nb0 + i < nbc) slots[(slot * 3 + k) * np + n] = v;
      }
}

template <int TR, int NWV = NW, bool STR = false>
__global__ void __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(4, 4)))
dec_bwd_kernel(DecChainBwdArgs a) {
  constexpr int DTK = 64 * NWV;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ __attribute__((aligned(16))) float cpa[2][128], cpb[2][128];   // conv2-s BN (gamma c, beta), conv1 BN
  const BwdLay L(a, TR, STR);
  const Tile tl = tile_of<TR>(blockIdx.x, a.npg);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, lg = lane >> 4;
  __bf16* wimg = reinterpret_cast<__bf16*>(smem + L.w);
  __bf16* d3 = reinterpret_cast<__bf16*>(smem + L.d3);
  __bf16* d2 = reinterpret_cast<__bf16*>(smem + L.d2);
  __bf16* d1 = reinterpret_cast<__bf16*>(smem + L.d1);
  float* slots = reinterpret_cast<float*>(smem + L.cps);
  const int own = tl.rend - tl.r0;
  const int t = blockIdx.x;
  const bool stamp = kdbg(a.dbg) & (1 << 21);   // measurement only, as dec_fwd_kernel (over pc1)
  unsigned long long ts[8] = {};
  if (stamp) ts[0] = __builtin_amdgcn_s_memrealtime();

  if (!(kdbg(a.dbg) & 32))
    for (int i = tid * 16; i < L.cps - L.d3; i += DTK * 16)
      *reinterpret_cast<uint4*>(smem + L.d3 + i) = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  // dY3 window [r0 - 6, r0 + own + 6), conv3^T weights
  if (!(kdbg(a.dbg) & 16))
    stage_window<NWV>(a.dy3, a.lddy3, a.s3, tl.r0 - 6, in_rows(TR + 8), own + 12, tl.glo, tl.ghi, a.k3t.kp,
                      reinterpret_cast<char*>(d3), a.zero);
  // conv3^T's image at the tail of the weight region when conv2^T's fits beside it: conv2^T's
  // DMA then runs under conv3^T (round 5; "W2t staged" was 0.9 us of a 20.5 us chain; the
  // dual tiles stream every tap instead)
  const int wb3 = L.d3 - L.w, k3o = wb3 - wimg_bytes(a.k3t);
  const bool pre2 = !STR && wimg_bytes(a.k2t) <= k3o && (k3o & 1023) == 0;
  __bf16* wimg3 = pre2 ? wimg + k3o / 2 : wimg;
  char* tb0 = reinterpret_cast<char*>(wimg);
  char* tb1 = tb0 + L.tapb;
  if constexpr (STR) stage_tap_async<NWV>(a.k3t, 0, tb0, kdbg(a.dbg));
  else stage_weights(a.k3t, reinterpret_cast<char*>(wimg3), kdbg(a.dbg));
  if (tid < 128) {
    const int n = tid;
    const ColMap ms{a.m2.a, 0, a.m2.a};
    cpa[0][n] = colpar(ms, n, a.g2s, nullptr) * kBnC;
    cpa[1][n] = colpar(ms, n, a.be2s, nullptr);
    cpb[0][n] = colpar(a.m1, n, a.g1, nullptr) * kBnC;
    cpb[1][n] = colpar(a.m1, n, a.be1, nullptr);
  }
  // dY2 n part of the window [r0 - 4, r0 + own + 4) (the heads' output) into the dY2 image
  {
    const int wr0 = tl.r0 - 4, nv = own + 8, kp2 = a.k2t.kp;
    const int nq = (a.m2.b + 3) / 4;             // 4-column groups of the n part
    for (int i = tid; i < ((kdbg(a.dbg) & 16) ? 0 : nv * nq); i += DTK) {
      const int row = i / nq, q = i - row * nq;
      const int gr = wr0 + row;
      if (gr < tl.glo || gr >= tl.ghi) continue;
      const int n0 = a.m2.offb + 4 * q;
      const bf16x4 v = *reinterpret_cast<const bf16x4*>(a.dy2 + (long long)gr * a.lddy2 + n0);
      *reinterpret_cast<bf16x4*>(img_at(d2, row, kp2, n0)) = v;
    }
  }
  wait_dma();
  if (!STR && pre2) stage_weights_async(a.k2t, reinterpret_cast<char*>(wimg), kdbg(a.dbg));
  if (stamp) ts[1] = __builtin_amdgcn_s_memrealtime();
  // ---- conv3^T: window [r0 - 4, r0 + own + 4): dU2s -> BN/lrelu backward -> dY2s
  {
    const int wr0 = tl.r0 - 4, n_out = own + 8, N = a.m2.a, kpo = a.k2t.kp;
    const int nbc = a.k3t.np >> 4, ncg = nbc, wpc = NWV / ncg;
    const int nb0 = w % ncg;
    float q[3][1][4] = {};
    auto pre3t = [&](int orow, int nb, f32x4 (&yp)[1]) {
                    yp[0] = f32x4{0.f, 0.f, 0.f, 0.f};
                    const int gr = wr0 + orow;
                    if (orow < n_out && gr >= tl.glo && gr < tl.ghi) {
                      const int n0 = 16 * nb + 4 * lg;
                      const float* p = a.y2 + (long long)gr * a.ldy2 + n0;
#pragma unroll
                      for (int e = 0; e < 4; ++e) if (n0 + e < N) yp[0][e] = p[e];
                    }
                  };
    auto epi3t = [&](int orow, int nb, f32x4 (&acc)[1], f32x4 (&yp)[1]) {
      if (orow >= n_out) return;
      const int gr = wr0 + orow;
      const bool ing = gr >= tl.glo && gr < tl.ghi, mine = gr >= tl.r0 && gr < tl.rend;
      const int n0 = 16 * nb + 4 * lg;
      // columns >= N: zero weights, gamma and beta, so dt = +0 there without a mask
      const f32x4 ga = *reinterpret_cast<const f32x4*>(&cpa[0][n0]);
      const f32x4 be = *reinterpret_cast<const f32x4*>(&cpa[1][n0]);
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dt = ing ? acc[0][e] * lrelu_grad(yp[0][e] * ga[e] + be[e]) : 0.f;
        o[e] = dt * ga[e];
        if (mine) { q[0][0][e] += dt * yp[0][e]; q[1][0][e] += dt; q[2][0][e] += o[e]; }
      }
      bf16x4 ob;
#pragma unroll
      for (int e = 0; e < 4; ++e) ob[e] = (__bf16)o[e];
      if (n0 < a.m2.offb || !a.m2.b)    // s part only (the n part came from the heads)
        *reinterpret_cast<bf16x4*>(img_at(d2, orow, kpo, n0)) = ob;
      if (mine && !(kdbg(a.dbg) & 8)) {
        __bf16* dp = a.dy2 + (long long)gr * a.lddy2 + n0;
        if (n0 + 3 < N) *reinterpret_cast<bf16x4*>(dp) = ob;
        else
#pragma unroll
          for (int e = 0; e < 4; ++e) if (n0 + e < N) dp[e] = ob[e];
      }
    };
    if constexpr (STR)
      conv_phase_str<1, 1, NWV, 2>(d3, a.k3t.kp, a.k3t, tb0, tb1, 0, &a.k2t, n_out, pre3t, epi3t, a.dbg);
    else conv_phase<1, 1>(d3, a.k3t.kp, wimg3, a.k3t.kp, a.k3t.np, n_out, pre3t, epi3t, a.dbg);
    if (w / ncg < wpc) colpart_flush<1>(q, slots, a.k3t.np, nb0, nbc, w / ncg);
    __syncthreads();
    for (int i = tid; i < 3 * N; i += DTK) {
      const int k = i / N, n = i - k * N;
      float s = 0.f;
      for (int sl = 0; sl < wpc; ++sl) s += slots[(sl * 3 + k) * a.k3t.np + n];
      a.pc2s[(long long)t * 3 * N + i] = s;
    }
  }
  __syncthreads();
  if (stamp) ts[2] = __builtin_amdgcn_s_memrealtime();
  if constexpr (!STR) {
    if (!pre2) stage_weights(a.k2t, reinterpret_cast<char*>(wimg), kdbg(a.dbg));
    wait_dma();
  }
  if (stamp) ts[3] = __builtin_amdgcn_s_memrealtime();
  // ---- conv2^T: window [r0 - 2, r0 + own + 2): dU1 -> BN/lrelu backward -> dY1
  {
    const int wr0 = tl.r0 - 2, n_out = own + 4, W1 = a.m1.phys(), kpo = a.k1t.kp;
    const int nbc = a.k2t.np >> 4, ncg = (nbc + 1) / 2, wpc = NWV / ncg;
    const int nb0 = 2 * (w % ncg);
    float q[3][2][4] = {};
    auto pre2t = [&](int orow, int nb, f32x4 (&yp)[2]) {
                    const int gr = wr0 + orow;
                    const bool ok = orow < n_out && gr >= tl.glo && gr < tl.ghi;
#pragma unroll
                    for (int i = 0; i < 2; ++i) {   // Y1's gap / pad columns hold +0 (np = ld1)
                      yp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                      const int n0 = 16 * (nb + i) + 4 * lg;
                      if (ok && nb + i < nbc) yp[i] = *reinterpret_cast<const f32x4*>(a.y1 + (long long)gr * a.ldy1 + n0);
                    }
                  };
    auto epi2t = [&](int orow, int nb, f32x4 (&acc)[2], f32x4 (&yp)[2]) {
      if (orow >= n_out) return;
      const int gr = wr0 + orow;
      const bool ing = gr >= tl.glo && gr < tl.ghi, mine = gr >= tl.r0 && gr < tl.rend;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (nb + i >= nbc) continue;
        const int n0 = 16 * (nb + i) + 4 * lg;
        // the U1 layout's gap / pad columns: zero weights, gamma, beta and Y1, so dt = +0
        const f32x4 ga = *reinterpret_cast<const f32x4*>(&cpb[0][n0]);
        const f32x4 be = *reinterpret_cast<const f32x4*>(&cpb[1][n0]);
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float dt = ing ? acc[i][e] * lrelu_grad(yp[i][e] * ga[e] + be[e]) : 0.f;
          o[e] = dt * ga[e];
          if (mine) { q[0][i][e] += dt * yp[i][e]; q[1][i][e] += dt; q[2][i][e] += o[e]; }
        }
        bf16x4 ob;
#pragma unroll
        for (int e = 0; e < 4; ++e) ob[e] = (__bf16)o[e];
        *reinterpret_cast<bf16x4*>(img_at(d1, orow, kpo, n0)) = ob;
        if (mine && !(kdbg(a.dbg) & 8)) *reinterpret_cast<bf16x4*>(a.dy1 + (long long)gr * a.lddy1 + n0) = ob;
      }
    };
    if constexpr (STR)
      conv_phase_str<2, 2, NWV, 3>(d2, a.k2t.kp, a.k2t, tb0, tb1, 5, &a.k1t, n_out, pre2t, epi2t, a.dbg);
    else conv_phase<2, 2>(d2, a.k2t.kp, wimg, a.k2t.kp, a.k2t.np, n_out, pre2t, epi2t, a.dbg);
    __syncthreads();   // slots: the conv3^T partials were consumed above
    if (w / ncg < wpc) colpart_flush<2>(q, slots, a.k2t.np, nb0, nbc, w / ncg);
    __syncthreads();
    for (int i = tid; i < 3 * W1; i += DTK) {
      const int k = i / W1, n = i - k * W1;
      float s = 0.f;
      for (int sl = 0; sl < wpc; ++sl) s += slots[(sl * 3 + k) * a.k2t.np + n];
      a.pc1[(long long)t * 3 * W1 + i] = s;
    }
  }
  __syncthreads();
  if (stamp) ts[4] = __builtin_amdgcn_s_memrealtime();
  if constexpr (!STR) {
    stage_weights(a.k1t, reinterpret_cast<char*>(wimg), kdbg(a.dbg));
    wait_dma();
  }
  if (stamp) ts[5] = __builtin_amdgcn_s_memrealtime();
  // ---- conv1^T: own rows -> dJ (fp32)
  {
    const int n_out = own, N = a.dj;
    auto nopre = [](int, int, auto&) {};
    auto epi1t = [&](int orow, int nb, f32x4 (&acc)[2], f32x4 (&)[2]) {
      if (orow >= n_out) return;
      const long long gr = tl.r0 + orow;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int n0 = 16 * (nb + i) + 4 * lg;
        if (n0 >= N || (kdbg(a.dbg) & 8)) continue;
        *reinterpret_cast<float4*>(a.dz + gr * a.lddz + n0) =
            make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
      }
    };
    if constexpr (STR)
      conv_phase_str<2, 4, NWV, 1>(d1, a.k1t.kp, a.k1t, tb0, tb1, 10, nullptr, n_out, nopre, epi1t, a.dbg);
    else conv_phase<2, 4>(d1, a.k1t.kp, wimg, a.k1t.kp, a.k1t.np, n_out, nopre, epi1t, a.dbg);
  }
  if (stamp) {
    ts[6] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (tid == 0) {
      ts[7] = __builtin_amdgcn_s_memrealtime();
      unsigned* o = reinterpret_cast<unsigned*>(a.pc1 + (long long)t * 3 * a.m1.phys());
      for (int k = 0; k < 8; ++k) o[k] = (unsigned)ts[k];
    }
  }
}

}  // namespace

// J wider than 64 (C5's 128): the weights streamed by tap, on 64-row tiles
static bool dec_str(int dj) { return dj > 64; }
int dec_rows(int ngraphs, int npg, int dj) {
  if (dec_str(dj)) return kDecRowsSmall;
  if (ngraphs * ((npg + kDecRows - 1) / kDecRows) >= kDecSmall) return kDecRows;
  return ngraphs * ((npg + kDecRowsSmall - 1) / kDecRowsSmall) < kDecTiny ? kDecRowsTiny : kDecRowsSmall;
}
int dec_tiles(int ngraphs, int npg, int dj) {
  const int tr = dec_rows(ngraphs, npg, dj);
  return ngraphs * ((npg + tr - 1) / tr);
}
int dec_head_parts(int cin, int cout) { return head_nq(cin, cout); }

// row blocks per wave of a streamed phase (n_out rows; np columns in NBH-block groups over
// 16 waves): conv_phase_str's MAXRB at each call site bounds it
static int rb_per_wave(int n_out, int np, int nbh) {
  const int ncg = (np / 16 + nbh - 1) / nbh, wpc = NW / ncg;
  return wpc < 1 ? 1 << 20 : ((n_out + 15) / 16 + wpc - 1) / wpc;
}

bool dec_fused_supported(int dj, const ColMap& m1, const ColMap& m2, int s3, int sd, int nf,
                         const DecImg& k1, const DecImg& k2, const DecImg& k3, const DecImg& k3t,
                         const DecImg& k2t, const DecImg& k1t) {
  if (!(s3 == 10 && sd == 2 && m2.b == 20 && nf == 1)) return false;   // built heads (10,2), (20,1)
  if (dj % 16 || dj > 128 || m1.phys() > 128 || m2.phys() > 64) return false;
  DecChainFwdArgs f{};
  f.k1 = k1; f.k2 = k2; f.k3 = k3; f.m1 = m1; f.m2 = m2; f.s3 = s3; f.dj = dj;
  DecChainBwdArgs b{};
  b.k3t = k3t; b.k2t = k2t; b.k1t = k1t; b.m1 = m1; b.m2 = m2; b.s3 = s3; b.dj = dj;
  const int lim = kDynLds;
  const bool str = dec_str(dj);
  const int T = str ? kDecRowsSmall : kDecRows;   // the largest tile the kernels run
  if (FwdLay(f, T, str).total > lim || BwdLay(b, T, str).total > lim) return false;
  if (str && !(rb_per_wave(T + 8, k1.np, 2) <= 3 && rb_per_wave(T + 4, k2.np, 2) <= 2 &&
               rb_per_wave(T, k3.np, 1) <= 1 && rb_per_wave(T + 8, k3t.np, 1) <= 2 &&
               rb_per_wave(T + 4, k2t.np, 2) <= 3 && rb_per_wave(T, k1t.np, 2) <= 1))
    return false;
  if (k2.kp - k1.np > 16) return false;   // dec_fwd zeroes at most 4 pad groups of U1 per row
  // image kp: conv inputs must match the packed images
  if (k3.kp > 64 || k3t.np != 32 || k2t.np > 128 || k1t.np != ((dj + 15) / 16) * 16) return false;
  // the epilogues move whole 16-column groups of Y1 / U1 / dY1 (Y2 / U2): every image
  // column must lie inside the row's leading dimension (round_up(phys, 8))
  if (k1.np > rup(m1.phys(), 8) || k2t.np > rup(m1.phys(), 8) || k2.np > rup(m2.phys(), 8)) return false;
  return 16 % ((k2t.np / 16 + 1) / 2) == 0 && 16 % (k3t.np / 16) == 0;
}

static int dec_init_attributes_once() {
  const void* ks[] = {reinterpret_cast<const void*>(dec_fwd_kernel<kDecRows>),
                      reinterpret_cast<const void*>(dec_bwd_kernel<kDecRows>),
                      reinterpret_cast<const void*>(dec_fwd_kernel<kDecRowsSmall>),
                      reinterpret_cast<const void*>(dec_bwd_kernel<kDecRowsSmall>),
                      reinterpret_cast<const void*>(dec_fwd_kernel<kDecRowsTiny>),
                      reinterpret_cast<const void*>(dec_bwd_kernel<kDecRowsTiny>),
                      reinterpret_cast<const void*>(dec_fwd_kernel<kDecRowsSmall, NW, true>),
                      reinterpret_cast<const void*>(dec_bwd_kernel<kDecRowsSmall, NW, true>)};
  for (const void* k : ks)
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kDynLds) != hipSuccess) {
      set_error("dec: hipFuncSetAttribute failed");
      return SND_ERR_HIP;
    }
  return 0;
}

// once per process, thread-safe (a function-local static's initialiser runs exactly once)
int dec_init_attributes() {
  static const int rc = dec_init_attributes_once();
  return rc;
}

int launch_dec_chain_fwd(const DecChainFwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(a.R == a.npg * a.ngraphs && a.R > 0, "dec_fwd: R != npg * ngraphs");
  SND_CHECK_ARG(a.zb && a.y1 && a.u1 && a.y2 && a.u2 && a.dy3 && a.dy2 && a.phs && a.phn && a.sse_s &&
                    a.sse_n && a.s_truth && a.x_truth && a.zero && a.k1.w && a.k2.w && a.k3.w,
                "dec_fwd: null operand");
  SND_CHECK_ARG(a.ldz % 8 == 0 && a.ldy1 % 4 == 0 && a.ldy2 % 4 == 0 && a.lddy3 % 4 == 0 && a.lddy2 % 4 == 0,
                "dec_fwd: leading dims");
  SND_TRY(dec_init_attributes());
  const int tr = dec_rows(a.ngraphs, a.npg, a.dj);
  const dim3 grid(dec_tiles(a.ngraphs, a.npg, a.dj));
  if (dec_str(a.dj)) {
    hipLaunchKernelGGL((dec_fwd_kernel<kDecRowsSmall, NW, true>), grid, dim3(DT), FwdLay(a, tr, true).total, s, a);
    SND_LAUNCH_CHECK("dec_fwd_kernel (streamed)");
    return 0;
  }
  const size_t lds = FwdLay(a, tr).total;
  if (tr == kDecRowsTiny) hipLaunchKernelGGL(dec_fwd_kernel<kDecRowsTiny>, grid, dim3(DT), lds, s, a);
  else if (tr == kDecRowsSmall) hipLaunchKernelGGL(dec_fwd_kernel<kDecRowsSmall>, grid, dim3(DT), lds, s, a);
  else hipLaunchKernelGGL(dec_fwd_kernel<kDecRows>, grid, dim3(DT), lds, s, a);
  SND_LAUNCH_CHECK("dec_fwd_kernel");
  return 0;
}

int launch_dec_chain_bwd(const DecChainBwdArgs& a, hipStream_t s) {
  SND_CHECK_ARG(a.R == a.npg * a.ngraphs && a.R > 0, "dec_bwd: R != npg * ngraphs");
  SND_CHECK_ARG(a.y1 && a.y2 && a.dy3 && a.dy2 && a.dy1 && a.dz && a.pc2s && a.pc1 && a.zero &&
                    a.k3t.w && a.k2t.w && a.k1t.w, "dec_bwd: null operand");
  SND_CHECK_ARG(a.lddy3 % 8 == 0 && a.lddy2 % 4 == 0 && a.lddy1 % 4 == 0 && a.lddz % 4 == 0,
                "dec_bwd: leading dims");
  SND_TRY(dec_init_attributes());
  const int tr = dec_rows(a.ngraphs, a.npg, a.dj);
  const dim3 grid(dec_tiles(a.ngraphs, a.npg, a.dj));
  if (dec_str(a.dj)) {
    hipLaunchKernelGGL((dec_bwd_kernel<kDecRowsSmall, NW, true>), grid, dim3(DT), BwdLay(a, tr, true).total, s, a);
    SND_LAUNCH_CHECK("dec_bwd_kernel (streamed)");
    return 0;
  }
  const size_t lds = BwdLay(a, tr).total;
  if (tr == kDecRowsTiny) hipLaunchKernelGGL(dec_bwd_kernel<kDecRowsTiny>, grid, dim3(DT), lds, s, a);
  else if (tr == kDecRowsSmall) hipLaunchKernelGGL(dec_bwd_kernel<kDecRowsSmall>, grid, dim3(DT), lds, s, a);
  else hipLaunchKernelGGL(dec_bwd_kernel<kDecRows>, grid, dim3(DT), lds, s, a);
  SND_LAUNCH_CHECK("dec_bwd_kernel");
  return 0;
}

}  // namespace snd
