// Generic small-GEMM engine on gfx950 MFMA for the SND-VAE dense ops:
// linear() (layers.py:566-576), GraphConvolution's X@w (layers.py:120-121),
// conv1d k=5 SAME as implicit GEMM (model_joint.py:115,138) and all their
// backward products.  Operands are fp32 in HBM; tiles are converted to the
// MFMA operand type (bf16 or f32) when staged into LDS; accumulation is fp32.
//
// Tile: 64(M) x 64(N) x 64(K), 256 threads = 4 waves in a 2x2 grid of 32x32
// wave tiles (2x2 MFMA 16x16 sub-tiles).  Operand "views" decouple memory
// layout from the GEMM: plain / transposed matrices, conv im2col (taps never
// cross a graph boundary: zero padding 2|2 per graph, TF SAME), flipped conv
// weights for the data gradient.  Two register stages of prefetch (tile t+2
// loads issued before tile t's MFMAs).  Weight gradients use deterministic split-K
// partial slabs reduced by snd_reduce (no float atomics: bitwise reproducible).
#include "snd_gemm.hpp"

#include <type_traits>

namespace snd {

namespace {

constexpr int BM = 64, BN = 64, BK = kGemmBK, NT = 256;

__device__ __forceinline__ int cdiv_d(int a, int b) { return (a + b - 1) / b; }

template <typename T> struct LdsStride;
template <> struct LdsStride<float> { static constexpr int v = BK + 2; };   // 66: conflict-free b32 reads
template <> struct LdsStride<__bf16> { static constexpr int v = BK + 8; };  // 72 (144 B rows): conflict-free b128

// ---- operand tile loaders, lane-contiguous: lane l of a wave reads element l
// of 64 consecutive elements along the operand's contiguous memory axis, and
// the 4 waves x 16 registers cover the 64 rows of the tile (row = wave + 4 i).
// Per-lane index math (conv tap t / channel c) is done once per tile.
// A views a(m, k): k-contiguous A_ROW, A_CONV;  m-contiguous A_COL, A_CONVT.
// B views b(k, n): n-contiguous B_ROW;          k-contiguous B_COL, B_FLIP.
constexpr int RPT = BK / 4;   // rows per thread per tile (16)

// node-local index of row `base + q + 4 i` inside its graph, stepped without division
struct LocalRow {
  int local, npg;
  __device__ __forceinline__ LocalRow(int row, int npg_) : local(row % npg_), npg(npg_) {}
  __device__ __forceinline__ void step4() {
    local += 4;
    while (local >= npg) local -= npg;
  }
};

template <int AM>
__device__ __forceinline__ void load_a_tile(const GemmArgs& g, int m0, int k0, float (&v)[RPT]) {
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  if constexpr (AM == A_ROW) {
    const int k = k0 + lane;
    const bool kv = k < g.K;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int m = m0 + q + 4 * i;
      v[i] = (kv && m < g.M) ? g.A[(long long)m * g.lda + k] : 0.f;
    }
  } else if constexpr (AM == A_CONV) {           // m = node row, k = t*cin + c
    const int k = k0 + lane;
    const bool kv = k < g.K;
    const int t = k / g.a_cin, c = k - t * g.a_cin;
    LocalRow lr(m0 + q, g.a_npg);
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int m = m0 + q + 4 * i;
      const int src = lr.local + t - 2;
      v[i] = (kv && m < g.M && src >= 0 && src < g.a_npg)
                 ? g.A[(long long)(m + t - 2) * g.lda + c] : 0.f;
      lr.step4();
    }
  } else if constexpr (AM == A_COL) {            // a(m, k) = A[k][m]
    const int m = m0 + lane;
    const bool mv = m < g.M, ones = (m + 1 == g.a_ones_m1);
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int k = k0 + q + 4 * i;
      v[i] = (mv && k < g.K) ? (ones ? 1.f : g.A[(long long)k * g.lda + m]) : 0.f;
    }
  } else {                                       // A_CONVT: m = t*cin + c, k = node row
    const int m = m0 + lane;
    const bool mv = m < g.M;
    const int t = m / g.a_cin, c = m - t * g.a_cin;
    LocalRow lr(k0 + q, g.a_npg);
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int k = k0 + q + 4 * i;
      const int src = lr.local + t - 2;
      v[i] = (mv && k < g.K && src >= 0 && src < g.a_npg)
                 ? g.A[(long long)(k + t - 2) * g.lda + c] : 0.f;
      lr.step4();
    }
  }
}

template <int BMODE>
__device__ __forceinline__ void load_b_tile(const GemmArgs& g, int k0, int n0, float (&v)[RPT]) {
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  if constexpr (BMODE == B_ROW) {                // n = lane, k = rows
    const int n = n0 + lane;
    const bool nv = n < g.N;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int k = k0 + q + 4 * i;
      v[i] = (nv && k < g.K) ? g.B[(long long)k * g.ldb + n] : 0.f;
    }
  } else if constexpr (BMODE == B_COL) {         // k = lane, n = rows
    const int k = k0 + lane;
    const bool kv = k < g.K;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int n = n0 + q + 4 * i;
      v[i] = (kv && n < g.N) ? g.B[(long long)n * g.ldb + k] : 0.f;
    }
  } else {                                       // B_FLIP: k = t*cout + o = lane, n = rows
    const int k = k0 + lane;
    const bool kv = k < g.K;
    const int t = k / g.b_cout, o = k - t * g.b_cout;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int n = n0 + q + 4 * i;
      v[i] = (kv && n < g.N) ? g.B[((long long)(4 - t) * g.N + n) * g.b_cout + o] : 0.f;
    }
  }
}

template <int I> using IC = std::integral_constant<int, I>;

template <typename T, int AM, int BMODE, int EPI>
__global__ void __launch_bounds__(NT) gemm_kernel(GemmArgs g) {
  constexpr int S = LdsStride<T>::v;
  __shared__ __attribute__((aligned(16))) T As[BM * S];
  __shared__ __attribute__((aligned(16))) T Bs[BN * S];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int ntile = kend > kbeg ? cdiv_d(kend - kbeg, BK) : 0;

  constexpr bool a_kc = (AM == A_ROW || AM == A_CONV);
  constexpr bool b_kc = (BMODE == B_COL || BMODE == B_FLIP);
  const int q = tid >> 6;

  float ra[2][RPT], rb[2][RPT];   // [stage][row]
  auto gload = [&](auto stc, int k0) {
    constexpr int st = decltype(stc)::value;
    load_a_tile<AM>(g, m0, k0, ra[st]);
    load_b_tile<BMODE>(g, k0, n0, rb[st]);
  };
  auto sstore = [&](auto stc) {
    constexpr int st = decltype(stc)::value;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int rr = q + 4 * i;
      if (a_kc) As[rr * S + lane] = (T)ra[st][i];     // row m = rr, col k = lane
      else As[lane * S + rr] = (T)ra[st][i];          // row m = lane, col k = rr
      if (b_kc) Bs[rr * S + lane] = (T)rb[st][i];     // row n = rr, col k = lane
      else Bs[lane * S + rr] = (T)rb[st][i];          // row n = lane, col k = rr
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&]() {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int ss = 0; ss < BK / 32; ++ss) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(&As[(32 * wr + 16 * i + fr) * S + 32 * ss + 8 * fq]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[(32 * wc + 16 * j + fr) * S + 32 * ss + 8 * fq]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = As[(32 * wr + 16 * i + fr) * S + 4 * ks + fq];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = Bs[(32 * wc + 16 * j + fr) * S + 4 * ks + fq];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // two register stages: tile t+2's loads are issued before tile t's MFMAs
  if (ntile > 0) gload(IC<0>{}, kbeg);
  if (ntile > 1) gload(IC<1>{}, kbeg + BK);
  for (int t = 0; t < ntile; t += 2) {
    sstore(IC<0>{});
    __syncthreads();
    if (t + 2 < ntile) gload(IC<0>{}, kbeg + (t + 2) * BK);
    compute();
    __syncthreads();
    if (t + 1 < ntile) {
      sstore(IC<1>{});
      __syncthreads();
      if (t + 3 < ntile) gload(IC<1>{}, kbeg + (t + 3) * BK);
      compute();
      __syncthreads();
    }
  }

  // epilogue: C/D map of 16x16 MFMA -- col = lane&15, row = 4*(lane>>4) + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 32 * wr + 16 * i + 4 * fq + r;
        const int n = n0 + 32 * wc + 16 * j + fr;
        if (m >= g.M || n >= g.N) continue;
        float v = acc[i][j][r];
        if constexpr (EPI == E_STORE) {
          if (g.bias) v += g.bias[n];
          if (g.accumulate) v += g.C[(long long)m * g.ldc + n];
          g.C[(long long)m * g.ldc + n] = v;
        } else if constexpr (EPI == E_CONV) {
          if (g.bias) v += g.bias[n];
          if (g.gamma) {
            g.pre[(long long)m * g.ldp + n] = v;
            v = lrelu(v * (g.gamma[n] * kBnC) + g.beta[n]);
          }
          g.C[(long long)m * g.ldc + n] = v;
        } else {  // E_PART: slab [z][M][N]
          g.C[((long long)blockIdx.z * g.M + m) * g.N + n] = v;
        }
      }
}

template <typename T, int AM, int BMODE>
int launch_epi(const GemmArgs& g, int epi, int splits, hipStream_t s) {
  dim3 grid(cdiv(g.M, BM), cdiv(g.N, BN), splits);
  switch (epi) {
    case E_STORE: hipLaunchKernelGGL((gemm_kernel<T, AM, BMODE, E_STORE>), grid, dim3(NT), 0, s, g); break;
    case E_CONV: hipLaunchKernelGGL((gemm_kernel<T, AM, BMODE, E_CONV>), grid, dim3(NT), 0, s, g); break;
    case E_PART: hipLaunchKernelGGL((gemm_kernel<T, AM, BMODE, E_PART>), grid, dim3(NT), 0, s, g); break;
    default: set_error("gemm: bad epilogue %d", epi); return SND_ERR_ARG;
  }
  SND_LAUNCH_CHECK("gemm_kernel");
  return 0;
}

template <typename T>
int launch_t(const GemmArgs& g, int am, int bm, int epi, int splits, hipStream_t s) {
#define SND_AB(AV, BV) \
  if (am == AV && bm == BV) return launch_epi<T, AV, BV>(g, epi, splits, s);
  SND_AB(A_ROW, B_ROW) SND_AB(A_ROW, B_COL) SND_AB(A_COL, B_ROW) SND_AB(A_COL, B_COL)
  SND_AB(A_CONV, B_ROW) SND_AB(A_CONV, B_FLIP) SND_AB(A_CONVT, B_ROW)
#undef SND_AB
  set_error("gemm: unsupported operand modes a=%d b=%d", am, bm);
  return SND_ERR_ARG;
}

}  // namespace

int launch_gemm(GemmArgs g, int amode, int bmode, int epi, int dtype, int splits,
                hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return 0;
  if (splits < 1) splits = 1;
  if (g.kchunk <= 0) g.kchunk = (int)round_up(cdiv(g.K, splits), BK);
  g.kchunk = (int)round_up(g.kchunk, BK);
  splits = cdiv(g.K, g.kchunk);
  if (splits < 1) splits = 1;
  if (epi != E_PART && splits != 1) {
    set_error("gemm: split-K requires the partial epilogue");
    return SND_ERR_ARG;
  }
  if (dtype == SND_BF16) return launch_t<__bf16>(g, amode, bmode, epi, splits, s);
  if (dtype == SND_F32) return launch_t<float>(g, amode, bmode, epi, splits, s);
  set_error("gemm: bad dtype %d", dtype);
  return SND_ERR_ARG;
}

int gemm_splits(int K, int target_blocks_per_tile) {
  int s = cdiv(K, 1024);
  if (s > target_blocks_per_tile) s = target_blocks_per_tile;
  return s < 1 ? 1 : s;
}

}  // namespace snd

using namespace snd;

extern "C" int snd_gemm(int trans_a, int trans_b, int m, int n, int k,
                        const float* a, int lda, const float* b, int ldb,
                        float* c, int ldc, const float* bias, int dtype,
                        snd_stream_t stream) {
  SND_CHECK_ARG(m >= 0 && n >= 0 && k >= 0, "snd_gemm: negative shape");
  SND_CHECK_ARG(a && b && c, "snd_gemm: null operand");
  GemmArgs g{};
  g.M = m; g.N = n; g.K = k;
  g.A = a; g.lda = lda; g.B = b; g.ldb = ldb; g.C = c; g.ldc = ldc; g.bias = bias;
  g.kchunk = (int)round_up(k > 0 ? k : 1, kGemmBK);
  return launch_gemm(g, trans_a ? A_COL : A_ROW, trans_b ? B_COL : B_ROW, E_STORE,
                     dtype, 1, (hipStream_t)stream);
}

extern "C" int snd_conv1d_same_fwd(const float* x, int ldx, int rows, int npg,
                                   int cin, const float* w, int cout,
                                   const float* bias, const float* gamma,
                                   const float* beta, float* y_pre, int ldy,
                                   float* out, int ldo, int dtype,
                                   snd_stream_t stream) {
  SND_CHECK_ARG(rows >= 0 && npg > 0 && rows % npg == 0, "conv1d: rows must be B*N");
  SND_CHECK_ARG(x && w && out, "conv1d: null operand");
  SND_CHECK_ARG(!gamma || (beta && y_pre), "conv1d: BN needs beta and y_pre");
  GemmArgs g{};
  g.M = rows; g.N = cout; g.K = 5 * cin;
  g.A = x; g.lda = ldx; g.a_cin = cin; g.a_npg = npg;
  g.B = w; g.ldb = cout;
  g.C = out; g.ldc = ldo; g.bias = bias; g.gamma = gamma; g.beta = beta;
  g.pre = y_pre; g.ldp = ldy;
  g.kchunk = (int)round_up(g.K, kGemmBK);
  return launch_gemm(g, A_CONV, B_ROW, E_CONV, dtype, 1, (hipStream_t)stream);
}

extern "C" int snd_conv1d_same_bwd_data(const float* dy, int lddy, int rows,
                                        int npg, int cout, const float* w,
                                        int cin, float* dx, int lddx, int dtype,
                                        snd_stream_t stream) {
  SND_CHECK_ARG(rows >= 0 && npg > 0 && rows % npg == 0, "conv1d: rows must be B*N");
  // dx[r,c] = sum_t sum_o dy[r - t + 2, o] w[t,c,o]  == conv over dy with taps
  // t' = 4 - t: A_CONV on dy (cin := cout) and B_FLIP weights.
  GemmArgs g{};
  g.M = rows; g.N = cin; g.K = 5 * cout;
  g.A = dy; g.lda = lddy; g.a_cin = cout; g.a_npg = npg;
  g.B = w; g.b_cout = cout;
  g.C = dx; g.ldc = lddx;
  g.kchunk = (int)round_up(g.K, kGemmBK);
  return launch_gemm(g, A_CONV, B_FLIP, E_STORE, dtype, 1, (hipStream_t)stream);
}

extern "C" size_t snd_conv1d_bwd_weight_workspace(int rows, int cin, int cout) {
  int splits = gemm_splits(rows, 64);
  return (size_t)splits * 5 * cin * cout * sizeof(float);
}

extern "C" int snd_conv1d_same_bwd_weight(const float* x, int ldx, const float* dy,
                                          int lddy, int rows, int npg, int cin,
                                          int cout, float* dw, void* ws,
                                          size_t ws_bytes, int dtype,
                                          snd_stream_t stream) {
  SND_CHECK_ARG(rows >= 0 && npg > 0 && rows % npg == 0, "conv1d: rows must be B*N");
  size_t need = snd_conv1d_bwd_weight_workspace(rows, cin, cout);
  SND_CHECK_ARG(ws && ws_bytes >= need, "conv1d bwd_weight: workspace %zu < %zu", ws_bytes, need);
  int splits = gemm_splits(rows, 64);
  GemmArgs g{};
  g.M = 5 * cin; g.N = cout; g.K = rows;
  g.A = x; g.lda = ldx; g.a_cin = cin; g.a_npg = npg;
  g.B = dy; g.ldb = lddy;
  g.C = (float*)ws;
  g.kchunk = (int)round_up(cdiv(rows, splits), kGemmBK);
  splits = cdiv(rows, g.kchunk);
  SND_TRY(launch_gemm(g, A_CONVT, B_ROW, E_PART, dtype, splits, (hipStream_t)stream));
  ReduceDesc d{(const float*)ws, dw, splits, 5 * cin * cout, 5 * cin * cout, 1.f, 0};
  return launch_reduce(&d, 1, (hipStream_t)stream);
}
