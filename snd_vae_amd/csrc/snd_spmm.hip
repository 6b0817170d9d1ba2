// CSR SpMM for GraphConvolution (layers.py:115-125) on the block-diagonal
// batch CSR, plus the per-edge terms of the inner-product CE.
//
// The reference multiplies the DENSE [B,N,N] adjacency (tf.matmul(adj,
// new_x), O(N^2 h) and N^2 bytes per graph).  Here each row gathers its
// neighbours' feature rows: 16 lanes per row, one float4 per lane per 64
// columns, neighbour loop unrolled x4 for memory-level parallelism.  The
// GraphConvolution epilogue (lrelu -> frozen BN -> concat X -> encoder_g BN,
// model.py:107-112) is fused, so H1/H2/G are written once.
// HBM-bound: per call 4(N+1) + 4 nnz + in/out feature bytes.
#include "snd_spmm.hpp"

namespace snd {
namespace {

constexpr int kRowsPerBlock = 16;  // 256 threads, 16 lanes per row

template <int EPI, bool VEC>
__global__ void __launch_bounds__(256) spmm_kernel(SpmmArgs a) {
  const int sub = threadIdx.x & 15;
  const int r = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 4);
  if (r >= a.n_rows) return;
  const int s = a.rowptr[r], e = a.rowptr[r + 1];
  constexpr int QMAX = 2;  // VEC: float4 x 2 -> width <= 128; scalar: 8 x 16 -> width <= 128
  if constexpr (VEC) {
    const int nq = a.width >> 6;  // float4 chunks of 64 columns (width % 64 == 0)
    float4 acc[QMAX];
#pragma unroll
    for (int q = 0; q < QMAX; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = s;
    for (; k + 4 <= e; k += 4) {
      int c0 = a.colidx[k], c1 = a.colidx[k + 1], c2 = a.colidx[k + 2], c3 = a.colidx[k + 3];
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        if (q >= nq) break;
        const int col = 64 * q + 4 * sub;
        float4 v0 = *reinterpret_cast<const float4*>(a.h + (long long)c0 * a.ldh + col);
        float4 v1 = *reinterpret_cast<const float4*>(a.h + (long long)c1 * a.ldh + col);
        float4 v2 = *reinterpret_cast<const float4*>(a.h + (long long)c2 * a.ldh + col);
        float4 v3 = *reinterpret_cast<const float4*>(a.h + (long long)c3 * a.ldh + col);
        acc[q].x += v0.x; acc[q].y += v0.y; acc[q].z += v0.z; acc[q].w += v0.w;
        acc[q].x += v1.x; acc[q].y += v1.y; acc[q].z += v1.z; acc[q].w += v1.w;
        acc[q].x += v2.x; acc[q].y += v2.y; acc[q].z += v2.z; acc[q].w += v2.w;
        acc[q].x += v3.x; acc[q].y += v3.y; acc[q].z += v3.z; acc[q].w += v3.w;
      }
    }
    for (; k < e; ++k) {
      int c0 = a.colidx[k];
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        if (q >= nq) break;
        float4 v0 = *reinterpret_cast<const float4*>(a.h + (long long)c0 * a.ldh + 64 * q + 4 * sub);
        acc[q].x += v0.x; acc[q].y += v0.y; acc[q].z += v0.z; acc[q].w += v0.w;
      }
    }
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      if (q >= nq) break;
      const int col = 64 * q + 4 * sub;
      float vals[4] = {acc[q].x, acc[q].y, acc[q].z, acc[q].w};
      if constexpr (EPI == SND_SPMM_PLAIN) {
        *reinterpret_cast<float4*>(a.out + (long long)r * a.ldo + col) = acc[q];
      } else {
        *reinterpret_cast<float4*>(a.pre + (long long)r * a.ldp + col) = acc[q];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int c = col + t;
          float y = lrelu(vals[t]) * (a.gamma[c] * kBnC) + a.beta[c];
          a.out[(long long)r * a.ldo + c] = y;
          if (a.out2) a.out2[(long long)r * a.ldo2 + c] = y * (a.gamma2[c] * kBnC) + a.beta2[c];
        }
      }
    }
  } else {
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    for (int k = s; k < e; ++k) {
      const float* hr = a.h + (long long)a.colidx[k] * a.ldh;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = sub + 16 * q;
        if (c < a.width) acc[q] += hr[c];
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = sub + 16 * q;
      if (c >= a.width) break;
      if constexpr (EPI == SND_SPMM_PLAIN) {
        a.out[(long long)r * a.ldo + c] = acc[q];
      } else {
        a.pre[(long long)r * a.ldp + c] = acc[q];
        float y = lrelu(acc[q]) * (a.gamma[c] * kBnC) + a.beta[c];
        a.out[(long long)r * a.ldo + c] = y;
        if (a.out2) a.out2[(long long)r * a.ldo2 + c] = y * (a.gamma2[c] * kBnC) + a.beta2[c];
      }
    }
  }
  if constexpr (EPI == SND_SPMM_GCN) {
    if (a.x && sub < a.fx) {  // concat([g, node_feature]) (model.py:109)
      const float xv = a.x[(long long)r * a.ldx + sub];
      a.out[(long long)r * a.ldo + a.width + sub] = xv;
      if (a.out2) {
        const int c = a.width + sub;
        a.out2[(long long)r * a.ldo2 + c] = xv * (a.gamma2[c] * kBnC) + a.beta2[c];
      }
    }
  }
}

// Per-edge CE terms.  For row i and each neighbour j (A_ij = 1):
//   L = z_i . z_j ;  loss += (pw - 1) softplus(L) - pw L ;  tp += (L > 0)
//   ej_i += ((pw - 1) sigmoid(L) - pw) z_j
// (pw == 1: loss -= L, ej_i = -(A z)_i.)  LPR lanes per row, float4 each.
template <int LPR, int NV>
__global__ void __launch_bounds__(256) edge_kernel(EdgeArgs a) {
  constexpr int RPB = 256 / LPR;
  const int sub = threadIdx.x % LPR;
  const int r = blockIdx.x * RPB + threadIdx.x / LPR;
  float lossr = 0.f;
  unsigned tp = 0;
  if (r < a.n_rows) {
    float4 zi[NV], acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      zi[v] = *reinterpret_cast<const float4*>(a.z + ((long long)a.row0 + r) * a.d + 4 * (sub + LPR * v));
      acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int s = a.rowptr[r], e = a.rowptr[r + 1];
    const float pw = a.pos_weight;
    auto edge = [&](const float4 (&zj)[NV], float dot) {
      float coef = -pw;
      if (pw != 1.f) {
        const float sg = 1.f / (1.f + __expf(-dot));
        const float sp = fmaxf(dot, 0.f) + log1pf(__expf(-fabsf(dot)));
        coef += (pw - 1.f) * sg;
        lossr += (pw - 1.f) * sp;
      }
      lossr -= pw * dot;
      tp += dot > 0.f ? 1u : 0u;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        acc[v].x += coef * zj[v].x; acc[v].y += coef * zj[v].y;
        acc[v].z += coef * zj[v].z; acc[v].w += coef * zj[v].w;
      }
    };
    auto dot4 = [&](const float4 (&zj)[NV]) {
      float d = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v)
        d += zi[v].x * zj[v].x + zi[v].y * zj[v].y + zi[v].z * zj[v].z + zi[v].w * zj[v].w;
      return d;
    };
    int k = s;
    for (; k + 4 <= e; k += 4) {            // 4 neighbours in flight, independent reductions
      int cc[4];
      float4 zj[4][NV];
      float dd[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) cc[u] = a.colidx[k + u];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v)
          zj[u][v] = *reinterpret_cast<const float4*>(a.z + (long long)cc[u] * a.d + 4 * (sub + LPR * v));
#pragma unroll
      for (int u = 0; u < 4; ++u) dd[u] = dot4(zj[u]);
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1)
#pragma unroll
        for (int u = 0; u < 4; ++u) dd[u] += __shfl_xor(dd[u], o, 64);
#pragma unroll
      for (int u = 0; u < 4; ++u) edge(zj[u], dd[u]);
    }
    for (; k < e; ++k) {
      const int c = a.colidx[k];
      float4 zj[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v)
        zj[v] = *reinterpret_cast<const float4*>(a.z + (long long)c * a.d + 4 * (sub + LPR * v));
      float dot = dot4(zj);
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
      edge(zj, dot);
    }
#pragma unroll
    for (int v = 0; v < NV; ++v)
      *reinterpret_cast<float4*>(a.ej + (long long)r * a.d + 4 * (sub + LPR * v)) = acc[v];
    if (sub != 0) { lossr = 0.f; tp = 0; }  // every lane of the row holds the same sums
  }
  __shared__ double sl[4];
  __shared__ unsigned st[4];
  double l = wave_sum_d((double)lossr);
  unsigned t = wave_sum_u(tp);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sl[w] = l; st[w] = t; }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.part[2 * blockIdx.x] = sl[0] + sl[1] + sl[2] + sl[3];
    a.part[2 * blockIdx.x + 1] = (double)(st[0] + st[1] + st[2] + st[3]);
  }
}

}  // namespace

int launch_spmm(const SpmmArgs& a, hipStream_t s) {
  if (a.n_rows <= 0) return 0;
  if (a.width <= 0 || a.width > 128) {
    set_error("spmm: width %d outside 1..128", a.width);
    return SND_ERR_ARG;
  }
  // float4 gathers need aligned input rows; the GCN epilogue stores `out`
  // per element (its ld, e.g. 67 = h + f_in, is not 16-B aligned)
  const bool vec = (a.width % 64 == 0) && (a.ldh % 4 == 0) &&
                   ((uintptr_t)a.h % 16 == 0) &&
                   (a.epilogue == SND_SPMM_PLAIN
                        ? (a.ldo % 4 == 0 && (uintptr_t)a.out % 16 == 0)
                        : (a.ldp % 4 == 0 && (uintptr_t)a.pre % 16 == 0));
  dim3 grid(cdiv(a.n_rows, kRowsPerBlock));
  if (a.epilogue == SND_SPMM_PLAIN) {
    if (vec) hipLaunchKernelGGL((spmm_kernel<SND_SPMM_PLAIN, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((spmm_kernel<SND_SPMM_PLAIN, false>), grid, dim3(256), 0, s, a);
  } else {
    if (vec) hipLaunchKernelGGL((spmm_kernel<SND_SPMM_GCN, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((spmm_kernel<SND_SPMM_GCN, false>), grid, dim3(256), 0, s, a);
  }
  SND_LAUNCH_CHECK("spmm_kernel");
  return 0;
}

int edge_blocks(int n_rows, int d) {
  const int lpr = d >= 64 ? 16 : d / 4;
  return cdiv(n_rows, 256 / lpr);
}

int launch_edge(const EdgeArgs& a, hipStream_t s) {
  dim3 grid(edge_blocks(a.n_rows, a.d));
  switch (a.d) {
    case 16: hipLaunchKernelGGL((edge_kernel<4, 1>), grid, dim3(256), 0, s, a); break;
    case 32: hipLaunchKernelGGL((edge_kernel<8, 1>), grid, dim3(256), 0, s, a); break;
    case 64: hipLaunchKernelGGL((edge_kernel<16, 1>), grid, dim3(256), 0, s, a); break;
    case 128: hipLaunchKernelGGL((edge_kernel<16, 2>), grid, dim3(256), 0, s, a); break;
    default: set_error("edge terms: d=%d not in {16,32,64,128}", a.d); return SND_ERR_ARG;
  }
  SND_LAUNCH_CHECK("edge_kernel");
  return 0;
}

}  // namespace snd

using namespace snd;

extern "C" int snd_csr_spmm(const int* rowptr, const int* colidx, int n_rows,
                            const float* h, int ldh, int width, float* out,
                            int ldo, int epilogue, const float* bn_gamma,
                            const float* bn_beta, float* preact, int ldp,
                            const float* concat_x, int ldx, int fx,
                            const float* bn2_gamma, const float* bn2_beta,
                            float* out2, int ldo2, snd_stream_t stream) {
  // colidx may be NULL for an edgeless batch (never dereferenced when nnz == 0)
  SND_CHECK_ARG(n_rows >= 0 && rowptr && h && out, "snd_csr_spmm: null operand");
  SND_CHECK_ARG(epilogue == SND_SPMM_PLAIN || epilogue == SND_SPMM_GCN,
                "snd_csr_spmm: bad epilogue %d", epilogue);
  SND_CHECK_ARG(epilogue == SND_SPMM_PLAIN || (bn_gamma && bn_beta && preact),
                "snd_csr_spmm: GCN epilogue needs gamma, beta, preact");
  SND_CHECK_ARG(!out2 || (bn2_gamma && bn2_beta), "snd_csr_spmm: out2 needs bn2");
  SND_CHECK_ARG(fx >= 0 && fx <= 16 && (fx == 0 || concat_x), "snd_csr_spmm: fx in 0..16");
  SpmmArgs a{};
  a.rowptr = rowptr; a.colidx = colidx; a.n_rows = n_rows;
  a.h = h; a.ldh = ldh; a.width = width; a.out = out; a.ldo = ldo;
  a.epilogue = epilogue; a.gamma = bn_gamma; a.beta = bn_beta; a.pre = preact; a.ldp = ldp;
  a.x = concat_x; a.ldx = ldx; a.fx = fx;
  a.gamma2 = bn2_gamma; a.beta2 = bn2_beta; a.out2 = out2; a.ldo2 = ldo2;
  return launch_spmm(a, (hipStream_t)stream);
}
