// SpatialGraphConvolution (layers.py:143-198) and the model_joint spatial-graph
// encoder layer lrelu(BN(SGConv)) (model_joint.py:77-80), forward and backward.
//
// The reference materialises B x N x N x N x (3F+3) message tensors.  Here the
// layer is factorised: lrelu acts on the CONCATENATED INPUTS (x, rel), so the
// first message layer is a sum of per-node / per-edge terms and the sum over k
// of the 2-hop messages collapses to node and edge quantities (A binary):
//   S3_ij = A_ij [ d_j (u_i + v_j + lr_ij m1r + b1) + w_j + e_j m1s + Q_ij m1t ]
//     u = lrelu(X) M1x, v = lrelu(X) M1y, w = (A lrelu(X)) M1z, d = degree,
//     lr_ij = lrelu(rel_ij), e_j = sum_k A_jk lr_jk, Q_ij = sum_k A_jk lrelu(rel_ik)
//   m2_i = d_i (lrelu(x_i) M2x + b2) + (A lrelu X)_i M2y + e_i m2r + P_i M2s,
//     P_i = sum_j A_ij lrelu(S3_ij)
//   out_i = [lrelu(x_i), lrelu(m2_i)] M3 + b3
// Cost O(nnz (h0 + deg)) + row GEMMs instead of O(B N^3 h0).  Edge scalars
// (lr, Q, reverse-edge index) depend only on the data and are prepared once per
// batch (snd_sg_prep).  The dense products run on the generic MFMA GEMM (fp32
// operands: exact fp32 FMA chains); weight gradients are deterministic split-K
// slabs reduced in fixed order.  Backward derivation: DESIGN.md §8 (SG encoder).
#include <algorithm>

#include "snd_gemm.hpp"
#include "snd_sg.hpp"

namespace snd {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ float lr(float x) { return x >= 0.f ? x : kLeak * x; }
__device__ __forceinline__ float lrg(float x) { return x >= 0.f ? 1.f : kLeak; }

struct Geo {   // per-layer widths and workspace map (floats)
  int F, h0, h1, h2, ld2, ld3;
  long long R;
  long long oZ2, oUVW, oM2P, oZ3, oDY, oDTY, oDZ3, oDM2, oDZ2, oDUVW, oTM, oDLX, oDAX, oSLAB;
  long long slab, total;
  int splits;
};

long long r64(long long n) { return (n + 63) / 64 * 64; }

Geo geo(long long R, int F, int h0, int h1, int h2) {
  Geo g{};
  g.F = F; g.h0 = h0; g.h1 = h1; g.h2 = h2; g.R = R;
  g.ld2 = 2 * F + 2 + h0;
  g.ld3 = F + h1 + 1;
  long long o = 0;
  auto take = [&](long long n) { long long r = o; o += r64(n); return r; };
  g.oZ2 = take(R * g.ld2);
  g.oUVW = take(R * 3 * h0);
  g.oM2P = take(R * h1);
  g.oZ3 = take(R * g.ld3);
  g.oDY = take(R * h2);
  g.oDTY = take(R * 2 * h2);
  g.oDZ3 = take(R * (F + h1));
  g.oDM2 = take(R * h1);
  g.oDZ2 = take(R * (2 * F + 1 + h0));
  g.oDUVW = take(R * 3 * h0);
  g.oTM = take(R * 4 * h0);
  g.oDLX = take(R * F);
  g.oDAX = take(R * F);
  g.splits = std::max(1, std::min(64, cdiv(R, 4096)));
  long long mn = std::max<long long>({(long long)g.ld3 * h2, (long long)g.ld2 * h1,
                                      (long long)F * h0, 2LL * h2, 4LL * h0});
  g.slab = (long long)g.splits * mn;
  g.oSLAB = take(g.slab);
  g.total = o;
  return g;
}

struct POff { long long M1, b1, M2, b2, M3, b3, gamma, beta, total; };
POff poff(int F, int h0, int h1, int h2) {
  POff p{};
  p.M1 = 0;
  p.b1 = p.M1 + (long long)(3 * F + 3) * h0;
  p.M2 = p.b1 + h0;
  p.b2 = p.M2 + (long long)(2 * F + 1 + h0) * h1;
  p.M3 = p.b2 + h1;
  p.b3 = p.M3 + (long long)(F + h1) * h2;
  p.gamma = p.b3 + h2;
  p.beta = p.gamma + h2;
  p.total = p.beta + h2;
  return p;
}

// ------------------------------------------------------------------ edge prep
// one thread per row i: for each edge (i, j): lr_ij, Q_ij = sum_{k in N(j)} lrelu(rel_ik),
// rev = position of (j, i) in row j (binary search; -1 and a count if absent), e_i, d_i.
__global__ void __launch_bounds__(NT) sg_prep_kernel(snd_sg_graph_t g, const float* rel,
                                                     int* unmatched) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= g.n_rows) return;
  const int n = g.n_per_graph, b = i / n, li = i - b * n;
  const float* rrow = rel + ((long long)b * n + li) * n;
  const int s = g.rowptr[i], e = g.rowptr[i + 1];
  float esum = 0.f;
  int bad = 0;
  for (int q = s; q < e; ++q) {
    const int j = g.colidx[q];
    const float l = lr(rrow[j - b * n]);
    esum += l;
    g.edge_lr[q] = l;
    float qs = 0.f;
    const int js = g.rowptr[j], je = g.rowptr[j + 1];
    int lo = js, hi = je;
    for (int t = js; t < je; ++t) qs += lr(rrow[g.colidx[t] - b * n]);
    while (lo < hi) {                          // colidx sorted within a row
      const int mid = (lo + hi) >> 1;
      if (g.colidx[mid] < i) lo = mid + 1; else hi = mid;
    }
    const int rev = (lo < je && g.colidx[lo] == i) ? lo : -1;
    bad += rev < 0;
    g.edge_q[q] = qs;
    g.edge_rev[q] = rev;
  }
  g.node_e[i] = esum;
  g.node_deg[i] = (float)(e - s);
  if (bad) atomicAdd(unmatched, bad);
}

// ------------------------------------------------------------------ forward
// thread per (row, f): LX, A LX; Z2e = [d LX | A LX | e | P (later) | d], Z3e = [LX | . | 1]
__global__ void __launch_bounds__(NT) sg_gather_kernel(snd_sg_graph_t g, const float* x, int ldx,
                                                       Geo G, float* ws) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.F) return;
  const int i = (int)(idx / G.F), f = (int)(idx - (long long)i * G.F);
  const float l = lr(x[(long long)i * ldx + f]);
  float ax = 0.f;
  for (int q = g.rowptr[i]; q < g.rowptr[i + 1]; ++q) ax += lr(x[(long long)g.colidx[q] * ldx + f]);
  const float d = g.node_deg[i];
  float* z2 = ws + G.oZ2 + (long long)i * G.ld2;
  float* z3 = ws + G.oZ3 + (long long)i * G.ld3;
  z2[f] = d * l;
  z2[G.F + f] = ax;
  z3[f] = l;
  if (f == 0) {
    z2[2 * G.F] = g.node_e[i];
    z2[2 * G.F + 1 + G.h0] = d;
    z3[G.F + G.h1] = 1.f;
  }
}

// S3 of edge q = (i -> j), channel c
__device__ __forceinline__ float s3_of(const float* uvw, int h0, int i, int j, int c, float dj,
                                       float ej, float lrq, float qq, const float* m1r,
                                       const float* m1s, const float* m1t, const float* b1) {
  const float* ui = uvw + (long long)i * 3 * h0;
  const float* uj = uvw + (long long)j * 3 * h0;
  return dj * (ui[c] + uj[h0 + c] + lrq * m1r[c] + b1[c]) + uj[2 * h0 + c] + ej * m1s[c] +
         qq * m1t[c];
}

// thread per (row i, c < h0): P_i = sum_j lrelu(S3_ij) -> Z2e[i, 2F+1+c]
__global__ void __launch_bounds__(NT) sg_edge_fwd_kernel(snd_sg_graph_t g, Geo G, const float* prm,
                                                         POff po, float* ws) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.h0) return;
  const int i = (int)(idx / G.h0), c = (int)(idx - (long long)i * G.h0);
  const float* m1 = prm + po.M1;
  const float* m1r = m1 + (long long)3 * G.F * G.h0;
  const float* m1s = m1r + G.h0;
  const float* m1t = m1s + G.h0;
  const float* uvw = ws + G.oUVW;
  float acc = 0.f;
  for (int q = g.rowptr[i]; q < g.rowptr[i + 1]; ++q) {
    const int j = g.colidx[q];
    acc += lr(s3_of(uvw, G.h0, i, j, c, g.node_deg[j], g.node_e[j], g.edge_lr[q], g.edge_q[q],
                    m1r, m1s, m1t, prm + po.b1));
  }
  ws[G.oZ2 + (long long)i * G.ld2 + 2 * G.F + 1 + c] = acc;
}

// Z3e[:, F + c] = lrelu(m2)
__global__ void __launch_bounds__(NT) sg_act_kernel(Geo G, float* ws) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.h1) return;
  const long long i = idx / G.h1;
  const int c = (int)(idx - i * G.h1);
  ws[G.oZ3 + i * G.ld3 + G.F + c] = lr(ws[G.oM2P + idx]);
}

// encoder epilogue: out = lrelu(BN(y)) (model_joint.py:78-79) or out = y
__global__ void __launch_bounds__(NT) sg_bn_fwd_kernel(long long n, int h2, const float* y,
                                                       const float* gamma, const float* beta,
                                                       float* out) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= n) return;
  const int c = (int)(idx % h2);
  out[idx] = lr(y[idx] * (gamma[c] * kBnC) + beta[c]);
}

// ------------------------------------------------------------------ backward
// DY = dout lrelu'(t) gamma c; DTY = [dT | dT y c] (column sums -> dbeta, dgamma)
__global__ void __launch_bounds__(NT) sg_bn_bwd_kernel(Geo G, const float* y, const float* dout,
                                                       const float* gamma, const float* beta,
                                                       float* ws) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.h2) return;
  const long long i = idx / G.h2;
  const int c = (int)(idx - i * G.h2);
  const float yv = y[idx];
  const float dt = dout[idx] * lrg(yv * (gamma[c] * kBnC) + beta[c]);
  ws[G.oDY + idx] = dt * gamma[c] * kBnC;
  float* dty = ws + G.oDTY + i * 2 * G.h2;
  dty[c] = dt;
  dty[G.h2 + c] = dt * yv * kBnC;
}

// DM2 = dZ3[:, F:] lrelu'(m2)
__global__ void __launch_bounds__(NT) sg_act_bwd_kernel(Geo G, float* ws) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.h1) return;
  const long long i = idx / G.h1;
  const int c = (int)(idx - i * G.h1);
  ws[G.oDM2 + idx] = ws[G.oDZ3 + i * (G.F + G.h1) + G.F + c] * lrg(ws[G.oM2P + idx]);
}

// thread per (row r, c < h0), G_ij = dP_i lrelu'(S3_ij):
//   du_r = sum_n G_rn d_n;  dw_r = sum_n G_nr (reverse edges);  dv_r = d_r dw_r
//   TM_r = [sum_n G_rn d_n lr_rn | du_r | sum_n G_rn e_n | sum_n G_rn Q_rn]
__global__ void __launch_bounds__(NT) sg_edge_bwd_kernel(snd_sg_graph_t g, Geo G, const float* prm,
                                                         POff po, float* ws) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.h0) return;
  const int r = (int)(idx / G.h0), c = (int)(idx - (long long)r * G.h0);
  const float* m1 = prm + po.M1;
  const float* m1r = m1 + (long long)3 * G.F * G.h0;
  const float* m1s = m1r + G.h0;
  const float* m1t = m1s + G.h0;
  const float* b1 = prm + po.b1;
  const float* uvw = ws + G.oUVW;
  const int ldz2 = 2 * G.F + 1 + G.h0;
  const float* dz2 = ws + G.oDZ2;
  const float dPr = dz2[(long long)r * ldz2 + 2 * G.F + 1 + c];
  const float dr = g.node_deg[r], er = g.node_e[r];
  float du = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f, dw = 0.f;
  for (int q = g.rowptr[r]; q < g.rowptr[r + 1]; ++q) {
    const int n = g.colidx[q];
    const float dn = g.node_deg[n], en = g.node_e[n];
    const float lq = g.edge_lr[q], qq = g.edge_q[q];
    const float Gf = dPr * lrg(s3_of(uvw, G.h0, r, n, c, dn, en, lq, qq, m1r, m1s, m1t, b1));
    du += Gf * dn;
    t1 += Gf * dn * lq;
    t2 += Gf * en;
    t3 += Gf * qq;
    const int qr = g.edge_rev[q];               // edge (n -> r)
    const float dPn = dz2[(long long)n * ldz2 + 2 * G.F + 1 + c];
    dw += dPn * lrg(s3_of(uvw, G.h0, n, r, c, dr, er, g.edge_lr[qr], g.edge_q[qr], m1r, m1s, m1t,
                          b1));
  }
  float* o = ws + G.oDUVW + (long long)r * 3 * G.h0;
  o[c] = du;
  o[G.h0 + c] = dr * dw;
  o[2 * G.h0 + c] = dw;
  float* t = ws + G.oTM + (long long)r * 4 * G.h0;
  t[c] = t1;
  t[G.h0 + c] = du;
  t[2 * G.h0 + c] = t2;
  t[3 * G.h0 + c] = t3;
}

// thread per (row i, f): dLX = dZ3[:, f] + d dZ2[:, f] + du M1x^T + dv M1y^T;
//                        dAX = dZ2[:, F + f] + dw M1z^T
__global__ void __launch_bounds__(NT) sg_bwd_node_kernel(snd_sg_graph_t g, Geo G, const float* prm,
                                                         POff po, float* ws) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.F) return;
  const int i = (int)(idx / G.F), f = (int)(idx - (long long)i * G.F);
  const float* m1 = prm + po.M1;
  const float* duvw = ws + G.oDUVW + (long long)i * 3 * G.h0;
  const float* dz2 = ws + G.oDZ2 + (long long)i * (2 * G.F + 1 + G.h0);
  float dlx = ws[G.oDZ3 + (long long)i * (G.F + G.h1) + f] + g.node_deg[i] * dz2[f];
  float dax = dz2[G.F + f];
  const float* mx = m1 + (long long)f * G.h0;
  const float* my = m1 + (long long)(G.F + f) * G.h0;
  const float* mz = m1 + (long long)(2 * G.F + f) * G.h0;
  for (int c = 0; c < G.h0; ++c) {
    dlx += duvw[c] * mx[c] + duvw[G.h0 + c] * my[c];
    dax += duvw[2 * G.h0 + c] * mz[c];
  }
  ws[G.oDLX + idx] = dlx;
  ws[G.oDAX + idx] = dax;
}

// dX = lrelu'(x) (dLX + A^T dAX), A symmetric
__global__ void __launch_bounds__(NT) sg_bwd_x_kernel(snd_sg_graph_t g, Geo G, const float* x,
                                                      int ldx, const float* ws, float* dx, int lddx) {
  const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
  if (idx >= G.R * G.F) return;
  const int i = (int)(idx / G.F), f = (int)(idx - (long long)i * G.F);
  float s = ws[G.oDLX + idx];
  for (int q = g.rowptr[i]; q < g.rowptr[i + 1]; ++q) s += ws[G.oDAX + (long long)g.colidx[q] * G.F + f];
  dx[(long long)i * lddx + f] = s * lrg(x[(long long)i * ldx + f]);
}

unsigned nblk(long long n) { return (unsigned)((n + NT - 1) / NT); }

// C[M, N] (row-major, ldc) = A[M, K] B[K, N]
int mm(const float* A, int lda, int amode, const float* B, int ldb, int bmode, int M, int N, int K,
       float* C, int ldc, hipStream_t s) {
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc;
  a.kchunk = (int)round_up(K > 0 ? K : 1, kGemmBK);
  return launch_gemm(a, amode, bmode, E_STORE, SND_F32, 1, s);
}

// weight gradient dst[m][n] (ld ldd) = sum_r A[r][m] D[r][n], split-K over the R rows
int wg(const Geo& G, float* ws, const float* A, int lda, int M, const float* D, int ldd_in, int N,
       float* dst, int ld_dst, hipStream_t s) {
  GemmArgs a{};
  a.M = M; a.N = N; a.K = (int)G.R; a.A = A; a.lda = lda; a.B = D; a.ldb = ldd_in;
  a.C = ws + G.oSLAB;
  a.kchunk = (int)round_up(cdiv(G.R, G.splits), kGemmBK);
  const int parts = cdiv(G.R, a.kchunk);
  SND_TRY(launch_gemm(a, A_COL, B_ROW, E_PART, SND_F32, parts, s));
  ReduceDesc rd{ws + G.oSLAB, dst, parts, N, (long long)M * N, 1.f, 0, M, N, ld_dst};
  return launch_reduce(&rd, 1, s);
}

// column sums of B [R, N] (ld N) as split-K partials [parts][N] in the slab; returns parts
int colsum(const Geo& G, float* ws, const float* ones, const float* B, int N, hipStream_t s) {
  GemmArgs a{};
  a.M = 1; a.N = N; a.K = (int)G.R; a.A = ones; a.lda = G.ld3; a.B = B; a.ldb = N;
  a.C = ws + G.oSLAB;
  a.kchunk = (int)round_up(cdiv(G.R, G.splits), kGemmBK);
  const int parts = cdiv(G.R, a.kchunk);
  SND_TRY(launch_gemm(a, A_COL, B_ROW, E_PART, SND_F32, parts, s));
  return parts;
}

}  // namespace
}  // namespace snd

using namespace snd;

namespace snd {
namespace {
__global__ void sg_mean_kernel(const float* z, float* zbar, int B, int S, int L) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * L) return;
  const int b = i / L, l = i - b * L;
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += z[((long long)b * S + s) * L + l];
  zbar[i] = acc / (float)S;
}
__global__ void sg_spread_kernel(const float* dzbar, float* dz, int B, int S, int L) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * S * L) return;
  const long long c = i / L;
  dz[i] = dzbar[(c / S) * L + (i - c * L)] / (float)S;
}
}  // namespace

int launch_sg_mean(const float* z, float* zbar, int B, int S, int L, hipStream_t s) {
  hipLaunchKernelGGL(sg_mean_kernel, dim3(cdiv(B * L, 256)), dim3(256), 0, s, z, zbar, B, S, L);
  SND_LAUNCH_CHECK("sg_mean_kernel");
  return 0;
}
int launch_sg_spread(const float* dzbar, float* dz, int B, int S, int L, hipStream_t s) {
  hipLaunchKernelGGL(sg_spread_kernel, dim3(cdiv((long long)B * S * L, 256)), dim3(256), 0, s, dzbar, dz, B,
                     S, L);
  SND_LAUNCH_CHECK("sg_spread_kernel");
  return 0;
}
}  // namespace snd

extern "C" long long snd_sg_param_count(int f, int h0, int h1, int h2) {
  if (f <= 0 || h0 <= 0 || h1 <= 0 || h2 <= 0) return -1;
  return poff(f, h0, h1, h2).total;
}

extern "C" size_t snd_sg_workspace(int n_rows, int f, int h0, int h1, int h2) {
  if (n_rows < 0 || f <= 0 || h0 <= 0 || h1 <= 0 || h2 <= 0) return 0;
  return (size_t)geo(n_rows, f, h0, h1, h2).total * sizeof(float);
}

extern "C" int snd_sg_prep(const snd_sg_graph_t* g, const float* rel, int* n_unmatched,
                           snd_stream_t stream) {
  SND_CHECK_ARG(g && rel && n_unmatched && g->rowptr && g->colidx && g->edge_lr && g->edge_q &&
                    g->edge_rev && g->node_deg && g->node_e,
                "snd_sg_prep: null argument");
  SND_CHECK_ARG(g->n_rows >= 0 && g->n_per_graph > 0 && g->n_rows % g->n_per_graph == 0,
                "snd_sg_prep: n_rows must be B * n_per_graph");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(n_unmatched, 0, sizeof(int), s) != hipSuccess) {
    set_error("snd_sg_prep: memset failed");
    return SND_ERR_HIP;
  }
  if (g->n_rows == 0) return 0;
  hipLaunchKernelGGL(sg_prep_kernel, dim3(nblk(g->n_rows)), dim3(NT), 0, s, *g, rel, n_unmatched);
  SND_LAUNCH_CHECK("sg_prep_kernel");
  return 0;
}

static int sg_args_ok(const snd_sg_graph_t* g, int f, int h0, int h1, int h2) {
  SND_CHECK_ARG(g && g->rowptr && g->colidx && g->edge_lr && g->edge_q && g->edge_rev &&
                    g->node_deg && g->node_e && g->n_rows >= 0,
                "snd_sg_layer: incomplete graph (run snd_sg_prep first)");
  SND_CHECK_ARG(f > 0 && f <= 4096 && h0 > 0 && h1 > 0 && h2 > 0, "snd_sg_layer: bad widths");
  return 0;
}

extern "C" int snd_sg_layer_fwd(const snd_sg_graph_t* g, const float* x, int ldx, int f, int h0,
                                int h1, int h2, const float* params, int bn_act, float* y,
                                float* out, void* workspace, snd_stream_t stream) {
  SND_TRY(sg_args_ok(g, f, h0, h1, h2));
  SND_CHECK_ARG(x && params && y && workspace && ldx >= f, "snd_sg_layer_fwd: null argument");
  SND_CHECK_ARG(!bn_act || out, "snd_sg_layer_fwd: bn_act needs out");
  hipStream_t s = (hipStream_t)stream;
  const Geo G = geo(g->n_rows, f, h0, h1, h2);
  const POff po = poff(f, h0, h1, h2);
  float* ws = (float*)workspace;
  if (G.R == 0) return 0;
  hipLaunchKernelGGL(sg_gather_kernel, dim3(nblk(G.R * f)), dim3(NT), 0, s, *g, x, ldx, G, ws);
  SND_LAUNCH_CHECK("sg_gather_kernel");
  const float* m1 = params + po.M1;
  float* uvw = ws + G.oUVW;
  // u = LX M1x, v = LX M1y, w = (A LX) M1z
  SND_TRY(mm(ws + G.oZ3, G.ld3, A_ROW, m1, h0, B_ROW, (int)G.R, h0, f, uvw, 3 * h0, s));
  SND_TRY(mm(ws + G.oZ3, G.ld3, A_ROW, m1 + (long long)f * h0, h0, B_ROW, (int)G.R, h0, f,
             uvw + h0, 3 * h0, s));
  SND_TRY(mm(ws + G.oZ2 + f, G.ld2, A_ROW, m1 + (long long)2 * f * h0, h0, B_ROW, (int)G.R, h0, f,
             uvw + 2 * h0, 3 * h0, s));
  hipLaunchKernelGGL(sg_edge_fwd_kernel, dim3(nblk(G.R * h0)), dim3(NT), 0, s, *g, G, params, po, ws);
  SND_LAUNCH_CHECK("sg_edge_fwd_kernel");
  // m2 = [d LX | A LX | e | P | d] [M2; b2]
  SND_TRY(mm(ws + G.oZ2, G.ld2, A_ROW, params + po.M2, h1, B_ROW, (int)G.R, h1, G.ld2,
             ws + G.oM2P, h1, s));
  hipLaunchKernelGGL(sg_act_kernel, dim3(nblk(G.R * h1)), dim3(NT), 0, s, G, ws);
  SND_LAUNCH_CHECK("sg_act_kernel");
  // y = [LX | lrelu(m2) | 1] [M3; b3]
  SND_TRY(mm(ws + G.oZ3, G.ld3, A_ROW, params + po.M3, h2, B_ROW, (int)G.R, h2, G.ld3, y, h2, s));
  if (bn_act) {
    hipLaunchKernelGGL(sg_bn_fwd_kernel, dim3(nblk(G.R * h2)), dim3(NT), 0, s, G.R * h2, h2, y,
                       params + po.gamma, params + po.beta, out);
    SND_LAUNCH_CHECK("sg_bn_fwd_kernel");
  }
  return 0;
}

extern "C" int snd_sg_layer_bwd(const snd_sg_graph_t* g, const float* x, int ldx, int f, int h0,
                                int h1, int h2, const float* params, int bn_act, const float* y,
                                const float* dout, float* dx, int lddx, float* grads,
                                void* workspace, snd_stream_t stream) {
  SND_TRY(sg_args_ok(g, f, h0, h1, h2));
  SND_CHECK_ARG(x && params && y && dout && grads && workspace && ldx >= f &&
                    (!dx || lddx >= f),
                "snd_sg_layer_bwd: null argument");
  hipStream_t s = (hipStream_t)stream;
  const Geo G = geo(g->n_rows, f, h0, h1, h2);
  const POff po = poff(f, h0, h1, h2);
  float* ws = (float*)workspace;
  const int R = (int)G.R;
  if (R == 0) return 0;
  const float* dy = dout;
  const float* ones = ws + G.oZ3 + G.F + G.h1;   // Z3e's constant column (ld ld3)
  if (bn_act) {
    hipLaunchKernelGGL(sg_bn_bwd_kernel, dim3(nblk(G.R * h2)), dim3(NT), 0, s, G, y, dout,
                       params + po.gamma, params + po.beta, ws);
    SND_LAUNCH_CHECK("sg_bn_bwd_kernel");
    dy = ws + G.oDY;
    // [dbeta | dgamma] = 1^T [dT | dT y c]
    const int parts = colsum(G, ws, ones, ws + G.oDTY, 2 * h2, s);
    if (parts < 0) return parts;
    ReduceDesc rd[2] = {
        {ws + G.oSLAB, grads + po.beta, parts, h2, 2LL * h2, 1.f, 0, 0, 0, 0},
        {ws + G.oSLAB + h2, grads + po.gamma, parts, h2, 2LL * h2, 1.f, 0, 0, 0, 0}};
    SND_TRY(launch_reduce(rd, 2, s));
  }
  // [dM3; db3] = Z3e^T dy
  SND_TRY(wg(G, ws, ws + G.oZ3, G.ld3, G.ld3, dy, h2, h2, grads + po.M3, h2, s));
  // dZ3 = dy M3^T
  SND_TRY(mm(dy, h2, A_ROW, params + po.M3, h2, B_COL, R, f + h1, h2, ws + G.oDZ3, f + h1, s));
  hipLaunchKernelGGL(sg_act_bwd_kernel, dim3(nblk(G.R * h1)), dim3(NT), 0, s, G, ws);
  SND_LAUNCH_CHECK("sg_act_bwd_kernel");
  // [dM2; db2] = Z2e^T dm2 ; dZ2 = dm2 M2^T
  SND_TRY(wg(G, ws, ws + G.oZ2, G.ld2, G.ld2, ws + G.oDM2, h1, h1, grads + po.M2, h1, s));
  SND_TRY(mm(ws + G.oDM2, h1, A_ROW, params + po.M2, h1, B_COL, R, 2 * f + 1 + h0, h1,
             ws + G.oDZ2, 2 * f + 1 + h0, s));
  hipLaunchKernelGGL(sg_edge_bwd_kernel, dim3(nblk(G.R * h0)), dim3(NT), 0, s, *g, G, params, po, ws);
  SND_LAUNCH_CHECK("sg_edge_bwd_kernel");
  // dM1x = LX^T du, dM1y = LX^T dv, dM1z = (A LX)^T dw
  float* gm1 = grads + po.M1;
  SND_TRY(wg(G, ws, ws + G.oZ3, G.ld3, f, ws + G.oDUVW, 3 * h0, h0, gm1, h0, s));
  SND_TRY(wg(G, ws, ws + G.oZ3, G.ld3, f, ws + G.oDUVW + h0, 3 * h0, h0, gm1 + (long long)f * h0,
             h0, s));
  SND_TRY(wg(G, ws, ws + G.oZ2 + f, G.ld2, f, ws + G.oDUVW + 2 * h0, 3 * h0, h0,
             gm1 + (long long)2 * f * h0, h0, s));
  // scalar rows: dm1r, db1, dm1s, dm1t = column sums of TM
  {
    const int parts = colsum(G, ws, ones, ws + G.oTM, 4 * h0, s);
    if (parts < 0) return parts;
    const long long st = 4LL * h0;
    float* m1row = gm1 + (long long)3 * f * h0;
    ReduceDesc rd[4] = {
        {ws + G.oSLAB, m1row, parts, h0, st, 1.f, 0, 0, 0, 0},
        {ws + G.oSLAB + h0, grads + po.b1, parts, h0, st, 1.f, 0, 0, 0, 0},
        {ws + G.oSLAB + 2 * h0, m1row + h0, parts, h0, st, 1.f, 0, 0, 0, 0},
        {ws + G.oSLAB + 3 * h0, m1row + 2 * h0, parts, h0, st, 1.f, 0, 0, 0, 0}};
    SND_TRY(launch_reduce(rd, 4, s));
  }
  if (dx) {
    hipLaunchKernelGGL(sg_bwd_node_kernel, dim3(nblk(G.R * f)), dim3(NT), 0, s, *g, G, params, po, ws);
    SND_LAUNCH_CHECK("sg_bwd_node_kernel");
    hipLaunchKernelGGL(sg_bwd_x_kernel, dim3(nblk(G.R * f)), dim3(NT), 0, s, *g, G, x, ldx, ws, dx,
                       lddx);
    SND_LAUNCH_CHECK("sg_bwd_x_kernel");
  }
  return 0;
}
