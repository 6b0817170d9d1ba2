// Disentangled-model pieces: the e2e edge-to-edge filter of
// the structure decoder and the latent regularisers of the disentangled objectives.
// Neither is on the benchmarked path: the reference runs them at N ~ 25-50 graphs
// and batches of 2-50 latents, so these are plain fp32 kernels with deterministic
// fixed-order sums (no atomics), sized for that regime.
//
// e2e (layers.py:431-450), x [B, N, N, C] NHWC, w1 [K, C, O] (the [1, K, C, O]
// kernel), TF SAME padding for stride 1 (pb = (K - 1) / 2 before):
//   out[b,i,j,o] = 2 b1[o] + sum_t sum_c w1[t,c,o] (x[b, i, j+t-pb, c] + x[b, i+t-pb, j, c])
// (conv1 slides the [1, K] row filter over j; conv2 = conv2d with transpose(w1, [1,0,2,3])
// slides the same taps over i; both add b1).  Backward:
//   dx[b,i,j,c] = sum_t sum_o w1[t,c,o] (dout[b, i, j-t+pb, o] + dout[b, i-t+pb, j, o])
//   dw1[t,c,o]  = sum_{b,i,j} dout[b,i,j,o] (x[b, i, j+t-pb, c] + x[b, i+t-pb, j, c])
//   db1[o]      = 2 sum_{b,i,j} dout[b,i,j,o]
//
// Latent regularisers of one group (optimizer.py:7-58, 159-190), mu / s / z [B, L]:
//   term = w_kl kl  (or cap_gamma relu(kl - cap_c): 'disentangled_C')
//        + w_dip DIP(mu; lambda_od, lambda_d) + w_tc TC(z, mu, s)
// kl = -0.5 mean(1 + 2 s - mu^2 - e^{2s}); DIP on the batch covariance of mu; TC the
// minibatch estimate E_j[log q(z_j) - sum_l log q(z_jl)] with logvar = 2 s.  The
// gradients with respect to mu and s include the path through z = mu + eps e^s
// (model.py:155-159): d mu += dz, d s += dz (z - mu).
#include "snd_common.hpp"

#include <algorithm>
#include <cmath>

namespace snd {
namespace {

constexpr int ET = 256;

__global__ void __launch_bounds__(ET) e2e_fwd_kernel(const float* x, int B, int N, int C, const float* w1,
                                                     const float* b1, int K, int O, float* out) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  const long long total = (long long)B * N * N * O;
  if (idx >= total) return;
  const int o = (int)(idx % O);
  const long long r = idx / O;
  const int j = (int)(r % N), i = (int)((r / N) % N), b = (int)(r / ((long long)N * N));
  const int pb = (K - 1) / 2;
  float acc = 0.f;
  for (int t = 0; t < K; ++t) {
    const int jj = j + t - pb, ii = i + t - pb;
    const float* wt = w1 + (long long)t * C * O + o;
    const bool vj = jj >= 0 && jj < N, vi = ii >= 0 && ii < N;
    const float* xr = x + (((long long)b * N + i) * N + (vj ? jj : 0)) * C;
    const float* xc = x + (((long long)b * N + (vi ? ii : 0)) * N + j) * C;
    for (int c = 0; c < C; ++c) {
      const float v = (vj ? xr[c] : 0.f) + (vi ? xc[c] : 0.f);
      acc = fmaf(v, wt[(long long)c * O], acc);
    }
  }
  out[idx] = acc + 2.f * b1[o];
}

__global__ void __launch_bounds__(ET) e2e_bwd_x_kernel(const float* dout, int B, int N, int C, const float* w1,
                                                       int K, int O, float* dx) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  const long long total = (long long)B * N * N * C;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const long long r = idx / C;
  const int j = (int)(r % N), i = (int)((r / N) % N), b = (int)(r / ((long long)N * N));
  const int pb = (K - 1) / 2;
  float acc = 0.f;
  for (int t = 0; t < K; ++t) {
    const int jj = j - t + pb, ii = i - t + pb;
    const bool vj = jj >= 0 && jj < N, vi = ii >= 0 && ii < N;
    const float* wt = w1 + ((long long)t * C + c) * O;
    const float* dr = dout + (((long long)b * N + i) * N + (vj ? jj : 0)) * O;
    const float* dc = dout + (((long long)b * N + (vi ? ii : 0)) * N + j) * O;
    for (int o = 0; o < O; ++o) {
      const float v = (vj ? dr[o] : 0.f) + (vi ? dc[o] : 0.f);
      acc = fmaf(v, wt[o], acc);
    }
  }
  dx[idx] = acc;
}

// one workgroup per (t, c) pair; thread o-strided over outputs, lanes over (b, i, j)
// with a fixed-order LDS tree: deterministic
__global__ void __launch_bounds__(ET) e2e_bwd_w_kernel(const float* x, const float* dout, int B, int N, int C,
                                                       int K, int O, float* dw1, float* db1) {
  __shared__ float red[ET];
  const int tc = blockIdx.x, t = tc / C, c = tc - t * C;
  const int pb = (K - 1) / 2;
  const long long P = (long long)B * N * N;
  for (int o = 0; o < O; ++o) {
    float acc = 0.f, accb = 0.f;
    for (long long q = threadIdx.x; q < P; q += ET) {
      const int j = (int)(q % N), i = (int)((q / N) % N), b = (int)(q / ((long long)N * N));
      const int jj = j + t - pb, ii = i + t - pb;
      float v = 0.f;
      if (jj >= 0 && jj < N) v += x[(((long long)b * N + i) * N + jj) * C + c];
      if (ii >= 0 && ii < N) v += x[(((long long)b * N + ii) * N + j) * C + c];
      const float d = dout[q * O + o];
      acc = fmaf(v, d, acc);
      accb += d;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int h = ET / 2; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) dw1[((long long)t * C + c) * O + o] = red[0];
    __syncthreads();
    if (tc == 0) {   // db1 from the first workgroup
      red[threadIdx.x] = accb;
      __syncthreads();
      for (int h = ET / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
      }
      if (threadIdx.x == 0) db1[o] = 2.f * red[0];
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- latent regularisers
constexpr int RT = 1024;

template <int NT = RT>
__device__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < NT / 64; ++k) t += sh[k];
  return t;
}

struct RegArgs {
  const float *mu, *s, *z;
  int B, L;
  float w_kl, cap_gamma, cap_c, w_dip, lambda_od, lambda_d, w_tc;
  float* dmu;
  float* ds;
  double* out;   // [kl, term, dip, tc]
  float* ws;     // DIP: L*L G + L mean | TC: B*B S, B*B*L lqp, B*L dz, B*L LSE_i lqp, B LSE_i S
};

__global__ void __launch_bounds__(RT) latent_reg_kernel(RegArgs a) {
  __shared__ double sh[RT / 64];
  const int B = a.B, L = a.L, n = B * L, tid = threadIdx.x;
  const float inv = 1.f / (float)n;
  // ---- KL (optimizer.py:160) and its gradient scale (capacity gate from the value)
  double kp = 0.0;
  for (int e = tid; e < n; e += RT) {
    const double m = a.mu[e], sv = a.s[e];
    kp += 1.0 + 2.0 * sv - m * m - exp(2.0 * sv);
  }
  const double klv = -0.5 * block_sum_d(kp, sh) / (double)n;
  const float wk = a.cap_gamma > 0.f ? (klv > (double)a.cap_c ? a.cap_gamma : 0.f) : a.w_kl;
  const double kterm = a.cap_gamma > 0.f ? (double)a.cap_gamma * fmax(klv - (double)a.cap_c, 0.0)
                                         : (double)a.w_kl * klv;
  for (int e = tid; e < n; e += RT) {
    const float m = a.mu[e], sv = a.s[e];
    a.dmu[e] = wk * m * inv;
    a.ds[e] = wk * (expf(2.f * sv) - 1.f) * inv;
  }
  __syncthreads();
  // ---- DIP (optimizer.py:7-21): cov = E[mu mu^T] - m m^T, G = d reg / d cov
  double dipv = 0.0;
  if (a.w_dip != 0.f) {
    float* cov = a.ws;
    float* mean = a.ws + (long long)L * L;
    for (int l = tid; l < L; l += RT) {
      float t = 0.f;
      for (int b = 0; b < B; ++b) t += a.mu[(long long)b * L + l];
      mean[l] = t / (float)B;
    }
    __syncthreads();
    double rp = 0.0;
    for (int e = tid; e < L * L; e += RT) {
      const int k = e / L, l = e - k * L;
      float t = 0.f;
      for (int b = 0; b < B; ++b) t += a.mu[(long long)b * L + k] * a.mu[(long long)b * L + l];
      const float cv = t / (float)B - mean[k] * mean[l];
      double r;
      float g;
      if (k == l) { r = (double)a.lambda_d * ((double)cv - 1.0) * ((double)cv - 1.0); g = 2.f * a.lambda_d * (cv - 1.f); }
      else { r = (double)a.lambda_od * (double)cv * (double)cv; g = 2.f * a.lambda_od * cv; }
      rp += r;
      cov[e] = g;   // G (symmetric)
    }
    dipv = block_sum_d(rp, sh);
    __syncthreads();
    // d mu_b = (2 / B) G (mu_b - m)
    for (int e = tid; e < n; e += RT) {
      const int b = e / L, k = e - b * L;
      float t = 0.f;
      for (int l = 0; l < L; ++l) t += cov[(long long)k * L + l] * (a.mu[(long long)b * L + l] - mean[l]);
      a.dmu[e] += a.w_dip * 2.f * t / (float)B;
    }
    __syncthreads();
  }
  // ---- total correlation (optimizer.py:23-58), logvar = 2 s
  double tcv = 0.0;
  if (a.w_tc != 0.f) {
    const float kLog2Pi = 1.8378770664093453f;
    float* S = a.ws;                          // [j][i] sum_l lqp
    float* Q = a.ws + (long long)B * B;       // [j][i][l] lqp
    float* dz = Q + (long long)B * B * L;     // [j][l]
    for (long long e = tid; e < (long long)B * B * L; e += RT) {
      const int l = (int)(e % L);
      const long long ji = e / L;
      const int i = (int)(ji % B), j = (int)(ji / B);
      const float tmp = a.z[(long long)j * L + l] - a.mu[(long long)i * L + l];
      const float sv = a.s[(long long)i * L + l];
      Q[e] = -0.5f * (tmp * tmp * expf(-2.f * sv) + 2.f * sv + kLog2Pi);
    }
    __syncthreads();
    for (int e = tid; e < B * B; e += RT) {
      float t = 0.f;
      for (int l = 0; l < L; ++l) t += Q[(long long)e * L + l];
      S[e] = t;
    }
    __syncthreads();
    // per j: log_qz = LSE_i S[j,i]; per (j, l): P = LSE_i Q[j,i,l]; W = (softmax_i S - softmax_i Q) / B
    float* PL = dz + (long long)B * L;        // [j][l] LSE_i Q
    float* SL = PL + (long long)B * L;        // [j]    LSE_i S
    for (int j = tid; j < B; j += RT) {
      float ms = -INFINITY;
      for (int i = 0; i < B; ++i) ms = fmaxf(ms, S[(long long)j * B + i]);
      float ss = 0.f;
      for (int i = 0; i < B; ++i) ss += expf(S[(long long)j * B + i] - ms);
      SL[j] = ms + logf(ss);
    }
    for (int e = tid; e < B * L; e += RT) {
      const int j = e / L, l = e - j * L;
      float mx = -INFINITY;
      for (int i = 0; i < B; ++i) mx = fmaxf(mx, Q[((long long)j * B + i) * L + l]);
      float sq = 0.f;
      for (int i = 0; i < B; ++i) sq += expf(Q[((long long)j * B + i) * L + l] - mx);
      PL[e] = mx + logf(sq);
    }
    __syncthreads();
    double tp = 0.0;
    for (int j = tid; j < B; j += RT) tp += (double)SL[j];
    for (int e = tid; e < B * L; e += RT) tp -= (double)PL[e];
    tcv = block_sum_d(tp, sh) / (double)B;
    auto wgt = [&](int j, int i, int l) {
      return (expf(S[(long long)j * B + i] - SL[j]) - expf(Q[((long long)j * B + i) * L + l] - PL[(long long)j * L + l])) /
             (float)B;
    };
    for (int e = tid; e < B * L; e += RT) {   // (j, l): dz through the densities of sample j
      const int j = e / L, l = e - j * L;
      const float zj = a.z[e];
      float dzv = 0.f;
      for (int i = 0; i < B; ++i)
        dzv -= wgt(j, i, l) * (zj - a.mu[(long long)i * L + l]) * expf(-2.f * a.s[(long long)i * L + l]);
      dz[e] = dzv;
    }
    __syncthreads();
    for (int e = tid; e < B * L; e += RT) {   // (i, l): d mu, d s through the densities
      const int i = e / L, l = e - i * L;
      const float mi = a.mu[e], sv = a.s[e], iv = expf(-2.f * sv);
      float dm = 0.f, dsv = 0.f;
      for (int j = 0; j < B; ++j) {
        const float w = wgt(j, i, l);
        const float tmp = a.z[(long long)j * L + l] - mi;
        dm += w * tmp * iv;
        dsv += w * (tmp * tmp * iv - 1.f);
      }
      // through z_i = mu_i + eps_i e^{s_i}: d mu += dz, d s += dz (z - mu)
      const float dzi = dz[e];
      a.dmu[e] += a.w_tc * (dm + dzi);
      a.ds[e] += a.w_tc * (dsv + dzi * (a.z[e] - mi));
    }
  }
  if (tid == 0) {
    a.out[0] = klv;
    a.out[1] = kterm + (double)a.w_dip * dipv + (double)a.w_tc * tcv;
    a.out[2] = dipv;
    a.out[3] = tcv;
  }
}

// ---------------------------------------------------------------- e2e structure decoder
// model.py:193-208 around the e2e filters, [B, N, N, *] NHWC fp32, frozen Keras BN
// y' = gamma c y + beta (c = 1/sqrt(1.001)) followed by relu:
//   pair:  x0[b,i,j,c] = relu(BN0([z_i | z_j])[c])        (model.py:193-195, loop head)
//   layer: x = relu(BN(y))                                (model.py:197-198)
//   head:  logits = relu(BN_adj(y)) W + b (d_e_lin2), the diagonal set to (1, 0)
//          (model.py:200-203); CE against [1 - A, A] (optimizer.py:142-144), mean over B N^2
__global__ void __launch_bounds__(ET) pair_bn_relu_kernel(const float* z, int B, int N, int D, const float* g,
                                                          const float* be, float* x) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  const int C2 = 2 * D;
  if (idx >= (long long)B * N * N * C2) return;
  const int c = (int)(idx % C2);
  const long long r = idx / C2;
  const int j = (int)(r % N), i = (int)((r / N) % N), b = (int)(r / ((long long)N * N));
  const float v = c < D ? z[((long long)b * N + i) * D + c] : z[((long long)b * N + j) * D + c - D];
  x[idx] = fmaxf(g[c] * kBnC * v + be[c], 0.f);
}

__global__ void __launch_bounds__(ET) bn_relu_kernel(const float* y, long long rows, int C, const float* g,
                                                     const float* be, float* x) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  if (idx >= rows * C) return;
  const int c = (int)(idx % C);
  x[idx] = fmaxf(g[c] * kBnC * y[idx] + be[c], 0.f);
}

// d (relu(BN(y))) -> dy, and per channel dgamma = sum dt c y, dbeta = sum dt: one
// workgroup per channel, fixed-order tree
__global__ void __launch_bounds__(ET) bn_relu_bwd_kernel(const float* dx, const float* y, long long rows, int C,
                                                         const float* g, const float* be, float* dy, float* dg,
                                                         float* db) {
  __shared__ float r1[ET], r2[ET];
  const int c = blockIdx.x;
  float sg = 0.f, sb = 0.f;
  for (long long r = threadIdx.x; r < rows; r += ET) {
    const long long e = r * C + c;
    const float t = g[c] * kBnC * y[e] + be[c];
    const float dt = t > 0.f ? dx[e] : 0.f;
    dy[e] = dt * g[c] * kBnC;
    sg = fmaf(dt, kBnC * y[e], sg);
    sb += dt;
  }
  r1[threadIdx.x] = sg;
  r2[threadIdx.x] = sb;
  __syncthreads();
  for (int h = ET / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) { r1[threadIdx.x] += r1[threadIdx.x + h]; r2[threadIdx.x] += r2[threadIdx.x + h]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { dg[c] = r1[0]; db[c] = r2[0]; }
}

// pair stage backward: one workgroup per (b, channel c of z's 2D): dgamma/dbeta partial
// over the graph's N^2 pairs and dz (row part: sum over j; column part: sum over i)
__global__ void __launch_bounds__(ET) pair_bwd_kernel(const float* dx0, const float* z, int B, int N, int D,
                                                      const float* g, const float* be, float* dz, float* pg,
                                                      float* pb) {
  __shared__ float r1[ET], r2[ET];
  const int C2 = 2 * D;
  const int b = blockIdx.x / C2, c = blockIdx.x - b * C2;
  const int d = c < D ? c : c - D;
  float sg = 0.f, sb = 0.f;
  // dz[b, n, d] (this channel's half): thread n-strided, sum over the partner index
  for (int n = threadIdx.x; n < N; n += ET) {
    float acc = 0.f;
    const float v = z[((long long)b * N + n) * D + d];
    const float t = g[c] * kBnC * v + be[c];
    for (int m = 0; m < N; ++m) {
      const long long e = c < D ? ((((long long)b * N + n) * N + m) * C2 + c) : ((((long long)b * N + m) * N + n) * C2 + c);
      const float dt = t > 0.f ? dx0[e] : 0.f;
      acc += dt;
    }
    // every pair holding z[b, n, d] in channel c has the same pre-activation t
    const float dzc = acc * g[c] * kBnC;
    sg = fmaf(acc, kBnC * v, sg);
    sb += acc;
    if (c < D) dz[((long long)b * N + n) * D + d] = dzc;
    else pg[(long long)B * C2 * 2 + ((long long)b * N + n) * D + d] = dzc;   // column half, added below
  }
  r1[threadIdx.x] = sg;
  r2[threadIdx.x] = sb;
  __syncthreads();
  for (int h = ET / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) { r1[threadIdx.x] += r1[threadIdx.x + h]; r2[threadIdx.x] += r2[threadIdx.x + h]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) { pg[(long long)b * C2 + c] = r1[0]; pb[(long long)b * C2 + c] = r2[0]; }
}

// dz += column halves; dgamma0 / dbeta0 = sum over graphs (fixed order)
__global__ void __launch_bounds__(ET) pair_bwd_finish_kernel(float* dz, int B, int N, int D, const float* pg,
                                                             const float* pb, float* dg, float* db) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  const int C2 = 2 * D;
  if (idx < (long long)B * N * D) dz[idx] += pg[(long long)B * C2 * 2 + idx];
  if (idx < C2) {
    float sg = 0.f, sb = 0.f;
    for (int b = 0; b < B; ++b) { sg += pg[(long long)b * C2 + idx]; sb += pb[(long long)b * C2 + idx]; }
    dg[idx] = sg;
    db[idx] = sb;
  }
}

// head: one workgroup walks every (b, i, j); out: [0] CE sum (double), [1] correct
// count; dy [rows, C] and the reduced grads dW [C][2], db [2], dgamma [C], dbeta [C]
constexpr int HC = 32;   // head input channels at most
constexpr int HT = 256;   // head threads (32-channel register arrays per thread)
__global__ void __launch_bounds__(HT) e2e_head_kernel(const float* y, const float* adj, int B, int N, int C,
                                                      const float* g, const float* be, const float* W,
                                                      const float* bl, float* dy, float* dW, float* dbl,
                                                      float* dg, float* dbe, double* out) {
  __shared__ double sh[HT / 64];
  const long long rows = (long long)B * N * N;
  const float invM = 1.f / (float)rows;
  float aW[HC][2], aG[HC], aB[HC], ab0 = 0.f, ab1 = 0.f;
#pragma unroll
  for (int k = 0; k < HC; ++k) { aW[k][0] = aW[k][1] = aG[k] = aB[k] = 0.f; }
  double ce = 0.0, cnt = 0.0;
  for (long long e = threadIdx.x; e < rows; e += HT) {
    const int j = (int)(e % N), i = (int)((e / N) % N);
    const float A = adj[e];
    float x[HC], t[HC];
    float l0 = bl[0], l1 = bl[1];
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      if (k < C) {
        t[k] = g[k] * kBnC * y[e * C + k] + be[k];
        x[k] = fmaxf(t[k], 0.f);
        l0 = fmaf(x[k], W[2 * k], l0);
        l1 = fmaf(x[k], W[2 * k + 1], l1);
      }
    }
    const bool dg_ = i == j;
    if (dg_) { l0 = 1.f; l1 = 0.f; }
    const float mx = fmaxf(l0, l1);
    const float lse = mx + logf(expf(l0 - mx) + expf(l1 - mx));
    ce += (double)(lse - (1.f - A) * l0 - A * l1);
    cnt += (double)(((l1 > l0) ? 1.f : 0.f) == A);
    const float p1 = expf(l1 - lse), p0 = expf(l0 - lse);
    const float d0 = dg_ ? 0.f : (p0 - (1.f - A)) * invM, d1 = dg_ ? 0.f : (p1 - A) * invM;
    ab0 += d0;
    ab1 += d1;
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      if (k < C) {
        aW[k][0] = fmaf(x[k], d0, aW[k][0]);
        aW[k][1] = fmaf(x[k], d1, aW[k][1]);
        const float dx = d0 * W[2 * k] + d1 * W[2 * k + 1];
        const float dt = t[k] > 0.f ? dx : 0.f;
        dy[e * C + k] = dt * g[k] * kBnC;
        aG[k] = fmaf(dt, kBnC * y[e * C + k], aG[k]);
        aB[k] += dt;
      }
    }
  }
  const double ces = block_sum_d<HT>(ce, sh), cnts = block_sum_d<HT>(cnt, sh);
#pragma unroll
  for (int k = 0; k < HC; ++k) {
    if (k < C) {   // uniform
      const double w0 = block_sum_d<HT>(aW[k][0], sh), w1 = block_sum_d<HT>(aW[k][1], sh);
      const double gg = block_sum_d<HT>(aG[k], sh), bb = block_sum_d<HT>(aB[k], sh);
      if (threadIdx.x == 0) { dW[2 * k] = (float)w0; dW[2 * k + 1] = (float)w1; dg[k] = (float)gg; dbe[k] = (float)bb; }
    }
  }
  const double s0 = block_sum_d<HT>(ab0, sh), s1 = block_sum_d<HT>(ab1, sh);
  if (threadIdx.x == 0) { dbl[0] = (float)s0; dbl[1] = (float)s1; out[0] = ces; out[1] = cnts; }
}

}  // namespace
}  // namespace snd

using namespace snd;

extern "C" int snd_e2e_fwd(const float* x, int n_graphs, int n, int c, const float* w1, const float* b1, int k,
                           int o, float* out, snd_stream_t stream) {
  SND_CHECK_ARG(x && w1 && b1 && out, "snd_e2e_fwd: null operand");
  SND_CHECK_ARG(n_graphs > 0 && n > 0 && c > 0 && k > 0 && o > 0, "snd_e2e_fwd: empty shape");
  const long long total = (long long)n_graphs * n * n * o;
  hipLaunchKernelGGL(e2e_fwd_kernel, dim3((unsigned)((total + ET - 1) / ET)), dim3(ET), 0, (hipStream_t)stream,
                     x, n_graphs, n, c, w1, b1, k, o, out);
  SND_LAUNCH_CHECK("e2e_fwd_kernel");
  return 0;
}

extern "C" int snd_e2e_bwd(const float* x, int n_graphs, int n, int c, const float* w1, int k, int o,
                           const float* dout, float* dx, float* dw1, float* db1, snd_stream_t stream) {
  SND_CHECK_ARG(x && w1 && dout && dx && dw1 && db1, "snd_e2e_bwd: null operand");
  SND_CHECK_ARG(n_graphs > 0 && n > 0 && c > 0 && k > 0 && o > 0, "snd_e2e_bwd: empty shape");
  const long long total = (long long)n_graphs * n * n * c;
  hipLaunchKernelGGL(e2e_bwd_x_kernel, dim3((unsigned)((total + ET - 1) / ET)), dim3(ET), 0, (hipStream_t)stream,
                     dout, n_graphs, n, c, w1, k, o, dx);
  SND_LAUNCH_CHECK("e2e_bwd_x_kernel");
  hipLaunchKernelGGL(e2e_bwd_w_kernel, dim3((unsigned)(k * c)), dim3(ET), 0, (hipStream_t)stream,
                     x, dout, n_graphs, n, c, k, o, dw1, db1);
  SND_LAUNCH_CHECK("e2e_bwd_w_kernel");
  return 0;
}

extern "C" size_t snd_latent_reg_workspace(int batch, int latent) {
  const size_t dipf = (size_t)latent * latent + latent;
  const size_t tcf = (size_t)batch * batch + (size_t)batch * batch * latent + 2 * (size_t)batch * latent + batch;
  return 4 * (dipf > tcf ? dipf : tcf);
}

extern "C" int snd_latent_reg(const float* mu, const float* logstd, const float* z, int batch, int latent,
                              const snd_latent_reg_t* w, float* dmu, float* dlogstd, double* out, void* workspace,
                              snd_stream_t stream) {
  SND_CHECK_ARG(mu && logstd && w && dmu && dlogstd && out, "snd_latent_reg: null operand");
  SND_CHECK_ARG(batch > 0 && latent > 0, "snd_latent_reg: empty shape");
  SND_CHECK_ARG((w->w_dip == 0.f && w->w_tc == 0.f) || workspace, "snd_latent_reg: DIP / TC need the workspace");
  SND_CHECK_ARG(w->w_tc == 0.f || z, "snd_latent_reg: TC needs z");
  RegArgs a{mu, logstd, z, batch, latent, w->w_kl, w->cap_gamma, w->cap_c, w->w_dip, w->lambda_od,
            w->lambda_d, w->w_tc, dmu, dlogstd, out, (float*)workspace};
  hipLaunchKernelGGL(latent_reg_kernel, dim3(1), dim3(RT), 0, (hipStream_t)stream, a);
  SND_LAUNCH_CHECK("latent_reg_kernel");
  return 0;
}

extern "C" int snd_e2e_pair_fwd(const float* z, int n_graphs, int n, int d, const float* gamma, const float* beta,
                                float* x, snd_stream_t stream) {
  SND_CHECK_ARG(z && gamma && beta && x && n_graphs > 0 && n > 0 && d > 0, "snd_e2e_pair_fwd: bad arguments");
  const long long total = (long long)n_graphs * n * n * 2 * d;
  hipLaunchKernelGGL(pair_bn_relu_kernel, dim3((unsigned)((total + ET - 1) / ET)), dim3(ET), 0, (hipStream_t)stream,
                     z, n_graphs, n, d, gamma, beta, x);
  SND_LAUNCH_CHECK("pair_bn_relu_kernel");
  return 0;
}

extern "C" size_t snd_e2e_pair_bwd_workspace(int n_graphs, int n, int d) {
  return 4 * ((size_t)n_graphs * 2 * d * 2 + (size_t)n_graphs * n * d);
}

extern "C" int snd_e2e_pair_bwd(const float* dx0, const float* z, int n_graphs, int n, int d, const float* gamma,
                                const float* beta, float* dz, float* dgamma, float* dbeta, void* workspace,
                                snd_stream_t stream) {
  SND_CHECK_ARG(dx0 && z && gamma && beta && dz && dgamma && dbeta && workspace && n_graphs > 0 && n > 0 && d > 0,
                "snd_e2e_pair_bwd: bad arguments");
  float* pg = (float*)workspace;
  float* pb = pg + (long long)n_graphs * 2 * d;
  hipLaunchKernelGGL(pair_bwd_kernel, dim3((unsigned)(n_graphs * 2 * d)), dim3(ET), 0, (hipStream_t)stream,
                     dx0, z, n_graphs, n, d, gamma, beta, dz, pg, pb);
  SND_LAUNCH_CHECK("pair_bwd_kernel");
  const long long cnt = std::max<long long>((long long)n_graphs * n * d, 2LL * d);
  hipLaunchKernelGGL(pair_bwd_finish_kernel, dim3((unsigned)((cnt + ET - 1) / ET)), dim3(ET), 0, (hipStream_t)stream,
                     dz, n_graphs, n, d, pg, pb, dgamma, dbeta);
  SND_LAUNCH_CHECK("pair_bwd_finish_kernel");
  return 0;
}

extern "C" int snd_bn_relu_fwd(const float* y, long long rows, int c, const float* gamma, const float* beta, float* x,
                               snd_stream_t stream) {
  SND_CHECK_ARG(y && gamma && beta && x && rows > 0 && c > 0, "snd_bn_relu_fwd: bad arguments");
  hipLaunchKernelGGL(bn_relu_kernel, dim3((unsigned)((rows * c + ET - 1) / ET)), dim3(ET), 0, (hipStream_t)stream,
                     y, rows, c, gamma, beta, x);
  SND_LAUNCH_CHECK("bn_relu_kernel");
  return 0;
}

extern "C" int snd_bn_relu_bwd(const float* dx, const float* y, long long rows, int c, const float* gamma,
                               const float* beta, float* dy, float* dgamma, float* dbeta, snd_stream_t stream) {
  SND_CHECK_ARG(dx && y && gamma && beta && dy && dgamma && dbeta && rows > 0 && c > 0, "snd_bn_relu_bwd: bad arguments");
  hipLaunchKernelGGL(bn_relu_bwd_kernel, dim3((unsigned)c), dim3(ET), 0, (hipStream_t)stream, dx, y, rows, c, gamma,
                     beta, dy, dgamma, dbeta);
  SND_LAUNCH_CHECK("bn_relu_bwd_kernel");
  return 0;
}

extern "C" int snd_e2e_head_ce(const float* y, const float* adj, int n_graphs, int n, int c, const float* gamma,
                               const float* beta, const float* w, const float* b, float* dy, float* dw, float* db,
                               float* dgamma, float* dbeta, double* out, snd_stream_t stream) {
  SND_CHECK_ARG(y && adj && gamma && beta && w && b && dy && dw && db && dgamma && dbeta && out,
                "snd_e2e_head_ce: null operand");
  SND_CHECK_ARG(n_graphs > 0 && n > 0 && c > 0 && c <= HC, "snd_e2e_head_ce: channels must be in [1, %d]", HC);
  hipLaunchKernelGGL(e2e_head_kernel, dim3(1), dim3(HT), 0, (hipStream_t)stream, y, adj, n_graphs, n, c, gamma,
                     beta, w, b, dy, dw, db, dgamma, dbeta, out);
  SND_LAUNCH_CHECK("e2e_head_kernel");
  return 0;
}

// ---- frozen Keras BN with an activation, either order (ABI 12) -----------------------
namespace snd {
namespace {
__device__ __forceinline__ float act_f(float v, int act) {
  return act == 1 ? fmaxf(v, 0.f) : (act == 2 ? fmaxf(v, kLeak * v) : v);
}
// d act / d v as TF routes it: relu' = 1 for v > 0; Maximum(v, 0.2 v)' = 1 for v >= 0
__device__ __forceinline__ float act_d(float v, int act) {
  return act == 1 ? (v > 0.f ? 1.f : 0.f) : (act == 2 ? (v >= 0.f ? 1.f : kLeak) : 1.f);
}
__global__ void __launch_bounds__(ET) bn_act_kernel(const float* y, int ldy, long long rows, int C,
                                                    const float* g, const float* be, int act, int pre,
                                                    float* x, int ldx) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  if (idx >= rows * C) return;
  const int c = (int)(idx % C);
  const long long r = idx / C;
  const float v = y[r * ldy + c];
  x[r * ldx + c] = pre ? g[c] * kBnC * act_f(v, act) + be[c] : act_f(g[c] * kBnC * v + be[c], act);
}
// one workgroup per channel, fixed-order tree: dy, dgamma = sum du c t, dbeta = sum du
__global__ void __launch_bounds__(ET) bn_act_bwd_kernel(const float* dx, int lddx, const float* y, int ldy,
                                                        long long rows, int C, const float* g, const float* be,
                                                        int act, int pre, float* dy, int lddy, float* dg,
                                                        float* db) {
  __shared__ float r1[ET], r2[ET];
  const int c = blockIdx.x;
  const float gc = g[c] * kBnC;
  float sg = 0.f, sb = 0.f;
  for (long long r = threadIdx.x; r < rows; r += ET) {
    const float v = y[r * ldy + c];
    float du, t;
    if (pre) {   // x = BN(act(y))
      t = act_f(v, act);
      du = dx[r * lddx + c];
      dy[r * lddy + c] = du * gc * act_d(v, act);
    } else {     // x = act(BN(y))
      t = v;
      du = dx[r * lddx + c] * act_d(gc * v + be[c], act);
      dy[r * lddy + c] = du * gc;
    }
    sg = fmaf(du, kBnC * t, sg);
    sb += du;
  }
  r1[threadIdx.x] = sg;
  r2[threadIdx.x] = sb;
  __syncthreads();
  for (int h = ET / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) { r1[threadIdx.x] += r1[threadIdx.x + h]; r2[threadIdx.x] += r2[threadIdx.x + h]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (dg) dg[c] = r1[0];
    if (db) db[c] = r2[0];
  }
}
// z = mu + eps e^s backward: dmu = dz + add_mu, ds = dz eps e^s + add_s (model.py:155-159)
__global__ void __launch_bounds__(ET) reparam_bwd_plain_kernel(const float* ms, int ldms, long long rows, int L,
                                                               const float* eps, const float* dz,
                                                               const float* add_mu, const float* add_s,
                                                               float* dms, int lddms) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  if (idx >= rows * L) return;
  const long long r = idx / L;
  const int l = (int)(idx - r * L);
  const float s = ms[r * ldms + L + l];
  const float d = dz ? dz[idx] : 0.f;
  dms[r * lddms + l] = d + (add_mu ? add_mu[idx] : 0.f);
  dms[r * lddms + L + l] = d * eps[idx] * expf(s) + (add_s ? add_s[idx] : 0.f);
}
}  // namespace
}  // namespace snd

extern "C" int snd_bn_act_fwd(const float* y, int ldy, long long rows, int c, const float* gamma,
                              const float* beta, int act, int act_first, float* x, int ldx, snd_stream_t stream) {
  SND_CHECK_ARG(y && gamma && beta && x && rows >= 0 && c > 0 && ldy >= c && ldx >= c && act >= 0 && act <= 2,
                "snd_bn_act_fwd: bad arguments");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(bn_act_kernel, dim3((unsigned)((rows * c + ET - 1) / ET)), dim3(ET), 0, (hipStream_t)stream,
                     y, ldy, rows, c, gamma, beta, act, act_first, x, ldx);
  SND_LAUNCH_CHECK("bn_act_kernel");
  return 0;
}

extern "C" int snd_bn_act_bwd(const float* dx, int lddx, const float* y, int ldy, long long rows, int c,
                              const float* gamma, const float* beta, int act, int act_first, float* dy, int lddy,
                              float* dgamma, float* dbeta, snd_stream_t stream) {
  SND_CHECK_ARG(dx && y && gamma && beta && dy && rows >= 0 && c > 0 && lddx >= c && ldy >= c && lddy >= c &&
                    act >= 0 && act <= 2,
                "snd_bn_act_bwd: bad arguments");
  hipLaunchKernelGGL(bn_act_bwd_kernel, dim3((unsigned)c), dim3(ET), 0, (hipStream_t)stream, dx, lddx, y, ldy, rows,
                     c, gamma, beta, act, act_first, dy, lddy, dgamma, dbeta);
  SND_LAUNCH_CHECK("bn_act_bwd_kernel");
  return 0;
}

extern "C" int snd_reparam_bwd(const float* ms, int ldms, int rows, int latent, const float* eps, const float* dz,
                               const float* add_mu, const float* add_logstd, float* dms, int lddms,
                               snd_stream_t stream) {
  SND_CHECK_ARG(ms && eps && dms && rows >= 0 && latent > 0 && ldms >= 2 * latent && lddms >= 2 * latent,
                "snd_reparam_bwd: bad arguments");
  const long long n = (long long)rows * latent;
  if (n == 0) return 0;
  hipLaunchKernelGGL(reparam_bwd_plain_kernel, dim3((unsigned)((n + ET - 1) / ET)), dim3(ET), 0,
                     (hipStream_t)stream, ms, ldms, (long long)rows, latent, eps, dz, add_mu, add_logstd, dms, lddms);
  SND_LAUNCH_CHECK("reparam_bwd_plain_kernel");
  return 0;
}

namespace snd {
namespace {
__global__ void __launch_bounds__(ET) add_strided_kernel(long long rows, int cols, float alpha, const float* x,
                                                         int ldx, float* y, int ldy) {
  const long long idx = (long long)blockIdx.x * ET + threadIdx.x;
  if (idx >= rows * cols) return;
  const long long r = idx / cols;
  const int c = (int)(idx - r * cols);
  y[r * ldy + c] += alpha * x[r * ldx + c];
}
}  // namespace
}  // namespace snd

extern "C" int snd_add_strided(long long rows, int cols, float alpha, const float* x, int ldx, float* y, int ldy,
                               snd_stream_t stream) {
  SND_CHECK_ARG(x && y && rows >= 0 && cols > 0 && ldx >= cols && ldy >= cols, "snd_add_strided: bad arguments");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(add_strided_kernel, dim3((unsigned)((rows * cols + ET - 1) / ET)), dim3(ET), 0,
                     (hipStream_t)stream, rows, cols, alpha, x, ldx, y, ldy);
  SND_LAUNCH_CHECK("add_strided_kernel");
  return 0;
}
