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

__device__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int k = 0; k < RT / 64; ++k) t += sh[k];
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
