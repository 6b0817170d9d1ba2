// The partial-dJ slab a symmetric (J >= I tiles) zz^T would need at C2 (B = 8 graphs,
// N = 4096, d = 64), measured on its own (DESIGN §5 "symmetric tiles, measured").
//
// A J >= I kernel computes each unordered logit block once and feeds both dJ_I += S Z_J
// and dJ_J += S^T Z_I, so every workgroup ends holding partial dJ rows for BOTH its row
// band and its column band.  With S x S super-tiles (S rows of accumulators per side on
// chip) a row of dJ receives N / S partials: S = 512 (the most a CU holds: 2 x 512 x 64
// fp32 = 256 KB of accumulators) gives 8 partials of 256 B per row, 64 MB per C2 step.
// All 256 workgroups (one per CU) finish together, so the partials leave as one burst,
// and a fixed-order reduction reads them back.  This program times both, each alone:
//   burst   256 workgroups x 1024 threads, each writes `per_wg` bytes (float4 stores)
//   reduce  out[r][c] = sum_k part[k][r][c], k < K, fixed order (r < 32768, c < 64)
// for S = 512 (K = 8, 256 KB per workgroup) and S = 256 (K = 16, 128 KB per workgroup,
// 1088 workgroups at 2 per CU -> same bytes per CU pair).
//   hipcc -O3 --offload-arch=gfx950 slab_cost.hip -o slab_cost && ./slab_cost
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(1024) burst(float4* out, long long per_wg_f4) {
  float4* o = out + blockIdx.x * per_wg_f4;
  const float v = (float)threadIdx.x;
  for (long long i = threadIdx.x; i < per_wg_f4; i += 1024) o[i] = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
}

__global__ void __launch_bounds__(256) reduce(const float4* part, float4* out, long long n4, int K) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 s = part[i];
  for (int k = 1; k < K; ++k) {
    const float4 p = part[(long long)k * n4 + i];
    s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
  }
  out[i] = s;
}

static float median(std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main() {
  const long long rows = 8LL * 4096, d = 64;
  const long long n4 = rows * d / 4;
  float4 *part, *out, *flush;
  const size_t maxbytes = 16 * rows * d * 4;                 // K = 16
  CK(hipMalloc(&part, maxbytes));
  CK(hipMalloc(&out, rows * d * 4));
  CK(hipMalloc(&flush, 512ull << 20));                       // evicts the Infinity Cache
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("{\"config\": \"C2: 8 graphs x 4096 rows x 64 fp32\", \"results\": [\n");
  const int Ks[2] = {8, 16};
  for (int t = 0; t < 2; ++t) {
    const int K = Ks[t];
    const int wgs = K == 8 ? 256 : 1088;
    const long long bytes = (long long)K * rows * d * 4;
    const long long per_wg_f4 = bytes / 16 / wgs;
    std::vector<float> tb, tr, trc;
    for (int rep = 0; rep < 12; ++rep) {
      CK(hipMemsetAsync(flush, rep, 512ull << 20, 0));
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(burst, dim3(wgs), dim3(1024), 0, 0, part, per_wg_f4);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tb.push_back(ms * 1000.f);
      // the reduction right after the burst (partials still in the Infinity Cache)
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(reduce, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, part, out, n4, K);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      tr.push_back(ms * 1000.f);
      // and from HBM (cache flushed in between)
      CK(hipMemsetAsync(flush, rep + 1, 512ull << 20, 0));
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(reduce, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, part, out, n4, K);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      trc.push_back(ms * 1000.f);
    }
    printf("  {\"K\": %d, \"workgroups\": %d, \"slab_MB\": %.1f, \"burst_us\": %.2f, \"reduce_cached_us\": %.2f, "
           "\"reduce_cold_us\": %.2f}%s\n", K, wgs, bytes / 1e6, median(tb), median(tr), median(trc), t ? "" : ",");
  }
  printf("]}\n");
  return 0;
}
