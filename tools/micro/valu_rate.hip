// Microbenchmark: VALU / transcendental / MFMA issue rates per SIMD on gfx950 as a
// function of waves per SIMD.  Every workgroup = W waves on ONE CU (1 workgroup
// per CU via LDS), 256 workgroups.  Reports ns per instruction per SIMD.
//   hipcc -O3 --offload-arch=gfx950 valu_rate.hip -o valu_rate && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int KIND>
__global__ void kern(float* out, int iters) {
  __shared__ float pad[40000];   // one workgroup per CU
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  f32x16 acc = {};
  bf16x8 av, bv;
  for (int e = 0; e < 8; ++e) { av[e] = (__bf16)(a0 + e); bv[e] = (__bf16)(a1 - e); }
  for (int i = 0; i < iters; ++i) {
    if constexpr (KIND == 0) {   // 8 independent fma chains
      a0 = __builtin_fmaf(a0, 1.0001f, 0.5f); a1 = __builtin_fmaf(a1, 1.0001f, 0.5f);
      a2 = __builtin_fmaf(a2, 1.0001f, 0.5f); a3 = __builtin_fmaf(a3, 1.0001f, 0.5f);
      a4 = __builtin_fmaf(a4, 1.0001f, 0.5f); a5 = __builtin_fmaf(a5, 1.0001f, 0.5f);
      a6 = __builtin_fmaf(a6, 1.0001f, 0.5f); a7 = __builtin_fmaf(a7, 1.0001f, 0.5f);
    } else if constexpr (KIND == 1) {   // 8 independent exp2
      a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_amdgcn_exp2f(a1);
      a2 = __builtin_amdgcn_exp2f(a2); a3 = __builtin_amdgcn_exp2f(a3);
      a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_amdgcn_exp2f(a5);
      a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_amdgcn_exp2f(a7);
    } else if constexpr (KIND == 2) {   // 4 exp2 + 4 fma
      a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_fmaf(a1, 1.0001f, 0.5f);
      a2 = __builtin_amdgcn_exp2f(a2); a3 = __builtin_fmaf(a3, 1.0001f, 0.5f);
      a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_fmaf(a5, 1.0001f, 0.5f);
      a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_fmaf(a7, 1.0001f, 0.5f);
    } else if constexpr (KIND == 3) {   // 1 MFMA 32x32x16 only
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    } else if constexpr (KIND == 4) {   // 1 MFMA + 8 exp2
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
      a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_amdgcn_exp2f(a1);
      a2 = __builtin_amdgcn_exp2f(a2); a3 = __builtin_amdgcn_exp2f(a3);
      a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_amdgcn_exp2f(a5);
      a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_amdgcn_exp2f(a7);
    } else if constexpr (KIND == 5) {   // 1 MFMA + 8 fma
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
      a0 = __builtin_fmaf(a0, 1.0001f, 0.5f); a1 = __builtin_fmaf(a1, 1.0001f, 0.5f);
      a2 = __builtin_fmaf(a2, 1.0001f, 0.5f); a3 = __builtin_fmaf(a3, 1.0001f, 0.5f);
      a4 = __builtin_fmaf(a4, 1.0001f, 0.5f); a5 = __builtin_fmaf(a5, 1.0001f, 0.5f);
      a6 = __builtin_fmaf(a6, 1.0001f, 0.5f); a7 = __builtin_fmaf(a7, 1.0001f, 0.5f);
    } else if constexpr (KIND == 6) {   // 8 v_cmp + ballot popcount (SALU)
      unsigned c = 0;
      c += __popcll(__ballot(a0 > 0.5f)); c += __popcll(__ballot(a1 > 0.5f));
      c += __popcll(__ballot(a2 > 0.5f)); c += __popcll(__ballot(a3 > 0.5f));
      c += __popcll(__ballot(a4 > 0.5f)); c += __popcll(__ballot(a5 > 0.5f));
      c += __popcll(__ballot(a6 > 0.5f)); c += __popcll(__ballot(a7 > 0.5f));
      a0 += (float)c;
    } else if constexpr (KIND == 8) {   // 8 v_dot2_f32_bf16 (accumulating)
      typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
      bf2 x = {av[0], av[1]}, one = {(__bf16)1.f, (__bf16)0.f};
      a0 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a0, false);
      a1 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a1, false);
      a2 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a2, false);
      a3 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a3, false);
      a4 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a4, false);
      a5 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a5, false);
      a6 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a6, false);
      a7 = __builtin_amdgcn_fdot2_f32_bf16(x, one, a7, false);
      av[0] = (__bf16)a7;
    } else if constexpr (KIND == 9) {   // 8 v_pk_add_f32 (2 floats each)
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, k = {0.5f, 0.25f};
      for (int u = 0; u < 2; ++u) { p0 += k; p1 += k; p2 += k; p3 += k; }
      a0 = p0[0]; a1 = p0[1]; a2 = p1[0]; a3 = p1[1]; a4 = p2[0]; a5 = p2[1]; a6 = p3[0]; a7 = p3[1];
    } else if constexpr (KIND == 7) {   // 4 rcp + 4 exp2
      a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_amdgcn_rcpf(a1);
      a2 = __builtin_amdgcn_exp2f(a2); a3 = __builtin_amdgcn_rcpf(a3);
      a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_amdgcn_rcpf(a5);
      a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_amdgcn_rcpf(a7);
    }
  }
  pad[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + acc[0] + acc[5];
  __syncthreads();
  out[blockIdx.x * blockDim.x + threadIdx.x] = pad[(threadIdx.x + 1) % blockDim.x];
}

template <int KIND>
void run(const char* name, int ninstr) {
  float* out;
  hipMalloc(&out, 256 * 1024 * sizeof(float));
  const int iters = 4000;
  for (int wps : {1, 2, 4}) {
    const int threads = 256 * wps;   // wps waves per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(kern<KIND>, dim3(256), dim3(threads), 0, 0, out, iters);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<KIND>, dim3(256), dim3(threads), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // per SIMD: wps waves x iters x ninstr instructions
    const double ns_per = ms * 1e6 / ((double)wps * iters * ninstr);
    printf("%-22s waves/SIMD %d: %7.3f ns per wave-instruction per SIMD (%5.2f cycles @2.4GHz)\n", name,
           wps, ns_per, ns_per * 2.4);
  }
  hipFree(out);
}

int main() {
  run<0>("fma x8", 8);
  run<1>("exp2 x8", 8);
  run<2>("exp2 x4 + fma x4", 8);
  run<7>("exp2 x4 + rcp x4", 8);
  run<3>("mfma32 x1", 1);
  run<4>("mfma32 + exp2 x8", 1);
  run<5>("mfma32 + fma x8", 1);
  run<6>("cmp+ballot x8", 8);
  run<8>("dot2_f32_bf16 x8", 8);
  run<9>("pk_add_f32 x8", 8);
  return 0;
}
