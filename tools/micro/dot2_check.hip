// v_dot2c_f32_bf16 with (1, 0) / (0, 1) as an fp32 accumulate of one bf16 half:
// compared bit for bit with the plain fp32 add of the unpacked value.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned* w, const float* c, unsigned* bad, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned lo1u, hi1u;
  asm volatile("s_mov_b32 %0, 0x3f80" : "=s"(lo1u));
  asm volatile("s_mov_b32 %0, 0x3f800000" : "=s"(hi1u));
  const bf16x2 x = __builtin_bit_cast(bf16x2, w[i]);
  const float a = __builtin_amdgcn_fdot2_f32_bf16(x, __builtin_bit_cast(bf16x2, lo1u), c[i], false);
  const float b = __builtin_amdgcn_fdot2_f32_bf16(x, __builtin_bit_cast(bf16x2, hi1u), c[i], false);
  const float ra = c[i] + __uint_as_float(w[i] << 16);
  const float rb = c[i] + __uint_as_float(w[i] & 0xFFFF0000u);
  const int ua = abs((int)__float_as_uint(a) - (int)__float_as_uint(ra));
  const int ub = abs((int)__float_as_uint(b) - (int)__float_as_uint(rb));
  // bits 0-7: ulp distance of the low-half accumulate (capped), 8-15: the high half
  bad[i] = (unsigned)min(ua, 255) | ((unsigned)min(ub, 255) << 8);
}
static float rnd(void) {
  return (float)((rand() / (double)RAND_MAX - 0.5) * std::pow(2.0, (rand() % 40) - 20));
}
int main() {
  const int n = 1 << 22;
  unsigned* hw = (unsigned*)malloc(4 * (size_t)n);
  float* hc = (float*)malloc(4 * (size_t)n);
  srand(1);
  for (int i = 0; i < n; ++i) {
    float x = rnd(), y = rnd();
    unsigned u, v;
    memcpy(&u, &x, 4);
    memcpy(&v, &y, 4);
    hw[i] = (u >> 16) | (v & 0xFFFF0000u);
    hc[i] = rnd();
  }
  unsigned *dw, *db;
  float* dc;
  if (hipMalloc(&dw, 4 * (size_t)n) || hipMalloc(&dc, 4 * (size_t)n) || hipMalloc(&db, 4 * (size_t)n)) return 1;
  if (hipMemcpy(dw, hw, 4 * (size_t)n, hipMemcpyHostToDevice) || hipMemcpy(dc, hc, 4 * (size_t)n, hipMemcpyHostToDevice)) return 1;
  k<<<n / 256, 256>>>(dw, dc, db, n);
  if (hipMemcpy(hw, db, 4 * (size_t)n, hipMemcpyDeviceToHost)) return 1;
  long lo = 0, hi = 0;
  unsigned mlo = 0, mhi = 0;
  for (int i = 0; i < n; ++i) {
    const unsigned a = hw[i] & 255u, b = (hw[i] >> 8) & 255u;
    lo += a != 0; hi += b != 0;
    mlo = a > mlo ? a : mlo; mhi = b > mhi ? b : mhi;
  }
  printf("dot2 accumulate vs fp32 add: %d cases, low half differs %ld (max %u ulp), high half differs %ld (max %u ulp)\n",
         n, lo, mlo, hi, mhi);
  return 0;
}
