// Internal launch interfaces shared by the kernel files and the step plan.
#pragma once
#include "snd_common.hpp"

namespace snd {

constexpr int kGemmBK = 64;  // K tile of the generic GEMM; split-K chunks are multiples

enum AMode { A_ROW = 0, A_COL = 1, A_CONV = 2, A_CONVT = 3 };
enum BMode { B_ROW = 0, B_COL = 1, B_FLIP = 2 };
enum Epi { E_STORE = 0, E_CONV = 1, E_PART = 2 };

struct GemmArgs {
  int M, N, K;
  const float* A; int lda; int a_cin; int a_npg;
  const float* B; int ldb; int b_cout;
  float* C; int ldc;
  const float* bias; const float* gamma; const float* beta;
  float* pre; int ldp;
  int kchunk;       // K range per blockIdx.z (multiple of 32)
  int accumulate;   // E_STORE: C += result
  int a_ones_m1;    // A_COL: 1 + row index m that reads as 1.0 (bias-gradient row); 0 = none
};

int launch_gemm(GemmArgs g, int amode, int bmode, int epi, int dtype, int splits,
                hipStream_t s);
int gemm_splits(int K, int target_blocks_per_tile);

// Deterministic reduction of partial slabs, fixed summation order:
//   dst[r*dst_rs + i] (+)= scale * sum_p src[p*stride + r*src_rs + i],  i < len, r < rows
// (rows == 0 means one row).
struct ReduceDesc {
  const float* src;
  float* dst;
  int nparts;
  int len;
  long long stride;
  float scale;
  int accumulate;
  int rows;
  long long src_rs, dst_rs;
};
constexpr int kMaxReduce = 48;
struct FinalizeArgs;
// TF1 Adam applied by the reduction itself (single device, snd_plan_fuse_adam): every
// element of a descriptor whose bit is set in mask is a complete gradient g of the
// parameter at (dst - gbase) of p / m / v; the reduction stores g and updates that
// parameter (same arithmetic as snd_adam_tf1).  stepn: the step the update uses,
// *step + 1, published by the step's reparameterisation kernel -- the finalize block of
// the same launch advances *step, so the reduction blocks cannot read *step itself.
struct ReduceAdam {
  const float* gbase;
  float* p; float* m; float* v;
  float lr, b1, b2, eps;
  const int* stepn;
  unsigned long long mask;      // bit i: descriptor i of the launch's descriptor list
};
// Deterministic slab reductions; with fin, the same launch also computes the loss
// terms (snd_elem.hpp FinalizeArgs) in an extra workgroup.
int launch_reduce(const ReduceDesc* d, int n, hipStream_t s, const FinalizeArgs* fin = nullptr,
                  const ReduceAdam* adam = nullptr);

// Column partial sums written by elementwise kernels are laid out as
// slab[block][ncols]; helpers compute the block count used.
constexpr int kColRows = 64;   // rows per block in column-reduction kernels

}  // namespace snd
