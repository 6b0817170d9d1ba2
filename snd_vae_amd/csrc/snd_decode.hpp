#pragma once
#include "snd_common.hpp"

namespace snd {

// generated_adj (model.py:205-208): for i != j the 2-class logits are (0, L_ij)
// with L = J J^T (layers.py:407-409), the diagonal is (1, 0); argmax picks index 1
// iff L_ij > 0 (ties go to index 0).  out[b][i][j] in {0, 1}, uint8 [B, n, n].
struct GenAdjArgs {
  const float* j; int ldj; int d;   // [B*n, ldj] fp32 decoder input J
  int n, ngraphs;
  unsigned char* out;
};
int launch_gen_adj(const GenAdjArgs& a, hipStream_t s);

}  // namespace snd
