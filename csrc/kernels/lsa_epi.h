// Host/device-shared argument block of the decode-GEMM epilogue extensions (kernels/common.h documents
// the semantics; bindings.cpp fills it from torch tensors).  Plain C layout, no HIP types.
#pragma once
#include <stdint.h>

struct LsaEpi {
  const long long* rowss;  // per-row sum of squares of the un-normalised X rows in Q24 fixed point (RMS row
                           // scale), or null
  float inv_k;         // 1 / hidden size
  float eps;           // RMSNorm epsilon
  float* h;            // EPI_RES: f32 residual [M][ldh], updated in place
  int ldh;
  uint16_t* xout;      // EPI_RES: bf16(h) for the next GEMM
  int xmt;             // row tiles of the fragment-major xout layout (0 = row-major)
  long long* ss_out;   // EPI_RES: per-row sum of h^2 in Q24 fixed point (x 2^24, int64 atomics: the
                       // total does not depend on the order the workgroups add in, so decoding is deterministic)
  int* tickets;        // EPI_RES with split-K: one zeroed arrival counter per workgroup column (grid.x);
                       // the last split to arrive finishes the column and resets its counter
};
