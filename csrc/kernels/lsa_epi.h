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

// Residual-reduce prologue of a batch-1 decode GEMM (gemm.hip, RR > 0): instead of a bf16 X row written by a
// residual-add launch, the GEMM reads the previous row-parallel projection's f32 split-K slabs and the f32
// residual stream and forms X = h + sum_s parts[s] itself (its own K slice, into LDS).  The workgroups of column
// group 0 also write that sum to h_out (the next residual stream; never the buffer being read), and the RMS row
// scale rsqrt(sum X^2 / K + eps) is either applied in the epilogue from the workgroup's own full-row sum
// (local = 1: splitk 1, every workgroup sees the whole row) or left to the consumer of the f32 slabs, the
// column-0 workgroups adding their slice's sum of squares to ss_out (Q24, integer atomics: order-independent).
struct LsaRr {
  const float* h;      // [K] f32 residual stream in
  const float* parts;  // [np][K] f32 split-K slabs of the producing projection (slab stride pstride floats)
  long pstride;
  int np;
  float* h_out;        // [K] f32: h + sum(parts)
  long long* ss_out;   // local = 0: Q24 accumulator of sum X^2 (zeroed before the step)
  int local;
  float inv_k;         // 1 / K (the hidden size)
  float eps;
};
