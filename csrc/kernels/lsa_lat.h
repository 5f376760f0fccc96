// Host/device-shared argument block of the batch-<=4 latency-path GEMV (kernels/decode_lat.hip documents the
// semantics; bindings.cpp fills it from torch tensors).  Plain C layout, no HIP types.
#pragma once
#include <stdint.h>

struct LatArgs {
  const void* W;    // fragment-major bf16 [N/16][KB][64 lanes][8]
  int KB, N, M, kb_per_split;
  const uint16_t* X;  // SRC_ACT
  int ldx;
  const long long* hq;            // SRC_HQ: Q32 residual [M][ldh] (ldh = K = the hidden size)
  int ldh;
  unsigned long long* ss_acc;     // SRC_HQ: per-row packed (Q16 sum of squares << 8) | publisher count, zeroed per step
  float eps, inv_k;
  long long timeout;              // SRC_HQ: wall-clock ticks a row-sum poll waits before computing the sums itself
  int* stats;                     // nullable: stats[0] += row-sum polls that fell back
  const float* opart;             // SRC_PART: attention partials [B][H][nsplit][128] f32 ...
  const unsigned long long* mlpart;  // ... and their (l << 32 | m) words [B][H][nsplit]
  const int* pos;                 // SRC_PART: decode positions (context = pos + 1 -> the split count)
  int nsplit, chunk_blocks, unsplit_max, H;
  float* out;                     // EPI_F32
  uint16_t* act;                  // EPI_SILU
  long long* hq_out;              // EPI_ATOM
};
