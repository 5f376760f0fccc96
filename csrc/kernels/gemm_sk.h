// Workspace of the stream-K prefill GEMM (gemm_tile256.hip lsa_gemm_sk), shared by the kernel and the bindings.
#pragma once

// f32 partial of one 256 x 256 output tile, in the accumulators' own order [wave][i][j][lane][4] (a tile
// configuration's slot is BM x BN floats)
#define LSA_SK_SLOT_FLOATS (256 * 256)

// a grid of P workgroups publishes at most two partial tiles per workgroup (the first and the last segment of its
// stream-K range) and has at most 2 P stream-K tiles (one ticket each).  P = ncu for the 8-wave tiles, 2 ncu for the
// 4-wave ones (two per CU) whose BM x BN <= 128 x 192 slots take at most 2 * 2 ncu * 24576 floats
static inline long long lsa_gemm_sk_ws_bytes(int ncu) { return 2LL * ncu * LSA_SK_SLOT_FLOATS * 4; }
static inline int lsa_gemm_sk_tickets(int ncu) { return 4 * ncu; }
