// Workspace of the stream-K prefill GEMM (gemm_tile256.hip lsa_gemm_sk), shared by the kernel and the bindings.
#pragma once

// f32 partial of one 256 x 256 output tile, in the accumulators' own order [wave][i][j][lane][4]
#define LSA_SK_SLOT_FLOATS (256 * 256)

// a grid of ncu workgroups publishes at most two partial tiles per workgroup (the first and the last segment of its
// stream-K range), and has at most 2 * ncu stream-K tiles (one ticket each)
static inline long long lsa_gemm_sk_ws_bytes(int ncu) { return 2LL * ncu * LSA_SK_SLOT_FLOATS * 4; }
static inline int lsa_gemm_sk_tickets(int ncu) { return 2 * ncu; }
