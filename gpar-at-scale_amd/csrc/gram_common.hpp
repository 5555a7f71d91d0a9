// gram_common.hpp -- tiling constants and tile maps shared by the Gram kernels (k_gram.hip:
// v1/v2 and the v3 OFF kernel; k_gram3v.hip: the v3 DG and chunk-correction kernels, compiled
// with VGPR-form MFMA accumulators).
#pragma once
#include "device_common.hpp"
#include "launch.hpp"

namespace gpar {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kPW = 64;               // panel width (columns of beta / of G)
constexpr int kBK = 16;               // time rows per K-step
constexpr int kPanelD = kBK * kPW;    // doubles per staged panel

// DG decomposition (v2 / v3): the lower triangle of a diagonal 128 x 128 block = 8 x 8 tiles of
// 16 x 16, 36 tiles split 18 + 18 over two waves: half 0 owns local tile rows {0, 1, 2, 3, 7},
// half 1 rows {4, 5, 6}; tile (row r, col c <= r) sits at index d2_tile within its half.
constexpr int kD2T = 18;   // tiles per DG wave (accumulators: 72 doubles)

template <int H>
__device__ __forceinline__ constexpr int d2_row(int ia) { return H == 0 ? (ia < 4 ? ia : 7) : 4 + ia; }
template <int H>
__device__ __forceinline__ constexpr int d2_na() { return H == 0 ? 5 : 3; }
template <int H>
__device__ __forceinline__ constexpr int d2_nb() { return H == 0 ? 8 : 7; }
template <int H>
__device__ __forceinline__ constexpr int d2_tile(int ia, int c) {
  int t = 0;
  for (int i = 0; i < ia; ++i) t += d2_row<H>(i) + 1;
  return t + c;
}
// local tile row r (0..7) of a diagonal block -> its half and the index of tile (r, 0)
__device__ __forceinline__ int d2_half_of(int r) { return (r >= 4 && r < 7) ? 1 : 0; }
__device__ __forceinline__ int d2_base_of(int r) {
  return r < 4 ? r * (r + 1) / 2 : (r == 7 ? 10 : (r == 4 ? 0 : (r == 5 ? 5 : 11)));
}

// v3 partial-tile slots per wave (OFF: 4 x 8 tiles; DG: 18 of the 32 used)
constexpr int kF3T = 32;

// (GramGroupPtrs, the grouped Gram's per-output pointer table: launch.hpp)

// v3 launchers living in k_gram3v.hip (VGPR-form MFMA accumulators)
// sw / rows_w: the first sw time splits take rows_w rows each, the others `rows` (sw = 0: all)
void launch_gram3_dg(hipStream_t st, int nwg, const double* beta, int64_t ldb, int64_t n,
                     const double* alpha, int npan, int ndg, int sdg, int64_t rows,
                     int64_t slot0, double* part, double* rpart, int bt_lo = 0, int bt_cnt = -1,
                     int sw = 0, int64_t rows_w = 0, const GramGroupPtrs* grp = nullptr,
                     int ngrp = 1);
void launch_gram3_corr_slim(hipStream_t st, int sdim, const double* ecor, const double* cin,
                            const double* qv, int64_t mc, int64_t nch, int npan, int noff, int ndg,
                            int soff, int sdg, int ncs, double* part, double* rpart,
                            const GramGroupPtrs* grp = nullptr, int ngrp = 1);
void launch_gram3_corr(hipStream_t st, int sdim, const double* ecor, const double* cin,
                       const double* qv, int64_t mc, int64_t nch, int npan, int noff, int ndg,
                       int soff, int sdg, int ncs, double* part, double* rpart,
                       const GramGroupPtrs* grp = nullptr, int ngrp = 1);

}  // namespace gpar
