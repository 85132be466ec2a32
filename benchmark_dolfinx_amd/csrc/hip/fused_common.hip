// Fused-kernel helpers: tile query and the interface-partials finalize pass.
#include "lap_fused.h"

// Packed 1D tables of the fused kernel (layout: FusedShape::OFF_*), written
// to host memory `out` (which the caller uploads).  Returns the count.
template <typename T, int ND, int NQ>
int pack_tables(const double* phi0, const double* dphi1, T* out) {
  using S = FusedShape<T, ND, NQ, 1, 1>;
  if (!out) return kFusedTabMax;
  for (int i = 0; i < kFusedTabMax; ++i) out[i] = T(0);
  for (int q = 0; q < NQ; ++q)
    for (int m = 0; m < NQ; ++m) {
      out[S::OFF_DR + q * S::XP + m] = static_cast<T>(dphi1[q * NQ + m]);
      out[S::OFF_DC + m * S::XP + q] = static_cast<T>(dphi1[q * NQ + m]);
    }
  for (int q = 0; q < NQ; ++q)
    for (int i = 0; i < ND; ++i) {
      out[S::OFF_PR + q * S::NP + i] = static_cast<T>(phi0[q * ND + i]);
      out[S::OFF_PC + i * S::XP + q] = static_cast<T>(phi0[q * ND + i]);
    }
  return kFusedTabMax;
}


extern "C" {

// Tile shape (cells in y, z) used by the fused kernel for a given nq.
int bdx_fused_tile(int nq, int* ty, int* tz) {
  switch (nq) {
#define BDX_T(NQ)                 \
  case NQ:                        \
    *ty = TileFor<NQ>::TY;        \
    *tz = TileFor<NQ>::TZ;        \
    return 0;
    BDX_T(2) BDX_T(3) BDX_T(4) BDX_T(5) BDX_T(6) BDX_T(7) BDX_T(8) BDX_T(9)
#undef BDX_T
  }
  return static_cast<int>(hipErrorInvalidValue);
}

#define BDX_FIN(T, SUF)                                                          \
  int bdx_fused_finalize_##SUF(const int64_t* latd, T* y, const T* yb, const T* zb, \
                               const T* cb, int nty, int ntz, int sy, int sz,      \
                               hipStream_t st) {                                   \
    const BdxLattice lat = BdxLattice::from(latd);                                 \
    const int64_t n = lat.L[0] * (nty - 1) * lat.L[2] + lat.L[0] * lat.L[1] * (ntz - 1); \
    if (n <= 0) return 0;                                                          \
    int64_t g = (n + 255) / 256;                                                   \
    if (g > 8192) g = 8192;                                                        \
    fused_finalize_kernel<T><<<static_cast<unsigned>(g), 256, 0, st>>>(            \
        lat, y, yb, zb, cb, nty, ntz, sy, sz);                                     \
    return static_cast<int>(hipGetLastError());                                    \
  }

BDX_FIN(double, f64)
BDX_FIN(float, f32)

#define BDX_TABS(T, SUF)                                                           \
  int bdx_fused_tables_##SUF(int nd, int nq, const double* phi0, const double* dphi1, \
                             T* out) {                                             \
    switch (nd * 16 + nq) {                                                        \
      case 2 * 16 + 2: return pack_tables<T, 2, 2>(phi0, dphi1, out);              \
      case 2 * 16 + 3: return pack_tables<T, 2, 3>(phi0, dphi1, out);              \
      case 3 * 16 + 3: return pack_tables<T, 3, 3>(phi0, dphi1, out);              \
      case 3 * 16 + 4: return pack_tables<T, 3, 4>(phi0, dphi1, out);              \
      case 4 * 16 + 4: return pack_tables<T, 4, 4>(phi0, dphi1, out);              \
      case 4 * 16 + 5: return pack_tables<T, 4, 5>(phi0, dphi1, out);              \
      case 5 * 16 + 5: return pack_tables<T, 5, 5>(phi0, dphi1, out);              \
      case 5 * 16 + 6: return pack_tables<T, 5, 6>(phi0, dphi1, out);              \
      case 6 * 16 + 6: return pack_tables<T, 6, 6>(phi0, dphi1, out);              \
      case 6 * 16 + 7: return pack_tables<T, 6, 7>(phi0, dphi1, out);              \
      case 7 * 16 + 7: return pack_tables<T, 7, 7>(phi0, dphi1, out);              \
      case 7 * 16 + 8: return pack_tables<T, 7, 8>(phi0, dphi1, out);              \
      case 8 * 16 + 8: return pack_tables<T, 8, 8>(phi0, dphi1, out);              \
      case 8 * 16 + 9: return pack_tables<T, 8, 9>(phi0, dphi1, out);              \
    }                                                                              \
    return -1;                                                                     \
  }
BDX_TABS(double, f64)
BDX_TABS(float, f32)

}  // extern "C"
