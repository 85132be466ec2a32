// Fused-kernel helpers: tile query and the interface-partials finalize pass.
#include "lap_fused.h"

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

}  // extern "C"
