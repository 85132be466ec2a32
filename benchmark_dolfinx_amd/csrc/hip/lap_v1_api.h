// extern "C" entry points of the v1 operator kernels (instantiated per scalar
// type in lap_v1_f64.hip / lap_v1_f32.hip).
#pragma once
#include "lap_v1.h"

template <typename T, int ND, int NQ, int MODE, int GEOM>
int launch_v1(const BdxLattice& lat, const OpTables<T>& tb, const T* G,
              const T* xv, T kappa, const T* kc, const T* u, T* y, const int64_t* lo,
              const int64_t* hi, hipStream_t st) {
  const int64_t e0 = hi[0] - lo[0], e1 = hi[1] - lo[1], e2 = hi[2] - lo[2];
  if (e0 <= 0 || e1 <= 0 || e2 <= 0) return 0;
  const int64_t ncell = e0 * e1 * e2;
  constexpr int cpb = V1Shape<NQ>::cpb;
  const int64_t nblk = (ncell + cpb - 1) / cpb;
  if (nblk > 0x7fffffffLL) return static_cast<int>(hipErrorInvalidValue);
  lap_v1_kernel<T, ND, NQ, MODE, GEOM>
      <<<static_cast<unsigned>(nblk), V1Shape<NQ>::threads, 0, st>>>(
          lat, tb, G, xv, kappa, kc, u, y, lo[0], lo[1], lo[2], e0, e1, e2);
  return static_cast<int>(hipGetLastError());
}

template <typename T, int MODE, int GEOM>
int dispatch_v1(int P, int nq, const BdxLattice& lat, const OpTables<T>& tb,
                const T* G, const T* xv, T kappa, const T* kc, const T* u, T* y,
                const int64_t* lo, const int64_t* hi, hipStream_t st) {
#define BDX_V1_CASE(PP)                                                    \
  case PP:                                                                 \
    if (nq == PP + 1)                                                      \
      return launch_v1<T, PP + 1, PP + 1, MODE, GEOM>(lat, tb, G, xv, kappa, \
                                                      kc, u, y, lo, hi, st); \
    if (nq == PP + 2)                                                      \
      return launch_v1<T, PP + 1, PP + 2, MODE, GEOM>(lat, tb, G, xv, kappa, \
                                                      kc, u, y, lo, hi, st); \
    break;
  switch (P) {
    BDX_V1_CASE(1)
    BDX_V1_CASE(2)
    BDX_V1_CASE(3)
    BDX_V1_CASE(4)
    BDX_V1_CASE(5)
    BDX_V1_CASE(6)
    BDX_V1_CASE(7)
  }
#undef BDX_V1_CASE
  return static_cast<int>(hipErrorInvalidValue);
}

// mode: 0 stiffness (stored G), 1 stiffness (on-the-fly geometry), 2 mass
#define BDX_V1_API(T, SUF)                                                     \
  extern "C" int bdx_v1_apply_##SUF(                                           \
      int mode, const int64_t* latd, int nq, const double* phi0,               \
      const double* dphi1, const double* wts, const double* qpts,              \
      int identity, const T* G, const T* xv, double kappa, const T* kc,        \
      const T* u, T* y,                                                        \
      const int64_t* lo, const int64_t* hi, hipStream_t st) {                  \
    const BdxLattice lat = BdxLattice::from(latd);                             \
    const int P = static_cast<int>(lat.P);                                     \
    const OpTables<T> tb =                                                     \
        make_op_tables<T>(P + 1, nq, phi0, dphi1, wts, qpts, identity);        \
    const T k = static_cast<T>(kappa);                                         \
    if (mode == 0)                                                             \
      return dispatch_v1<T, kModeStiffness, kGeomStored>(P, nq, lat, tb, G, xv, \
                                                         k, kc, u, y, lo, hi, st); \
    if (mode == 1)                                                             \
      return dispatch_v1<T, kModeStiffness, kGeomOTF>(P, nq, lat, tb, G, xv, k, \
                                                      kc, u, y, lo, hi, st);   \
    return dispatch_v1<T, kModeMass, kGeomOTF>(P, nq, lat, tb, G, xv, k, nullptr, \
                                               u, y, lo, hi, st);              \
  }
