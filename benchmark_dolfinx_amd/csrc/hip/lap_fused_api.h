// extern "C" launchers of the fused structured kernel; one TU per (T, P)
// (lap_fused_<T>_p<P>.hip) keeps compile units small and parallel.
#pragma once
#include "lap_v1.h"  // kGeomStored / kGeomOTF
#include "lap_fused.h"

template <typename T, int ND, int NQ, int GEOM, int MODE>
int launch_fused(const FusedArgs<T>& a, const FusedTables<T>& tb, hipStream_t st) {
  using TF = TileFor<NQ>;
  using S = FusedShape<T, ND, NQ, TF::TY, TF::TZ>;
  const int nblk = a.nty * a.ntz;
  if (nblk <= 0) return 0;
  lap_fused_kernel<T, ND, NQ, TF::TY, TF::TZ, GEOM, MODE>
      <<<nblk, S::threads, 0, st>>>(a, tb);
  return static_cast<int>(hipGetLastError());
}

template <typename T, int ND, int NQ>
int launch_fused_any(int geom, int mode, const FusedArgs<T>& a, const FusedTables<T>& tb,
                     hipStream_t st) {
  if (geom == kGeomOTF) {
    return mode == kFusedCG ? launch_fused<T, ND, NQ, kGeomOTF, kFusedCG>(a, tb, st)
                            : launch_fused<T, ND, NQ, kGeomOTF, kFusedAction>(a, tb, st);
  }
  return mode == kFusedCG ? launch_fused<T, ND, NQ, kGeomStored, kFusedCG>(a, tb, st)
                          : launch_fused<T, ND, NQ, kGeomStored, kFusedAction>(a, tb, st);
}

// Per-(T, P) entry point: nq in {P+1, P+2}.
#define BDX_FUSED_TU(T, SUF, PP)                                                   \
  extern "C" int bdx_fused_apply_##SUF##_p##PP(                                   \
      int geom, int mode, const int64_t* latd, int nq, const double* phi0,        \
      const double* dphi1, const double* wts, const double* qpts, const T* u,     \
      const T* pold, T* pnew, T* y, T* yb, T* zb, T* cb, const T* G, const T* xv, \
      const T* tabs /* host, kFusedTabMax values */,                              \
      double kappa, const double* scal, double* partials, int beta_num,           \
      int beta_den, int nty, int ntz, hipStream_t st) {                            \
    FusedArgs<T> a;                                                               \
    a.lat = BdxLattice::from(latd);                                               \
    a.u = u;                                                                      \
    a.pold = pold;                                                                \
    a.pnew = pnew;                                                                \
    a.y = y;                                                                      \
    a.yb = yb;                                                                    \
    a.zb = zb;                                                                    \
    a.cb = cb;                                                                    \
    a.G = G;                                                                      \
    a.xv = xv;                                                                    \
    a.scal = scal;                                                                \
    a.partials = partials;                                                        \
    a.beta_num = beta_num;                                                        \
    a.beta_den = beta_den;                                                        \
    a.nty = nty;                                                                  \
    a.ntz = ntz;                                                                  \
    a.kappa = static_cast<T>(kappa);                                              \
    FusedTables<T> tb;                                                            \
    for (int i = 0; i < kFusedTabMax; ++i) tb.tab[i] = T(0);                      \
    if (!tabs) return static_cast<int>(hipErrorInvalidValue);                     \
    for (int i = 0; i < kFusedTabMax; ++i) tb.tab[i] = tabs[i];                   \
    for (int q = 0; q < kMaxNq; ++q) {                                            \
      tb.qpts[q] = q < nq ? static_cast<T>(qpts[q]) : T(0);                       \
      tb.wts[q] = q < nq ? static_cast<T>(wts[q]) : T(0);                         \
    }                                                                             \
    (void)phi0;                                                                   \
    (void)dphi1;                                                                  \
    if (nq == PP + 1) return launch_fused_any<T, PP + 1, PP + 1>(geom, mode, a, tb, st); \
    if (nq == PP + 2) return launch_fused_any<T, PP + 1, PP + 2>(geom, mode, a, tb, st); \
    return static_cast<int>(hipErrorInvalidValue);                                \
  }
