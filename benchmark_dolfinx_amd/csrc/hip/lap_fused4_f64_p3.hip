// Fused v4 operator kernels (MFMA core), double, degree 3.
#include "lap_fused4.h"

// fused4 apply entry (CG-fused or plain action) for Q3 FP64.
extern "C" int bdx_fused4_apply_f64_p3(
    int mode, int affine_ok, const int64_t* latd, int nq, const double* wts, const double* qpts,
    const double* u, const double* pold, double* pnew, double* x, double* y, double* yb,
    double* zb, double* cb, const double* xv, const double* kc, const double* tabs, double kappa,
    const double* scal, double* partials, int beta_num, int beta_den, int xa_num, int xa_den,
    int nty, int ntz, const int* rect, hipStream_t st) {
  (void)wts;
  (void)qpts;
  (void)nq;
  // the Kronecker factorisation needs a constant Jacobian per cell
  if (!affine_ok || !tabs) return static_cast<int>(hipErrorInvalidValue);
  Fused2Args<double> a;
  BDX_CHECK(static_cast<hipError_t>(make_fused2_args(a, latd, nty, ntz)));
  BDX_CHECK(static_cast<hipError_t>(fused_set_rect(a, rect)));
  BDX_CHECK(static_cast<hipError_t>(fused_set_segments(a, mode >> 8)));
  mode &= 0xff;
  a.u = u;
  a.pold = pold;
  a.pnew = pnew;
  a.x = x;
  a.y = y;
  a.yb = yb;
  a.zb = zb;
  a.cb = cb;
  a.xv = xv;
  a.kc = kc;
  a.scal = scal;
  a.partials = partials;
  a.beta_num = beta_num;
  a.beta_den = beta_den;
  a.xa_num = xa_num;
  a.xa_den = xa_den;
  a.kappa = kappa;
  FusedTables<double> tb;
  for (int i = 0; i < kFusedTabMax; ++i) tb.tab[i] = tabs[i];
  for (int q = 0; q < kMaxNq; ++q) tb.qpts[q] = tb.wts[q] = 0.0;
  return mode == kFusedCG ? launch_fused4<kFusedCG>(a, tb, st)
                          : launch_fused4<kFusedAction>(a, tb, st);
}

// Pack the 1D M / K / C tables of the quadrature rule for fused4.
extern "C" int bdx_fused4_tables_f64(int nd, int nq, const double* phi0, const double* Dd,
                                     const double* wts, double* out) {
  return pack_tables4(nd, nq, phi0, Dd, wts, out);
}

// Cell tile (TY, TZ) of the fused4 instance, for the host-side launch geometry.
extern "C" int bdx_fused4_tile(int* ty, int* tz) {
  *ty = kF4TY;
  *tz = kF4TZ;
  return 0;
}

// x segments per tile for a launch of `tiles` tiles marching `ncx` layers
// (fused_choose_segments with this kernel's resident workgroups).
extern "C" int bdx_fused4_segments(int tiles, int ncx) {
  constexpr int TY = kF4TY, TZ = kF4TZ;
  int per_cu = 0, dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, lap_fused4_kernel<TY, TZ, kFusedCG>, TY * TZ * 16, 0) != hipSuccess)
    return 1;
  return fused_choose_segments(tiles, ncx, per_cu * cus);
}
