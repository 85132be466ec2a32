// Shared (host + device) description of one rank's piece of the box mesh.
//
// Layout of the packed int64 descriptor produced by
// benchmark_dolfinx_amd.fem.mesh.LocalLattice.as_int64():
//   [0..2]  n   local cells per axis
//   [3..5]  L   local dof lattice extent per axis (n*P + 1)
//   [6..8]  g0  global lattice index of local index 0
//   [9..11] N   global lattice extent per axis
//   [12..14] gh 1 if the upper plane of the axis is a ghost plane
//   [15]    P   polynomial degree
//   [16]    ld  z pitch of the storage (>= L[2], rows 128-byte aligned)
//   [17..20] tiled storage (0 = the lattice layout above): tile node sizes
//           tsy, tsz, storage tiles along z tntz, and the tile-column
//           stride tcol = L[0] tsy tsz.  In the tiled layout node (i, j, k)
//           lives at ((j / tsy) tntz + k / tsz) tcol + i tsy tsz
//           + (j % tsy) tsz + k % tsz: a (y, z) tile's patch of an x-plane
//           is contiguous (the CG runtime's layout for the x-march kernels,
//           whose writes of 96-byte row segments ran at 1.7 TB/s in the
//           lattice layout and 5.4 TB/s tiled, profiles/r2_march_bw.md).
//
// The mesh is a structured lattice by construction (see fem/mesh.py), so the
// cell -> dof map is arithmetic: dof(c, i, j, k) = lattice index
// ((cx*P+i)*Ly + cy*P+j)*ld + cz*P+k.  This replaces the explicit DOLFINx
// dofmap the reference copies to the device (src/laplacian.hpp:105-114).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define BDX_HD __host__ __device__ __forceinline__
#else
#define BDX_HD inline
#endif

struct BdxLattice {
  int64_t n[3];
  int64_t L[3];
  int64_t g0[3];
  int64_t N[3];
  int64_t gh[3];
  int64_t P;
  int64_t ld;
  int64_t tsy, tsz, tntz, tcol;  // tiled storage (tsy = 0: lattice layout)

  static BdxLattice from(const int64_t* d) {
    BdxLattice l;
    for (int a = 0; a < 3; ++a) {
      l.n[a] = d[a];
      l.L[a] = d[3 + a];
      l.g0[a] = d[6 + a];
      l.N[a] = d[9 + a];
      l.gh[a] = d[12 + a];
    }
    l.P = d[15];
    l.ld = d[16];
    l.tsy = d[17];
    l.tsz = d[18];
    l.tntz = d[19];
    l.tcol = d[20];
    return l;
  }

  // lattice-layout index (every lattice kernel)
  BDX_HD int64_t idx(int64_t i, int64_t j, int64_t k) const {
    return (i * L[1] + j) * ld + k;
  }
  // storage index in whichever layout the descriptor selects (the kernels
  // that also run on the CG runtime's tiled storage)
  BDX_HD int64_t sidx(int64_t i, int64_t j, int64_t k) const {
    if (tsy) return ((j / tsy) * tntz + k / tsz) * tcol + (i * tsy + j % tsy) * tsz + k % tsz;
    return (i * L[1] + j) * ld + k;
  }
  BDX_HD int64_t size() const {
    return tsy ? ((L[1] - 1) / tsy + 1) * tntz * tcol : L[0] * L[1] * ld;
  }
  // Dirichlet dof: on the boundary of the global unit cube.
  BDX_HD bool is_bc(int64_t i, int64_t j, int64_t k) const {
    int64_t gi = g0[0] + i, gj = g0[1] + j, gk = g0[2] + k;
    return gi == 0 || gj == 0 || gk == 0 || gi == N[0] - 1 || gj == N[1] - 1 ||
           gk == N[2] - 1;
  }
  // Owned by this rank (not on a ghost plane).
  BDX_HD bool is_owned(int64_t i, int64_t j, int64_t k) const {
    return i < L[0] - gh[0] && j < L[1] - gh[1] && k < L[2] - gh[2];
  }
  BDX_HD int64_t vidx(int64_t a, int64_t b, int64_t c) const {
    return ((a * (n[1] + 1) + b) * (n[2] + 1) + c);
  }
};
