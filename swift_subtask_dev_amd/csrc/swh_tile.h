// swh_tile.h — the tile neighbour loop (loop variant 3, the default).
//
// One 64-lane wave serves NS = 64/SG i-groups, one per SG-lane row (SG = 16:
// the DPP row). A group is an octree leaf of the Morton-ordered cells with
// <= SG particles (swh_space.hip group_kernel), so each row's particles are
// compact in space. Per row:
//   staging : the row enumerates the cells overlapping its bounding box grown
//             by the reach (SG cells per pass, one per lane, from the
//             per-cell span table), then streams their particles SG at a time
//             (coalesced loads), prunes each against the exact box distance
//             (density/gradient: H_group, force: max(H_group, H_j)) and
//             appends the survivors - position plus the loop's j record - to
//             the row's LDS region;
//   phase A : every lane tests its own i against each staged candidate of
//             its row (LDS broadcast reads, fp64, the loop's exact accept())
//             and appends hits to its per-lane list (LDS slot indices);
//   phase B : drains the lists; interactions read only LDS, so all lanes with
//             pending hits work, none waits on global memory.
// The drain runs whenever a list may overflow and before the staged region
// is reused. Summation order differs from the per-particle variants only in
// fp64 rounding.
#pragma once

#include "swh_gather.h"

namespace swh {

constexpr int kTileCap = 32;  // per-lane hit list (checked every 8 candidates)

// Staged candidate slots per wave: density/gradient 256, force 128 (its j
// record is three float4s).
template <int LOOP>
struct TileSlots {
  static constexpr int value = (LOOP == LOOP_FORCE) ? 128 : 256;
};

template <int SG, int TS, int NPAY>
struct TileLds {
  double4 pos[TS];  // x, y, z (image-shifted unless nearest-image), h
  float4 pay[NPAY][TS];
  int candj[TS];
  int meta[TS];
  int cell_j0[64];
  int cell_pre[64];
  int cell_code[64];
  unsigned short hits[kTileCap * 64];  // [k][lane] slot indices
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Reductions within a row of SG lanes (xor offsets < SG stay in the row).
template <int SG>
__device__ __forceinline__ double row_min(double v) {
  for (int o = SG / 2; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}
template <int SG>
__device__ __forceinline__ double row_max(double v) {
  for (int o = SG / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ double shift_of(int code, double box) {
  return code == 1 ? -box : (code == 2 ? box : 0.);
}

template <typename T, class S, class LDS>
__device__ __forceinline__ void tile_drain(const GridDev& g, const CellRange& c,
                                           const double4& pi, LDS& L, int& nh, int lane,
                                           S& st) {
  for (int k = 0; k < nh; k++) {
    const int slot = L.hits[k * 64 + lane];
    const double4 cj = L.pos[slot];
    double dx = pi.x - cj.x, dy = pi.y - cj.y, dz = pi.z - cj.z;
    if (c.full[0]) dx = wrap_nearest(dx, g.dim[0]);
    if (c.full[1]) dy = wrap_nearest(dy, g.dim[1]);
    if (c.full[2]) dz = wrap_nearest(dz, g.dim[2]);
    const T tdx = (T)dx, tdy = (T)dy, tdz = (T)dz;
    const T r2 = tdx * tdx + tdy * tdy + tdz * tdz;
    float4 p[S::kPay];
#pragma unroll
    for (int q = 0; q < S::kPay; q++) p[q] = L.pay[q][slot];
    st.interact_staged(p, L.meta[slot], cj, tdx, tdy, tdz, r2);
  }
  nh = 0;
}

// Phase A over the staged regions (each row its own), then the drain that
// frees the regions. A lane's list holds <= kTileCap - 8 entries at the start
// of every block of 8 candidates, so it never overflows.
template <int SG, typename T, class S, class LDS>
__device__ __forceinline__ void tile_consume(const GridDev& g, const CellRange& c,
                                             const double4& pi, bool act, int rbase, int nst,
                                             LDS& L, int& nh, int lane, S& st) {
  int kmax = nst;
  for (int o = 32; o >= SG; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
  for (int k = 0; k < kmax; k++) {
    if ((k & 7) == 0 && __any(nh > kTileCap - 8)) tile_drain<T>(g, c, pi, L, nh, lane, st);
    if (k < nst) {
      const int slot = rbase + k;
      const double4 cj = L.pos[slot];
      double dx = pi.x - cj.x, dy = pi.y - cj.y, dz = pi.z - cj.z;
      if (c.full[0]) dx = wrap_nearest(dx, g.dim[0]);
      if (c.full[1]) dy = wrap_nearest(dy, g.dim[1]);
      if (c.full[2]) dz = wrap_nearest(dz, g.dim[2]);
      const T tdx = (T)dx, tdy = (T)dy, tdz = (T)dz;
      const T r2 = tdx * tdx + tdy * tdy + tdz * tdz;
      if (act && st.accept(L.candj[slot], cj, r2)) {
        L.hits[nh * 64 + lane] = (unsigned short)slot;
        nh++;
      }
    }
  }
  tile_drain<T>(g, c, pi, L, nh, lane, st);
}

template <int LOOP, typename T, int SG, class LDS>
__device__ __forceinline__ void tile_loop(const GridDev& g, SoA& a,
                                          const int2* __restrict__ groups, int ngroups,
                                          int max_active_bin, T a2H,
                                          const unsigned int* __restrict__ hmax_bits,
                                          unsigned long long* counter, int* __restrict__ ncount,
                                          LDS& L) {
  using S = LoopState<LOOP, T>;
  constexpr int NS = 64 / SG;
  constexpr int TS = TileSlots<LOOP>::value;
  constexpr int CR = TS / NS;  // slots per row
  const int lane = threadIdx.x & 63;
  const int row = lane / SG, r = lane % SG;
  const int gid = blockIdx.x * NS + row;
  const int2 gr = gid < ngroups ? groups[gid] : make_int2(0, 0);
  const int i = r < gr.y ? gr.x + r : -1;
  const bool act = i >= 0 && a.tb[i] <= max_active_bin;
  S st;
  st.n = 0;
  double4 pi = make_double4(0., 0., 0., 0.);
  if (act) {
    st.load_i(a, i, a2H, hmax_bits);
    pi = a.pos[i];
  }
  // row bounding box, largest H, cell range
  const double Hg = row_max<SG>(act ? pi.w * (double)kGamma : 0.);
  double lo[3], hi[3];
  lo[0] = row_min<SG>(act ? pi.x : 1e300);
  lo[1] = row_min<SG>(act ? pi.y : 1e300);
  lo[2] = row_min<SG>(act ? pi.z : 1e300);
  hi[0] = row_max<SG>(act ? pi.x : -1e300);
  hi[1] = row_max<SG>(act ? pi.y : -1e300);
  hi[2] = row_max<SG>(act ? pi.z : -1e300);
  bool rdone = !(Hg > 0.);
  const double hmax_reach = (double)__uint_as_float(*hmax_bits) * (double)kGamma;
  const double reach = (LOOP == LOOP_FORCE) ? fmax(Hg, hmax_reach) : Hg;
  CellRange c;
  int nx = 1, ny = 1, ncells = 0;
  for (int k = 0; k < 3; k++) {
    c.full[k] = false;
    c.lo[k] = c.hi[k] = 0;
  }
  if (!rdone) {
    for (int k = 0; k < 3; k++) {
      c.lo[k] = (int)floor((lo[k] - g.origin[k] - reach) * g.inv_w[k]);
      c.hi[k] = (int)floor((hi[k] - g.origin[k] + reach) * g.inv_w[k]);
      if (g.periodic) {
        c.full[k] = (c.hi[k] - c.lo[k] + 1 >= g.cdim[k]);
        if (c.full[k]) {
          c.lo[k] = 0;
          c.hi[k] = g.cdim[k] - 1;
        }
      } else {
        c.lo[k] = max(c.lo[k], 0);
        c.hi[k] = min(c.hi[k], g.cdim[k] - 1);
      }
    }
    nx = c.hi[0] - c.lo[0] + 1;
    ny = c.hi[1] - c.lo[1] + 1;
    ncells = nx * ny * (c.hi[2] - c.lo[2] + 1);
  }
  const int rbase = row * CR;  // this row's staged region
  const int cbase = row * SG;  // this row's cell table
  int cb = 0, total = 0, base = 0, nst = 0, nh = 0;
  for (;;) {
    if (!rdone && base >= total) {  // row-uniform: next batch of SG cells
      if (cb >= ncells) {
        rdone = true;
      } else {
        const int cl = cb + r;
        int cnt = 0, j0 = 0, code = 0;
        if (cl < ncells) {
          double sx, sy, sz;
          const int wx = wrap_cell(g, c, 0, c.lo[0] + cl % nx, sx);
          const int wy = wrap_cell(g, c, 1, c.lo[1] + (cl / nx) % ny, sy);
          const int wz = wrap_cell(g, c, 2, c.lo[2] + cl / (nx * ny), sz);
          code = (sx < 0. ? 1 : (sx > 0. ? 2 : 0)) | ((sy < 0. ? 1 : (sy > 0. ? 2 : 0)) << 2) |
                 ((sz < 0. ? 1 : (sz > 0. ? 2 : 0)) << 4);
          const int2 sp = cell_range_of(g, wx, wy, wz);
          j0 = sp.x;
          cnt = sp.y - sp.x;
        }
        int inc = cnt;
        for (int o = 1; o < SG; o <<= 1) {
          const int t = __shfl_up(inc, o, SG);
          if (r >= o) inc += t;
        }
        total = __shfl(inc, SG - 1, SG);
        L.cell_j0[lane] = j0;
        L.cell_pre[lane] = inc - cnt;
        L.cell_code[lane] = code;
        base = 0;
        cb += SG;
      }
    }
    if (__all(rdone)) break;
    wave_sync();
    bool keep = false;
    double4 p = make_double4(0., 0., 0., 0.);
    int j = 0;
    if (!rdone && base < total) {
      const int q = base + r;
      if (q < total) {
        int k = 0;  // last cell of the row whose prefix is <= q
        for (int step = SG / 2; step > 0; step >>= 1)
          if (L.cell_pre[cbase + k + step] <= q) k += step;
        j = L.cell_j0[cbase + k] + (q - L.cell_pre[cbase + k]);
        const int sc = L.cell_code[cbase + k];
        p = a.pos[j];
        p.x += shift_of(sc & 3, g.dim[0]);
        p.y += shift_of((sc >> 2) & 3, g.dim[1]);
        p.z += shift_of((sc >> 4) & 3, g.dim[2]);
        const double ex = c.full[0] ? 0. : fmax(fmax(lo[0] - p.x, p.x - hi[0]), 0.);
        const double ey = c.full[1] ? 0. : fmax(fmax(lo[1] - p.y, p.y - hi[1]), 0.);
        const double ez = c.full[2] ? 0. : fmax(fmax(lo[2] - p.z, p.z - hi[2]), 0.);
        const double rj = (LOOP == LOOP_FORCE) ? fmax(Hg, p.w * (double)kGamma) : Hg;
        keep = ex * ex + ey * ey + ez * ez <= rj * rj;
      }
      base += SG;
    }
    const unsigned long long m = __ballot(keep);
    const unsigned long long rowbits =
        SG == 64 ? m : (m >> (row * SG)) & ((1ull << (SG & 63)) - 1ull);
    if (keep) {
      const int slot = rbase + nst + __popcll(rowbits & ((1ull << r) - 1ull));
      float4 pay[S::kPay];
      int meta;
      S::load_j(a, j, pay, meta);
      L.pos[slot] = p;
#pragma unroll
      for (int q = 0; q < S::kPay; q++) L.pay[q][slot] = pay[q];
      L.candj[slot] = j;
      L.meta[slot] = meta;
    }
    nst += __popcll(rowbits);
    if (__any(nst > CR - SG)) {
      wave_sync();
      tile_consume<SG, T>(g, c, pi, act, rbase, nst, L, nh, lane, st);
      nst = 0;
    }
    wave_sync();
  }
  wave_sync();
  tile_consume<SG, T>(g, c, pi, act, rbase, nst, L, nh, lane, st);
  if (act) {
    st.store(a, i);
    if (ncount) ncount[i] = st.n;
  }
  if (counter) {
    unsigned long long v = (unsigned long long)(act ? st.n : 0);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0 && v) atomicAdd(counter, v);
  }
}

}  // namespace swh
