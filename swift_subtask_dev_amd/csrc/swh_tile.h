// swh_tile.h — the tile neighbour loop (loop variant 3, the default).
//
// One 64-lane wave serves NS = 64/SG i-groups, one per SG-lane row (SG = 16:
// the DPP row). A group is an octree leaf of the Morton-ordered cells with
// <= SG particles (swh_space.hip group_kernel), so each row's particles are
// compact in space. Per row:
//   staging : the row enumerates the cells overlapping its bounding box grown
//             by the reach (4*SG cells per batch from the per-cell span
//             table), then streams their particles U*SG at a time (all loads
//             of a pass in flight together), prunes each against the exact
//             box distance (density/gradient: H_group, force:
//             max(H_group, H_j)) and appends the survivors' positions to the
//             row's LDS region;
//   phase A : every lane tests its own i against each staged candidate of
//             its row (LDS broadcast reads, fp64, the loop's exact accept())
//             and appends hits (global j) to its per-lane list in LDS;
//   phase B : drains the lists once any lane's list is nearly full (and at
//             the end): every lane with pending hits evaluates the iact on
//             the j record read from HBM/L2, the next hit's loads issued
//             before the current hit is computed.
// Hit lists outlive the staged regions, so drains run with nearly full lists
// instead of at every region turnover. Summation order differs from the
// per-particle variants only in fp64 rounding.
#pragma once

#include "swh_gather.h"

namespace swh {

#ifndef SWH_TILE_CAP
#define SWH_TILE_CAP 32
#endif
constexpr int kTileCap = SWH_TILE_CAP;  // per-lane hit list (checked every 8 candidates)

// Staged candidate slots per wave and candidates fetched per lane per pass.
template <int LOOP>
struct TileSlots {
  static constexpr int value = 256;
};
#ifndef SWH_TILE_FETCH
#define SWH_TILE_FETCH 2
#endif
template <int LOOP>
struct TileFetch {
  static constexpr int value = SWH_TILE_FETCH;
};

template <int SG, int TS, int NPAY>
struct TileLds {
  // per row: CR = TS*SG/64 slots + 1 pad slot, so the rows' broadcast reads
  // fall on different LDS banks
  double4 pos[TS + 64 / SG];  // x, y, z (image-shifted unless nearest-image), h
  int candj[TS + 64 / SG];
  int cell_j0[256];  // per row: 4*SG cells of the current batch
  int cell_pre[256];
  unsigned char cell_code[256];
  int hits[kTileCap * 64];  // [k][lane] global j
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

// Phase B: evaluate this lane's pending hits. The separation uses the
// nearest periodic image, which is the image phase A accepted (every hit lies
// within the reach, and the reach is < box/2 unless that dimension already
// used the nearest image).
template <bool PWRAP, typename T, class S, class LDS>
__device__ __forceinline__ void tile_drain(const GridDev& g, const SoA& a, const double4& pi,
                                           LDS& L, int& nh, int lane, S& st) {
  if (nh > 0) {
    int jn = L.hits[lane];
    double4 pn = a.pos[jn];
    JRec<S::kPay> rn = S::load_j(a, jn);
    for (int k = 0; k < nh; k++) {
      const double4 pj = pn;
      const JRec<S::kPay> rj = rn;
      if (k + 1 < nh) {  // issue the next hit's loads before this hit's math
        jn = L.hits[(k + 1) * 64 + lane];
        pn = a.pos[jn];
        rn = S::load_j(a, jn);
      }
      double dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
      if (PWRAP) {  // some candidate of this wave came through a periodic image
        dx = wrap_nearest(dx, g.dim[0]);
        dy = wrap_nearest(dy, g.dim[1]);
        dz = wrap_nearest(dz, g.dim[2]);
      }
      const T tdx = (T)dx, tdy = (T)dy, tdz = (T)dz;
      const T r2 = tdx * tdx + tdy * tdy + tdz * tdz;
      st.interact_staged(rj.p, rj.meta, pj, tdx, tdy, tdz, r2);
    }
  }
  nh = 0;
}

// Phase A over the staged regions (each row its own), in blocks of 8
// candidates: the block's LDS reads are all issued first, then the 8 tests,
// then the appends, so a block costs one LDS round trip, not eight. A lane's
// list holds <= kTileCap - 8 entries at the start of a block, so it never
// overflows. Slots past a row's count hold stale data and are masked.
template <int SG, bool WRAP, bool PWRAP, typename T, class S, class LDS>
__device__ __forceinline__ void tile_consume(const GridDev& g, const SoA& a, const CellRange& c,
                                             const double4& pi, bool act, int rbase, int nst,
                                             LDS& L, int& nh, int lane, S& st) {
  int kmax = nst;
  for (int o = 32; o >= SG; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
  for (int k0 = 0; k0 < kmax; k0 += 8) {
    if (__any(nh > kTileCap - 8)) tile_drain<PWRAP, T>(g, a, pi, L, nh, lane, st);
    double4 cv[8];
    int jv[8];
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
      cv[kk] = L.pos[rbase + k0 + kk];
      jv[kk] = L.candj[rbase + k0 + kk];
    }
    bool hit[8];
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
      double dx = pi.x - cv[kk].x, dy = pi.y - cv[kk].y, dz = pi.z - cv[kk].z;
      if (WRAP) {
        if (c.full[0]) dx = wrap_nearest(dx, g.dim[0]);
        if (c.full[1]) dy = wrap_nearest(dy, g.dim[1]);
        if (c.full[2]) dz = wrap_nearest(dz, g.dim[2]);
      }
      const T tdx = (T)dx, tdy = (T)dy, tdz = (T)dz;
      const T r2 = tdx * tdx + tdy * tdy + tdz * tdz;
      hit[kk] = act & (k0 + kk < nst) & st.accept(jv[kk], cv[kk], r2);
    }
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
      if (hit[kk]) L.hits[nh * 64 + lane] = jv[kk];
      nh += hit[kk] ? 1 : 0;
    }
  }
}

template <int LOOP, typename T, int SG, class LDS>
__device__ __forceinline__ void tile_loop(const GridDev& g, SoA& a,
                                          const int2* __restrict__ groups, int ngroups,
                                          int max_active_bin, T a2H,
                                          const unsigned int* __restrict__ hmax_bits,
                                          unsigned long long* counter, int* __restrict__ ncount,
                                          int diag, LDS& L) {
  using S = LoopState<LOOP, T>;
  constexpr int NS = 64 / SG;
  constexpr int TS = TileSlots<LOOP>::value;
  constexpr int CR = TS / NS;  // slots per row
  const int lane = threadIdx.x & 63;
  const int row = lane / SG, r = lane % SG;
  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so
  // workgroup w runs on XCD w % 8; give each XCD a contiguous stretch of the
  // Morton-ordered groups so neighbouring groups share that XCD's L2.
  const int nwg = gridDim.x;
  const int per_xcd = (nwg + 7) / 8;
  const int xcd = blockIdx.x % 8, slot_in_xcd = blockIdx.x / 8;
  const int full_xcds = nwg - (per_xcd - 1) * 8;  // XCDs that get per_xcd blocks
  const int wg = xcd < full_xcds ? xcd * per_xcd + slot_in_xcd
                                 : full_xcds * per_xcd + (xcd - full_xcds) * (per_xcd - 1) +
                                       slot_in_xcd;
  const int gid = wg * NS + row;
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
  constexpr int CT = 4 * SG;              // cell-table entries per row (4 per lane)
  constexpr int U = TileFetch<LOOP>::value;  // candidates per lane per fetch pass
  const int rbase = row * (CR + 1);  // this row's staged region (padded: rows on distinct banks)
  const int ctb = row * CT;    // this row's cell table
  // wave-uniform code paths: a nearest-image dimension anywhere (phase A
  // wraps), or any periodic image at all (the drain wraps)
  const bool wrap = __any(c.full[0] || c.full[1] || c.full[2]);
  const bool pwrap =
      g.periodic && __any(c.full[0] || c.full[1] || c.full[2] || c.lo[0] < 0 || c.lo[1] < 0 ||
                          c.lo[2] < 0 || c.hi[0] >= g.cdim[0] || c.hi[1] >= g.cdim[1] ||
                          c.hi[2] >= g.cdim[2]);
  int cb = 0, total = 0, base = 0, nst = 0, nh = 0, k = 0;
  for (;;) {
    if (!rdone && base >= total) {  // row-uniform: next batch of CT cells
      if (cb >= ncells) {
        rdone = true;
      } else {
        // every lane loads 4 consecutive cells' spans (independent loads)
        int cnt[4], j0[4], code[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int cl = cb + r * 4 + u;
          cnt[u] = 0;
          j0[u] = 0;
          code[u] = 0;
          if (cl < ncells) {
            double sx, sy, sz;
            const int wx = wrap_cell(g, c, 0, c.lo[0] + cl % nx, sx);
            const int wy = wrap_cell(g, c, 1, c.lo[1] + (cl / nx) % ny, sy);
            const int wz = wrap_cell(g, c, 2, c.lo[2] + cl / (nx * ny), sz);
            code[u] = (sx < 0. ? 1 : (sx > 0. ? 2 : 0)) |
                      ((sy < 0. ? 1 : (sy > 0. ? 2 : 0)) << 2) |
                      ((sz < 0. ? 1 : (sz > 0. ? 2 : 0)) << 4);
            const int2 sp = cell_range_of(g, wx, wy, wz);
            j0[u] = sp.x;
            cnt[u] = sp.y - sp.x;
          }
        }
        const int lsum = cnt[0] + cnt[1] + cnt[2] + cnt[3];
        int inc = lsum;
        for (int o = 1; o < SG; o <<= 1) {
          const int t = __shfl_up(inc, o, SG);
          if (r >= o) inc += t;
        }
        total = __shfl(inc, SG - 1, SG);
        int pre = inc - lsum;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          L.cell_j0[ctb + r * 4 + u] = j0[u];
          L.cell_pre[ctb + r * 4 + u] = pre;
          L.cell_code[ctb + r * 4 + u] = (unsigned char)code[u];
          pre += cnt[u];
        }
        base = 0;
        k = 0;
        cb += CT;
      }
    }
    if (__all(rdone)) break;
    wave_sync();
    // locate U candidates per lane (q = base + r + SG u; monotone per lane, so
    // a forward cursor over the cell prefixes replaces a search), then issue
    // all their loads before using any
    int jj[U], sc[U];
    bool val[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int q = base + r + SG * u;
      val[u] = !rdone && q < total;
      jj[u] = 0;
      sc[u] = 0;
      if (val[u]) {
        while (k + 1 < CT && L.cell_pre[ctb + k + 1] <= q) k++;
        jj[u] = L.cell_j0[ctb + k] + (q - L.cell_pre[ctb + k]);
        sc[u] = L.cell_code[ctb + k];
      }
    }
    double4 pp[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (val[u]) pp[u] = a.pos[jj[u]];
#pragma unroll
    for (int u = 0; u < U; u++) {
      bool keep = false;
      double4 p = pp[u];
      if (val[u]) {
        p.x += shift_of(sc[u] & 3, g.dim[0]);
        p.y += shift_of((sc[u] >> 2) & 3, g.dim[1]);
        p.z += shift_of((sc[u] >> 4) & 3, g.dim[2]);
        // exact distance from the group box (nearest-image dims not pruned)
        const double ex = c.full[0] ? 0. : fmax(fmax(lo[0] - p.x, p.x - hi[0]), 0.);
        const double ey = c.full[1] ? 0. : fmax(fmax(lo[1] - p.y, p.y - hi[1]), 0.);
        const double ez = c.full[2] ? 0. : fmax(fmax(lo[2] - p.z, p.z - hi[2]), 0.);
        const double rj = (LOOP == LOOP_FORCE) ? fmax(Hg, p.w * (double)kGamma) : Hg;
        keep = ex * ex + ey * ey + ez * ez <= rj * rj;
      }
      const unsigned long long m = __ballot(keep);
      const unsigned long long rowbits =
          SG == 64 ? m : (m >> (row * SG)) & ((1ull << (SG & 63)) - 1ull);
      if (keep) {
        const int slot = rbase + nst + __popcll(rowbits & ((1ull << r) - 1ull));
        L.pos[slot] = p;
        L.candj[slot] = jj[u];
      }
      nst += __popcll(rowbits);
    }
    if (!rdone) base += SG * U;
    if (__any(nst > CR - SG * U)) {
      wave_sync();
      if (diag == 1) {
        nst = 0;
        continue;
      }
      if (diag == 2) nh = 0;
      if (wrap)
        tile_consume<SG, true, true, T>(g, a, c, pi, act, rbase, nst, L, nh, lane, st);
      else if (pwrap)
        tile_consume<SG, false, true, T>(g, a, c, pi, act, rbase, nst, L, nh, lane, st);
      else
        tile_consume<SG, false, false, T>(g, a, c, pi, act, rbase, nst, L, nh, lane, st);
      nst = 0;
    }
    wave_sync();
  }
  wave_sync();
  if (diag == 1) nst = 0;
  if (diag == 2) nh = 0;
  if (wrap) {
    tile_consume<SG, true, true, T>(g, a, c, pi, act, rbase, nst, L, nh, lane, st);
    tile_drain<true, T>(g, a, pi, L, nh, lane, st);
  } else if (pwrap) {
    tile_consume<SG, false, true, T>(g, a, c, pi, act, rbase, nst, L, nh, lane, st);
    tile_drain<true, T>(g, a, pi, L, nh, lane, st);
  } else {
    tile_consume<SG, false, false, T>(g, a, c, pi, act, rbase, nst, L, nh, lane, st);
    tile_drain<false, T>(g, a, pi, L, nh, lane, st);
  }
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
