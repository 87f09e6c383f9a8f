// swh_tile4.h — the tile neighbour loop with fp32 candidate tests (loop
// variant 4).
//
// Same skeleton as swh_tile.h (one 64-lane wave serves NS = 64/SG i-groups,
// one per SG-lane row: staging -> phase A -> phase B), with the candidate side
// of phase A in fp32 (a wave64 f32 VALU op issues in half the cycles of an f64
// one) and a staged record of 20 B instead of 36 B:
//   staging : each candidate is stored relative to its row's centre c as
//             floats, (x_j - c) rounded once from fp64; the prune against the
//             row box uses the same floats, widened by the rounding bound;
//   phase A : r2 of every (i, candidate) of the row in fp32, accepted when
//             below (H + 16 u D)^2 (1 + 8u) (u = 2^-24, D bounds |x - c| over
//             the row's i and candidates: the worst-case error of the rounded
//             separation), so the hit lists are a superset of the exact hits;
//   phase B : re-tests every hit with the loop's exact fp64 criterion
//             (DOPAIR1/DOSELF1: r < H_i; DOPAIR2/DOSELF2: r < max(H_i, H_j);
//             j != i; runner_doiact_functions_hydro.h:1143-1150, 1642-1660)
//             before the fp64 iact, so the accepted pair set is exactly the
//             one of variants 1-3 and of the f64 oracle.
#pragma once

#include "swh_tile.h"

namespace swh {

constexpr double kUnitRound = 5.9604644775390625e-8;   // u = 2^-24
constexpr float kThrSlack = 1.f + 8.f * 5.9604645e-8f;  // (1 + 8u)

// Per-lane hit-list capacity of variant 4: 64 (measured at 128^3:
// force 2.46 ms at 64, 2.75 ms at 48, 2.97 ms at 32; density 1.72 / 1.65 / 1.74).
#ifndef SWH_TILE4_CAP
#define SWH_TILE4_CAP 64
#endif
constexpr int kTile4Cap = SWH_TILE4_CAP;

template <int SG, int TS>
struct Tile4Lds {
  static constexpr int kSlots = TS + 4 * (64 / SG);  // rows padded by 4 slots
  float4 cand[kSlots];  // x, y, z relative to the row centre; w = force: inflated H_j^2
  int candj[kSlots];
  int cell_j0[256];  // per row: 4*SG cells of the current batch
  int cell_pre[256];
  unsigned char cell_code[256];
  int hits[kTile4Cap * 64];  // [k][lane] global j
};

// Work counters of a counted launch (swh_space_info.loop_stats): candidates
// loaded, candidates staged, phase-A candidate steps and phase-B hit steps,
// both per wave (every lane of the wave executes them).
struct TileStats {
  unsigned int loaded = 0, staged = 0, asteps = 0, bsteps = 0;
};

__device__ __forceinline__ float wrap_nearest_f(float d, float box) {
  return d > 0.5f * box ? d - box : (d < -0.5f * box ? d + box : d);
}

// Phase B: evaluate this lane's pending hits that pass the exact criterion.
template <bool PWRAP, typename T, class S, class LDS>
__device__ __forceinline__ void tile4_drain(const GridDev& g, const SoA& a, const double4& pi,
                                            LDS& L, int& nh, int lane, S& st, TileStats& ts) {
  int wmax = nh;
  for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, __shfl_xor(wmax, o));
  ts.bsteps += (unsigned int)wmax;
  if (nh > 0) {
    int jn = L.hits[lane];
    double4 pn = a.pos[jn];
    JRec<S::kPay> rn = S::load_j(a, jn);
    for (int k = 0; k < nh; k++) {
      const int j = jn;
      const double4 pj = pn;
      const JRec<S::kPay> rj = rn;
      if (k + 1 < nh) {  // issue the next hit's loads before this hit's math
        jn = L.hits[(k + 1) * 64 + lane];
        pn = a.pos[jn];
        rn = S::load_j(a, jn);
      }
      double dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
      if (PWRAP) {
        dx = wrap_nearest(dx, g.dim[0]);
        dy = wrap_nearest(dy, g.dim[1]);
        dz = wrap_nearest(dz, g.dim[2]);
      }
      const T tdx = (T)dx, tdy = (T)dy, tdz = (T)dz;
      const T r2 = tdx * tdx + tdy * tdy + tdz * tdz;
      if (st.accept(j, pj, r2)) st.interact_staged(rj.p, rj.meta, pj, tdx, tdy, tdz, r2);
    }
  }
  nh = 0;
}

// Phase A over the staged region of each row, 8 candidates per block. A
// lane's list holds <= kTile4Cap - 8 entries at the start of a block; every
// candidate's j is written at the list end and kept only on a hit, so the
// appends need no branch.
template <int LOOP, int SG, bool WRAP, bool PWRAP, typename T, class S, class LDS>
__device__ __forceinline__ void tile4_consume(const GridDev& g, const SoA& a,
                                              const CellRange& c, const double4& pi, float xi,
                                              float yi, float zi, float thr_i, bool act,
                                              int rbase, int nst, LDS& L, int& nh, int lane,
                                              S& st, TileStats& ts, T a2H,
                                              const unsigned int* hmax_bits) {
  int kmax = nst;
  for (int o = 32; o >= SG; o >>= 1) kmax = max(kmax, __shfl_xor(kmax, o));
  ts.asteps += (unsigned int)kmax;
  const float bx = (float)g.dim[0], by = (float)g.dim[1], bz = (float)g.dim[2];
  for (int k0 = 0; k0 < kmax; k0 += 8) {
    if (__any(nh > kTile4Cap - 8))
      tile4_drain<PWRAP, T>(g, a, pi, L, nh, lane, st, ts);
    float4 cv[8];
#pragma unroll
    for (int kk = 0; kk < 8; kk++) cv[kk] = L.cand[rbase + k0 + kk];
    const int4 J0 = *reinterpret_cast<const int4*>(&L.candj[rbase + k0]);
    const int4 J1 = *reinterpret_cast<const int4*>(&L.candj[rbase + k0 + 4]);
    const int lim = act ? nst - k0 : 0;  // valid candidates of this block
    bool hit[8];
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
      float dx = xi - cv[kk].x, dy = yi - cv[kk].y, dz = zi - cv[kk].z;
      if (WRAP) {
        if (c.full[0]) dx = wrap_nearest_f(dx, bx);
        if (c.full[1]) dy = wrap_nearest_f(dy, by);
        if (c.full[2]) dz = wrap_nearest_f(dz, bz);
      }
      float r2 = dx * dx;
      r2 = fmaf(dy, dy, r2);
      r2 = fmaf(dz, dz, r2);
      const float thr = (LOOP == LOOP_FORCE) ? fmaxf(thr_i, cv[kk].w) : thr_i;
      hit[kk] = (r2 < thr) & (kk < lim);
    }
    const int jv[8] = {J0.x, J0.y, J0.z, J0.w, J1.x, J1.y, J1.z, J1.w};
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
      L.hits[nh * 64 + lane] = jv[kk];
      nh += hit[kk] ? 1 : 0;
    }
  }
}

template <int LOOP, typename T, int SG, class LDS>
__device__ __forceinline__ void tile4_loop(const GridDev& g, SoA& a,
                                           const int2* __restrict__ groups, int ngroups,
                                           int max_active_bin, T a2H,
                                           const unsigned int* __restrict__ hmax_bits,
                                           unsigned long long* counter, int* __restrict__ ncount,
                                           int diag, LDS& L) {
  using S = LoopState<LOOP, T>;
  constexpr int NS = 64 / SG;
  constexpr int TS = TileSlots<LOOP>::value;
  constexpr int CR = TS / NS;  // slots per row
  constexpr int RP = CR + 4;   // row stride (keeps int4 alignment, staggers LDS banks)
  const int lane = threadIdx.x & 63;
  const int row = lane / SG, r = lane % SG;
  // XCD-aware order (swh_tile.h): each XCD takes a contiguous stretch of the
  // Morton-ordered groups so neighbouring groups share its L2.
  const int wg = xcd_block_id();
  const int gid = wg * NS + row;
  const int2 gr = gid < ngroups ? groups[gid] : make_int2(0, 0);
  const int i = r < gr.y ? gr.x + r : -1;
  const bool act = i >= 0 && active_part(a, i, max_active_bin);
  S st;
  st.n = 0;
  double4 pi = make_double4(0., 0., 0., 0.);
  if (act) {
    st.load_i(a, i, a2H, hmax_bits);
    pi = a.pos[i];
  }
  const double Hi = act ? pi.w * (double)kGamma : 0.;
  const double Hg = row_max<SG>(Hi);
  double lo[3], hi[3];
  lo[0] = row_min<SG>(act ? pi.x : 1e300);
  lo[1] = row_min<SG>(act ? pi.y : 1e300);
  lo[2] = row_min<SG>(act ? pi.z : 1e300);
  hi[0] = row_max<SG>(act ? pi.x : -1e300);
  hi[1] = row_max<SG>(act ? pi.y : -1e300);
  hi[2] = row_max<SG>(act ? pi.z : -1e300);
  bool rdone = !(Hg > 0.);
  const double hmax_reach = (double)__uint_as_float(*hmax_bits) * (double)kGamma;
  const double reach = ((LOOP == LOOP_FORCE) ? fmax(Hg, hmax_reach) : Hg) + g.dx;
  CellRange c;
  int nx = 1, ny = 1, ncells = 0;
  for (int k = 0; k < 3; k++) {
    c.full[k] = false;
    c.lo[k] = c.hi[k] = 0;
  }
  // row frame: centre, half extents, and D >= |x - centre| over the row's i
  // and candidates (bounds the rounding of the fp32 relative coordinates)
  double ctr[3] = {0., 0., 0.}, half[3] = {0., 0., 0.};
  double D2 = 0.;
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
      ctr[k] = 0.5 * (lo[k] + hi[k]);
      half[k] = 0.5 * (hi[k] - lo[k]);
      const double ext = c.full[k] ? g.dim[k] : half[k] + reach;
      D2 += ext * ext;
    }
    nx = c.hi[0] - c.lo[0] + 1;
    ny = c.hi[1] - c.lo[1] + 1;
    ncells = nx * ny * (c.hi[2] - c.lo[2] + 1);
  }
  const double delta = 16. * kUnitRound * sqrt(D2);
  const float deltaf = (float)delta;
  // phase-A operands of this lane: i relative to the row centre, threshold
  const float xi = (float)(pi.x - ctr[0]);
  const float yi = (float)(pi.y - ctr[1]);
  const float zi = (float)(pi.z - ctr[2]);
  const float thr_i = act ? (float)((Hi + delta) * (Hi + delta)) * kThrSlack : -1.f;
  // staging prune: the row box widened by delta, reach Hg (force: max(Hg, H_j))
  const float hxf = (float)(half[0] + delta), hyf = (float)(half[1] + delta),
              hzf = (float)(half[2] + delta);
  const float Hgf = (float)(Hg + delta);
  constexpr int CT = 4 * SG;
  constexpr int U = TileFetch<LOOP>::value;
  const int rbase = row * RP;
  const int ctb = row * CT;
  const bool wrap = __any(c.full[0] || c.full[1] || c.full[2]);
  const bool pwrap =
      g.periodic && __any(c.full[0] || c.full[1] || c.full[2] || c.lo[0] < 0 || c.lo[1] < 0 ||
                          c.lo[2] < 0 || c.hi[0] >= g.cdim[0] || c.hi[1] >= g.cdim[1] ||
                          c.hi[2] >= g.cdim[2]);
  TileStats ts;
  int cb = 0, total = 0, base = 0, nst = 0, nh = 0, k = 0;
  for (;;) {
    if (!rdone && base >= total) {  // row-uniform: next batch of CT cells
      if (cb >= ncells) {
        rdone = true;
      } else {
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
      float4 cf = make_float4(0.f, 0.f, 0.f, 0.f);
      if (val[u]) {
        const double4 p = pp[u];
        double rx = p.x + shift_of(sc[u] & 3, g.dim[0]) - ctr[0];
        double ry = p.y + shift_of((sc[u] >> 2) & 3, g.dim[1]) - ctr[1];
        double rz = p.z + shift_of((sc[u] >> 4) & 3, g.dim[2]) - ctr[2];
        if (c.full[0]) rx = wrap_nearest(rx, g.dim[0]);
        if (c.full[1]) ry = wrap_nearest(ry, g.dim[1]);
        if (c.full[2]) rz = wrap_nearest(rz, g.dim[2]);
        cf.x = (float)rx;
        cf.y = (float)ry;
        cf.z = (float)rz;
        // distance from the (widened) row box; nearest-image dims not pruned
        const float ex = c.full[0] ? 0.f : fmaxf(fabsf(cf.x) - hxf, 0.f);
        const float ey = c.full[1] ? 0.f : fmaxf(fabsf(cf.y) - hyf, 0.f);
        const float ez = c.full[2] ? 0.f : fmaxf(fabsf(cf.z) - hzf, 0.f);
        float rj = Hgf;
        if (LOOP == LOOP_FORCE) {
          const float hj = (float)(p.w * (double)kGamma) + deltaf;
          cf.w = hj * hj * kThrSlack;
          rj = fmaxf(Hgf, hj);
        }
        keep = ex * ex + ey * ey + ez * ez <= rj * rj * kThrSlack;
      }
      const unsigned long long m = __ballot(keep);
      const unsigned long long rowbits =
          SG == 64 ? m : (m >> (row * SG)) & ((1ull << (SG & 63)) - 1ull);
      if (keep) {
        const int slot = rbase + nst + __popcll(rowbits & ((1ull << r) - 1ull));
        L.cand[slot] = cf;
        L.candj[slot] = jj[u];
      }
      nst += __popcll(rowbits);
      ts.loaded += val[u] ? 1u : 0u;
      ts.staged += keep ? 1u : 0u;
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
        tile4_consume<LOOP, SG, true, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act, rbase, nst,
                                               L, nh, lane, st, ts, a2H, hmax_bits);
      else if (pwrap)
        tile4_consume<LOOP, SG, false, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act, rbase, nst,
                                                L, nh, lane, st, ts, a2H, hmax_bits);
      else
        tile4_consume<LOOP, SG, false, false, T>(g, a, c, pi, xi, yi, zi, thr_i, act, rbase,
                                                 nst, L, nh, lane, st, ts, a2H, hmax_bits);
      nst = 0;
    }
    wave_sync();
  }
  wave_sync();
  if (diag == 1) nst = 0;
  if (diag == 2) nh = 0;
  if (wrap) {
    tile4_consume<LOOP, SG, true, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act, rbase, nst, L,
                                           nh, lane, st, ts, a2H, hmax_bits);
    tile4_drain<true, T>(g, a, pi, L, nh, lane, st, ts);
  } else if (pwrap) {
    tile4_consume<LOOP, SG, false, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act, rbase, nst, L,
                                            nh, lane, st, ts, a2H, hmax_bits);
    tile4_drain<true, T>(g, a, pi, L, nh, lane, st, ts);
  } else {
    tile4_consume<LOOP, SG, false, false, T>(g, a, c, pi, xi, yi, zi, thr_i, act, rbase, nst,
                                             L, nh, lane, st, ts, a2H, hmax_bits);
    tile4_drain<false, T>(g, a, pi, L, nh, lane, st, ts);
  }
  if (act) {
    st.store(a, i);
    if (ncount) ncount[i] = st.n;
  }
  if (counter) {
    unsigned long long v = (unsigned long long)(act ? st.n : 0);
    unsigned long long ld = ts.loaded, sg = ts.staged;
    for (int o = 32; o > 0; o >>= 1) {
      v += __shfl_xor(v, o);
      ld += __shfl_xor(ld, o);
      sg += __shfl_xor(sg, o);
    }
    if (lane == 0) {
      if (v) atomicAdd(counter, v);
      atomicAdd(counter + 4, ld);
      atomicAdd(counter + 5, sg);
      atomicAdd(counter + 6, (unsigned long long)ts.asteps);
      atomicAdd(counter + 7, (unsigned long long)ts.bsteps);
    }
  }
}

}  // namespace swh
