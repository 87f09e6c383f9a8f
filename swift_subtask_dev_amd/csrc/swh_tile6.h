// swh_tile6.h — balanced phase B for the fp32-test tile loop (loop variant 6).
//
// Variant 4 (swh_tile4.h) drains each lane's own hit list: a drain costs the
// LONGEST list of the wave, and with octree leaves of ~11 particles in 16-lane
// rows plus list-length spread only ~31% of the lanes do an interaction per
// phase-B step (measured: 98.5 M interactions in 4.9 M wave steps at 128^3).
// Here a drain deals the wave's hits out over all 64 lanes instead:
//   * a chunk length C is chosen (the smallest tried, from ceil(total/64) up)
//     with sum_o ceil(nh_o / C) <= 64, and owner o (the lane whose list it is)
//     gets m_o = ceil(nh_o / C) consecutive lanes, each taking C consecutive
//     hits of o's list; every lane serves ONE owner, so it loads o's i-state
//     once per drain (no per-hit owner switches);
//   * each lane's partial accumulator goes to LDS part[lane]; owner o adds the
//     partials of its m_o lanes in lane order to its register accumulator, so
//     the sums are deterministic.
// A drain costs C steps instead of the longest list of the wave.
// The pair set and the per-pair arithmetic are those of variant 4 (exact fp64
// re-test of every fp32 hit, runner_doiact_functions_hydro.h:1143-1150,
// 1642-1660); only the order of the fp64 additions within a sum differs.
#pragma once

#include <cfloat>
#include <climits>

#include "swh_tile4.h"

namespace swh {

template <int SG, int TS, class ACC>
struct Tile6Lds : Tile4Lds<SG, TS> {
  int bpre[65];   // first lane of each owner's chunks; bpre[64] = lanes in use
  int cnt[64];     // list length of each owner
  int own_i[64];   // particle of each lane (-1: none)
  ACC part[64];    // partial accumulator of each lane's chunk
  int partn[64];   // interaction counts of the partials
};

// Identity and combination of the loops' accumulators (sums add; v_sig and
// alpha_visc_max_ngb take the max; the limiter takes the min).
template <typename T>
__device__ __forceinline__ void acc_reset(DensityAcc<T>& A) { A.zero(); }
template <typename T>
__device__ __forceinline__ void acc_add(DensityAcc<T>& d, const DensityAcc<T>& s) {
  d.rho += s.rho;
  d.rho_dh += s.rho_dh;
  d.wcount += s.wcount;
  d.wcount_dh += s.wcount_dh;
  d.div_v += s.div_v;
  d.rot_x += s.rot_x;
  d.rot_y += s.rot_y;
  d.rot_z += s.rot_z;
}
template <typename T>
__device__ __forceinline__ void acc_reset(GradientAcc<T>& A) {
  A.v_sig = (T)-FLT_MAX;
  A.alpha_visc_max_ngb = (T)-FLT_MAX;
  A.laplace_u = (T)0;
}
template <typename T>
__device__ __forceinline__ void acc_add(GradientAcc<T>& d, const GradientAcc<T>& s) {
  d.v_sig = tmax(d.v_sig, s.v_sig);
  d.alpha_visc_max_ngb = tmax(d.alpha_visc_max_ngb, s.alpha_visc_max_ngb);
  d.laplace_u += s.laplace_u;
}
template <typename T>
__device__ __forceinline__ void acc_reset(ForceAcc<T>& A) {
  A.ax = A.ay = A.az = A.u_dt = A.h_dt = (T)0;
  A.min_ngb_time_bin = INT_MAX;
}
template <typename T>
__device__ __forceinline__ void acc_add(ForceAcc<T>& d, const ForceAcc<T>& s) {
  d.ax += s.ax;
  d.ay += s.ay;
  d.az += s.az;
  d.u_dt += s.u_dt;
  d.h_dt += s.h_dt;
  d.min_ngb_time_bin = min(d.min_ngb_time_bin, s.min_ngb_time_bin);
}

template <bool PWRAP, typename T, class S, class LDS>
__device__ __forceinline__ void tile6_drain(const GridDev& g, const SoA& a, LDS& L, int& nh,
                                            int lane, S& st, TileStats& ts, T a2H,
                                            const unsigned int* __restrict__ hmax_bits) {
  int total = nh;
  for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o);
  if (total == 0) return;  // wave-uniform
  // chunk length C: the smallest tried with sum_o ceil(nh_o / C) <= 64 lanes
  int C = (total + 63) >> 6;
  int m, M;
  for (;;) {
    m = (nh + C - 1) / C;
    M = m;
    for (int o = 32; o > 0; o >>= 1) M += __shfl_xor(M, o);
    if (M <= 64) break;
    C = max(C + 1, (C * M + 63) / 64);
  }
  int inc = m;
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o);
    if (lane >= o) inc += t;
  }
  const int first = inc - m;  // first lane of this owner's chunks
  ts.bsteps += (unsigned int)C;
  L.bpre[lane] = first;
  L.cnt[lane] = nh;
  if (lane == 63) L.bpre[64] = M;
  wave_sync();
  if (lane < M) {
    // owner of lane: the largest o with bpre[o] <= lane (m_o > 0)
    int lo = 0, hi = 63;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (L.bpre[mid] <= lane) lo = mid;
      else hi = mid - 1;
    }
    const int o = lo;
    const int p0 = (lane - L.bpre[o]) * C;
    const int p1 = min(p0 + C, L.cnt[o]);
    const int io = L.own_i[o];
    S cur;
    cur.load_i(a, io, a2H, hmax_bits);
    acc_reset(cur.A);
    const double4 pi = a.pos[io];
    int jn = L.hits[p0 * 64 + o];
    double4 pn = a.pos[jn];
    JRec<S::kPay> rn = S::load_j(a, jn);
    for (int p = p0; p < p1; p++) {
      const int j = jn;
      const double4 pj = pn;
      const JRec<S::kPay> rj = rn;
      if (p + 1 < p1) {  // issue the next hit's loads before this hit's math
        jn = L.hits[(p + 1) * 64 + o];
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
      if (cur.accept(j, pj, r2)) cur.interact_staged(rj.p, rj.meta, pj, tdx, tdy, tdz, r2);
    }
    L.part[lane] = cur.A;
    L.partn[lane] = cur.n;
  }
  wave_sync();
  if (nh > 0) {  // owner: combine its chunks in lane order
    auto R = L.part[first];
    int rn = L.partn[first];
    for (int k = first + 1; k < first + m; k++) {
      acc_add(R, L.part[k]);
      rn += L.partn[k];
    }
    acc_add(st.A, R);
    st.n += rn;
  }
  nh = 0;
  wave_sync();
}

}  // namespace swh
