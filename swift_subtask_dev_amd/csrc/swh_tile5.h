// swh_tile5.h — the group-per-wave neighbour loop (loop variant 5).
//
// One 64-lane wave serves ONE i-group (an octree leaf of <= 64/LPI particles,
// swh_space.hip group_kernel) with LPI lanes per i-particle. Everything that
// belongs to the group (its box, reach, cell range, staging cursor, region
// fill) is wave-uniform and lives in SGPRs, which keeps the VGPR budget low
// enough for more waves per SIMD than swh_tile.h / swh_tile4.h (four groups
// per wave, their row state in VGPRs: 2 waves per SIMD).
//   staging : the wave enumerates the cells overlapping the group box grown
//             by the reach (64 cells per batch, one per lane, prefix-summed),
//             streams their particles 64*U at a time and appends the ones
//             within reach of the box (fp32 coordinates relative to the box
//             centre, as swh_tile4.h) to one LDS region;
//   phase A : sub-lane s of i tests slots s, s+LPI, ... of the region in fp32
//             with the inflated threshold of swh_tile4.h and appends the hits'
//             region slots to i's list, shared by its LPI lanes (a prefix sum
//             over the LPI lanes gives each lane its positions);
//   phase B : at every region turnover the LPI lanes of i split i's list
//             round-robin, re-test each hit with the loop's exact fp64
//             criterion (runner_doiact_functions_hydro.h:1143-1150,
//             1642-1660) and evaluate the fp64 iact; the LPI partial sums are
//             combined at the end.
// The accepted pair set is exactly the f64 oracle's (and variants 1-4's).
#pragma once

#include "swh_tile4.h"

namespace swh {

constexpr int kT5Region = 256;  // staged candidates per region
#ifndef SWH_T5_KB
#define SWH_T5_KB 8
#endif
constexpr int kT5Blk = SWH_T5_KB;  // phase-A candidates per lane per block
#ifndef SWH_T5_U
#define SWH_T5_U 1
#endif

template <int LPI>
struct Tile5Lds {
  static constexpr int GS = 64 / LPI;
  static constexpr int kICap = LPI >= 4 ? 128 : (LPI == 2 ? 96 : 48);  // list entries per i
  static constexpr int kStride = kICap + 2;  // odd dword stride: lists start on different banks
  float4 cand[kT5Region];  // x, y, z relative to the box centre; w = force: inflated H_j^2
  int candj[kT5Region];
  int cell_j0[64];
  int cell_pre[64];
  unsigned char cell_code[64];
  unsigned short hits[GS * kStride + 64];  // [i slot][entry] region slots; + per-lane dummies
};

__device__ __forceinline__ int uni_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uni_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ double uni_d(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned int lo = (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)b);
  const unsigned int hi =
      (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double wave_min_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// Stream compaction with one atomic per workgroup (blockDim.x <= 1024): the
// threads with `pred` get consecutive slots, in thread order. Every thread of
// the block must call it (it synchronises the block). Same-address atomics
// serialise in L2, so per-wave appends of millions of items cost ~0.3 ms.
template <typename C>
__device__ __forceinline__ int block_append(bool pred, C* counter) {
  __shared__ int wcnt[16];
  __shared__ int wbase[16];
  const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
  const int nw = (int)((blockDim.x + 63) >> 6);
  const unsigned long long m = __ballot(pred);
  if (lane == 0) wcnt[w] = (int)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int k = 0; k < nw; k++) {
      wbase[k] = tot;
      tot += wcnt[k];
    }
    const int b = tot ? (int)atomicAdd(counter, (C)tot) : 0;
    for (int k = 0; k < nw; k++) wbase[k] += b;
  }
  __syncthreads();
  return pred ? wbase[w] + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// Stream compaction with one atomic per wave: the lanes with `pred` get
// consecutive slots (in lane order) of the list whose length is *counter.
// Every lane of the wave must call it.
template <typename C>
__device__ __forceinline__ int wave_append(bool pred, C* counter) {
  const unsigned long long m = __ballot(pred);
  if (m == 0ull) return -1;
  const int lane = (int)(threadIdx.x & 63);
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = (int)atomicAdd(counter, (C)__popcll(m));
  base = __shfl(base, leader);
  return pred ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// Combine the LPI partial states of one i-particle (lanes differing in the
// low log2(LPI) bits): sums add, v_sig / alpha_max take the max, the limiter
// takes the min.
template <int W, typename T>
__device__ __forceinline__ void reduce_lanes(LoopState<LOOP_DENSITY, T>& s) {
  for (int o = 1; o < W; o <<= 1) {
    s.A.rho += __shfl_xor(s.A.rho, o);
    s.A.rho_dh += __shfl_xor(s.A.rho_dh, o);
    s.A.wcount += __shfl_xor(s.A.wcount, o);
    s.A.wcount_dh += __shfl_xor(s.A.wcount_dh, o);
    s.A.div_v += __shfl_xor(s.A.div_v, o);
    s.A.rot_x += __shfl_xor(s.A.rot_x, o);
    s.A.rot_y += __shfl_xor(s.A.rot_y, o);
    s.A.rot_z += __shfl_xor(s.A.rot_z, o);
    s.n += __shfl_xor(s.n, o);
  }
}
template <int W, typename T>
__device__ __forceinline__ void reduce_lanes(LoopState<LOOP_GRADIENT, T>& s) {
  for (int o = 1; o < W; o <<= 1) {
    s.A.v_sig = tmax(s.A.v_sig, (T)__shfl_xor(s.A.v_sig, o));
    s.A.alpha_visc_max_ngb =
        tmax(s.A.alpha_visc_max_ngb, (T)__shfl_xor(s.A.alpha_visc_max_ngb, o));
    s.A.laplace_u += __shfl_xor(s.A.laplace_u, o);
    s.n += __shfl_xor(s.n, o);
  }
}
template <int W, typename T>
__device__ __forceinline__ void reduce_lanes(LoopState<LOOP_FORCE, T>& s) {
  for (int o = 1; o < W; o <<= 1) {
    s.A.ax += __shfl_xor(s.A.ax, o);
    s.A.ay += __shfl_xor(s.A.ay, o);
    s.A.az += __shfl_xor(s.A.az, o);
    s.A.u_dt += __shfl_xor(s.A.u_dt, o);
    s.A.h_dt += __shfl_xor(s.A.h_dt, o);
    s.A.min_ngb_time_bin = min(s.A.min_ngb_time_bin, __shfl_xor(s.A.min_ngb_time_bin, o));
    s.n += __shfl_xor(s.n, o);
  }
}

// Phase B: the LPI lanes of each i split its list round-robin.
template <int LPI, bool PWRAP, typename T, class S, class LDS>
__device__ __forceinline__ void tile5_drain(const GridDev& g, const SoA& a, const double4& pi,
                                            LDS& L, int& nq, int il, int s, S& st,
                                            TileStats& ts) {
  wave_sync();  // list entries were written by the other lanes of i
  const int nmax = uni_i(wave_max_i(nq));
  const int steps = (nmax + LPI - 1) / LPI;
  ts.bsteps += (unsigned int)steps;
  if (steps > 0) {
    const unsigned short* list = &L.hits[il * LDS::kStride];
    int t = s;
    int jn = t < nq ? L.candj[list[t]] : -1;
    double4 pn = make_double4(0., 0., 0., 0.);
    JRec<S::kPay> rn{};
    if (jn >= 0) {
      pn = a.pos[jn];
      rn = S::load_j(a, jn);
    }
    for (int q = 0; q < steps; q++) {
      const int j = jn;
      const double4 pj = pn;
      const JRec<S::kPay> rj = rn;
      t += LPI;
      jn = t < nq ? L.candj[list[t]] : -1;  // issue the next hit's loads first
      if (jn >= 0) {
        pn = a.pos[jn];
        rn = S::load_j(a, jn);
      }
      if (j >= 0) {
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
  }
  nq = 0;
  wave_sync();
}

// Phase A over the region [0, nst), then phase B. Sub-lane s tests slots
// s + LPI*m, 8 slots per lane per block; every lane writes 8 list entries per
// block, the misses to its own dummy slot (no branch).
template <int LOOP, int LPI, bool WRAP, bool PWRAP, typename T, class S, class LDS>
__device__ __forceinline__ void tile5_consume(const GridDev& g, const SoA& a,
                                              const CellRange& c, const double4& pi, float xi,
                                              float yi, float zi, float thr_i, bool act,
                                              int nst, LDS& L, int& nq, int il, int s, S& st,
                                              TileStats& ts) {
  constexpr int GS = 64 / LPI;
  const int dummy = GS * LDS::kStride + il * LPI + s;
  const int nblk = (nst + kT5Blk * LPI - 1) / (kT5Blk * LPI);
  ts.asteps += (unsigned int)(nblk * kT5Blk);
  const float bx = (float)g.dim[0], by = (float)g.dim[1], bz = (float)g.dim[2];
  for (int b = 0; b < nblk; b++) {
    if (__any(nq > LDS::kICap - kT5Blk * LPI))
      tile5_drain<LPI, PWRAP, T>(g, a, pi, L, nq, il, s, st, ts);
    const int c0 = b * kT5Blk * LPI + s;
    float4 cv[kT5Blk];
#pragma unroll
    for (int kk = 0; kk < kT5Blk; kk++) cv[kk] = L.cand[min(c0 + kk * LPI, kT5Region - 1)];
    bool hit[kT5Blk];
    int cnt = 0;
#pragma unroll
    for (int kk = 0; kk < kT5Blk; kk++) {
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
      hit[kk] = act & (c0 + kk * LPI < nst) & (r2 < thr);
      cnt += hit[kk] ? 1 : 0;
    }
    // this lane's first position in i's list: i's count + earlier sub-lanes' hits
    int inc = cnt;
    for (int o = 1; o < LPI; o <<= 1) {
      const int tt = __shfl_up(inc, o, LPI);
      if (s >= o) inc += tt;
    }
    const int tot = __shfl(inc, LPI - 1, LPI);
    int pos = il * LDS::kStride + nq + inc - cnt;
#pragma unroll
    for (int kk = 0; kk < kT5Blk; kk++) {
      L.hits[hit[kk] ? pos : dummy] = (unsigned short)(c0 + kk * LPI);
      pos += hit[kk] ? 1 : 0;
    }
    nq += tot;
  }
  tile5_drain<LPI, PWRAP, T>(g, a, pi, L, nq, il, s, st, ts);
}

template <int LOOP, typename T, int LPI, class LDS>
__device__ __forceinline__ void tile5_loop(const GridDev& g, SoA& a,
                                           const int2* __restrict__ groups, int ngroups,
                                           int max_active_bin, T a2H,
                                           const unsigned int* __restrict__ hmax_bits,
                                           unsigned long long* counter, int* __restrict__ ncount,
                                           int diag, LDS& L) {
  using S = LoopState<LOOP, T>;
  constexpr int U = SWH_T5_U;  // candidates per lane per staging pass
  const int lane = threadIdx.x & 63;
  const int il = lane / LPI, s = lane % LPI;
  // XCD-aware order (swh_tile.h): each XCD takes a contiguous stretch of the
  // Morton-ordered groups so neighbouring groups share its L2.
  const int gid = xcd_block_id();
  const int2 gr = gid < ngroups ? groups[gid] : make_int2(0, 0);
  const int i = il < gr.y ? gr.x + il : -1;
  const bool act = i >= 0 && active_part(a, i, max_active_bin);
  S st;
  st.n = 0;
  double4 pi = make_double4(0., 0., 0., 0.);
  if (act) {
    st.load_i(a, i, a2H, hmax_bits);
    pi = a.pos[i];
  }
  const double Hi = act ? pi.w * (double)kGamma : 0.;
  // group box and reach (wave-uniform)
  const double Hg = uni_d(wave_max_d(Hi));
  double lo[3], hi[3];
  lo[0] = uni_d(wave_min_d(act ? pi.x : 1e300));
  lo[1] = uni_d(wave_min_d(act ? pi.y : 1e300));
  lo[2] = uni_d(wave_min_d(act ? pi.z : 1e300));
  hi[0] = uni_d(wave_max_d(act ? pi.x : -1e300));
  hi[1] = uni_d(wave_max_d(act ? pi.y : -1e300));
  hi[2] = uni_d(wave_max_d(act ? pi.z : -1e300));
  TileStats ts;
  if (Hg > 0.) {
    const double hmax_reach = (double)__uint_as_float(*hmax_bits) * (double)kGamma;
    const double reach = ((LOOP == LOOP_FORCE) ? fmax(Hg, hmax_reach) : Hg) + g.dx;
    CellRange c;
    double ctr[3], half[3];
    double D2 = 0.;
    for (int k = 0; k < 3; k++) {
      c.lo[k] = uni_i((int)floor((lo[k] - g.origin[k] - reach) * g.inv_w[k]));
      c.hi[k] = uni_i((int)floor((hi[k] - g.origin[k] + reach) * g.inv_w[k]));
      c.full[k] = false;
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
      ctr[k] = uni_d(0.5 * (lo[k] + hi[k]));
      half[k] = 0.5 * (hi[k] - lo[k]);
      const double ext = c.full[k] ? g.dim[k] : half[k] + reach;
      D2 += ext * ext;
    }
    const int nx = c.hi[0] - c.lo[0] + 1;
    const int ny = c.hi[1] - c.lo[1] + 1;
    const int ncells = nx * ny * (c.hi[2] - c.lo[2] + 1);
    const double delta = 16. * kUnitRound * sqrt(D2);
    const float deltaf = uni_f((float)delta);
    const float xi = (float)(pi.x - ctr[0]);
    const float yi = (float)(pi.y - ctr[1]);
    const float zi = (float)(pi.z - ctr[2]);
    const float thr_i = act ? (float)((Hi + delta) * (Hi + delta)) * kThrSlack : -1.f;
    const float hxf = uni_f((float)(half[0] + delta)), hyf = uni_f((float)(half[1] + delta)),
                hzf = uni_f((float)(half[2] + delta));
    const float Hgf = uni_f((float)(Hg + delta));
    const bool wrap = c.full[0] || c.full[1] || c.full[2];
    const bool pwrap = g.periodic && (wrap || c.lo[0] < 0 || c.lo[1] < 0 || c.lo[2] < 0 ||
                                      c.hi[0] >= g.cdim[0] || c.hi[1] >= g.cdim[1] ||
                                      c.hi[2] >= g.cdim[2]);
    int nst = 0, nq = 0;
    for (int cb = 0; cb < ncells; cb += 64) {
      // batch of 64 cells, one per lane
      int cnt = 0, j0 = 0, code = 0;
      const int cl = cb + lane;
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
      for (int o = 1; o < 64; o <<= 1) {
        const int tt = __shfl_up(inc, o);
        if (lane >= o) inc += tt;
      }
      const int total = uni_i(__shfl(inc, 63));
      wave_sync();
      L.cell_j0[lane] = j0;
      L.cell_pre[lane] = inc - cnt;
      L.cell_code[lane] = (unsigned char)code;
      wave_sync();
      int k = 0;
      for (int base = 0; base < total; base += 64 * U) {
        int jj[U], sc[U];
        bool val[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int q = base + lane + 64 * u;
          val[u] = q < total;
          jj[u] = 0;
          sc[u] = 0;
          if (val[u]) {
            while (k + 1 < 64 && L.cell_pre[k + 1] <= q) k++;
            jj[u] = L.cell_j0[k] + (q - L.cell_pre[k]);
            sc[u] = L.cell_code[k];
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
          if (keep) {
            const int slot = nst + __popcll(m & ((1ull << lane) - 1ull));
            L.cand[slot] = cf;
            L.candj[slot] = jj[u];
          }
          nst += __popcll(m);
          ts.loaded += val[u] ? 1u : 0u;
          ts.staged += keep ? 1u : 0u;
        }
        if (nst > kT5Region - 64 * U) {  // region full: consume it
          wave_sync();
          if (diag != 1) {
            if (wrap)
              tile5_consume<LOOP, LPI, true, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act, nst,
                                                      L, nq, il, s, st, ts);
            else if (pwrap)
              tile5_consume<LOOP, LPI, false, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act,
                                                       nst, L, nq, il, s, st, ts);
            else
              tile5_consume<LOOP, LPI, false, false, T>(g, a, c, pi, xi, yi, zi, thr_i, act,
                                                        nst, L, nq, il, s, st, ts);
          }
          nst = 0;
          wave_sync();
        }
      }
    }
    wave_sync();
    if (diag != 1 && nst > 0) {
      if (wrap)
        tile5_consume<LOOP, LPI, true, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act, nst, L, nq,
                                                il, s, st, ts);
      else if (pwrap)
        tile5_consume<LOOP, LPI, false, true, T>(g, a, c, pi, xi, yi, zi, thr_i, act, nst, L,
                                                 nq, il, s, st, ts);
      else
        tile5_consume<LOOP, LPI, false, false, T>(g, a, c, pi, xi, yi, zi, thr_i, act, nst, L,
                                                  nq, il, s, st, ts);
    }
  }
  reduce_lanes<LPI, T>(st);
  if (act && s == 0) {
    st.store(a, i);
    if (ncount) ncount[i] = st.n;
  }
  if (counter) {
    unsigned long long v = (unsigned long long)((act && s == 0) ? st.n : 0);
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
