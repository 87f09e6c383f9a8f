// swh_list.h — the step's pair lists (loop variant 7, the default).
//
// SWIFT builds its neighbour structure once (runner_do_hydro_sort,
// src/runner_sort.c:201-431) and every loop of the step walks it: density,
// the ghost's subset reruns, gradient and force (runner_doiact_functions_
// hydro.h DOPAIR1/DOPAIR2 walk the same sort lists). The batch path does the
// same with explicit pair lists:
//
//   list build (list_build): one wave per i-group (an octree leaf of <= 16
//     particles, swh_space.hip group_kernel), four lanes per i. The wave
//     stages the candidates of the cells around its group (four cells per
//     pass, 16 lanes per cell; fp32 coordinates relative to the group centre
//     from the cell-local fp32 copy of the positions, pruned by the exact box
//     distance), tests every (i, candidate) in fp32 against
//       r < max(R_i, R_j),  R = gamma h (1 + skin)
//     with the threshold inflated by the worst-case rounding bound, and
//     appends the hits to i's list. The list is a superset of every pair
//     the three loops accept (density/gradient: r < H_i, DOPAIR1/DOSELF1;
//     force: r < max(H_i, H_j), DOPAIR2/DOSELF2), and stays one while no
//     particle's H grows past its R (the ghost checks that: skin = SWIFT's
//     space_maxreldx-style slack for h changes between loops).
//   list walk (list_walk): LPI lanes per active i over consecutive sorted
//     particles (every lane of the wave busy), each lane walking every
//     LPI-th entry of i's list: fp64 separation (nearest periodic image),
//     the loop's exact fp64 criterion and the fp64 non-symmetric iact
//     (hydro_iact.h:130, 276, 488), index loads two entries ahead and
//     particle loads one entry ahead. The LPI partial sums are combined at
//     the end. The accepted pair set is exactly the f64 oracle's.
//
// Layout: the lists of one i-group (16 slots) form a block of 16 K entries;
// entry k of slot sl sits at row k/4, column 4 sl + k%4 of the block's
// 64-entry rows. The four lanes of an i read one 16-byte segment per row and
// a wave reads whole 256-byte rows. Particles with more than K hits
// (cnt > K) are walked by the wave-per-particle search (overflow_kernel).
#pragma once

#include "swh_wave.h"

namespace swh {

constexpr int kListSlots = 16;   // list columns per i-group (max group size)
constexpr int kListLpiBuild = 4;  // lanes per i in the list build
#ifndef SWH_LIST_REGION
#define SWH_LIST_REGION 192
#endif
#ifndef SWH_LIST_ICAP
#define SWH_LIST_ICAP 64
#endif
constexpr int kListRegion = SWH_LIST_REGION;  // staged candidates per region of the build
constexpr int kListBlk = 8;  // candidates per lane per test block of the build

// Lanes per i of the list walks (WL); the list layout follows it.
#ifndef SWH_WALK_LPI
#define SWH_WALK_LPI 4
#endif
constexpr int kWalkLpi = SWH_WALK_LPI;
static_assert(kWalkLpi == 2 || kWalkLpi == 4 || kWalkLpi == 8, "walk lanes per i: 2, 4 or 8");
constexpr int kWinInts = kListSlots * kWalkLpi * 4;  // one window row of a group's lists

// Layout of a group's lists: 16 slots x KS entries (KS = K rounded up to
// 4 WL). Entry k of slot sl is the m-th entry (m = k / WL) of walk lane
// s = k % WL of that slot; the lane keeps its entries 4w .. 4w + 3 in one
// 16-byte word of window w (a row of 16 slots x WL words), so a walk lane
// reads four indices with one load, and at each step the WL lanes of an i
// take WL consecutive entries.
__host__ __device__ constexpr int list_ks(int K) {
  return (K + 4 * kWalkLpi - 1) & ~(4 * kWalkLpi - 1);
}
__device__ __forceinline__ size_t list_lane(int base, int KS) {  // base = group * 16 + slot
  return (size_t)(base >> 4) * (size_t)(kListSlots * KS) + (size_t)((base & 15) * kWalkLpi * 4);
}
__device__ __forceinline__ size_t list_off4(int s, int m) {
  return (size_t)((m >> 2) * kWinInts + s * 4 + (m & 3));
}
__device__ __forceinline__ size_t list_at(int base, int KS, int k) {
  return list_lane(base, KS) + list_off4(k % kWalkLpi, k / kWalkLpi);
}

// Per i-group box of the list build (group_prep_kernel): the active
// particles' bounding box and the largest R = gamma h (1 + skin); Rg = 0: no
// active particle. The group's 16 lanes reduce it once, so the build's waves
// read it with scalar loads instead of reducing across lanes.
struct GroupBox {
  double lo[3], hi[3], Rg, pad;
};

// The wave-uniform part of a group's list build, computed once per group by
// group_prep_kernel from its box (so the build wave starts from scalar loads
// instead of ~170 VALU instructions of fp64 setup): the cell range around the
// box out to reach = max(R_group, R_max) + dx, the box centre and half
// extent, and the rounding bound delta of the fp32 relative coordinates.
struct BuildPlan {
  double ctr[3], half[3];
  double Rg, Rmax, delta;
  int lo[3], hi[3];
  int full;  // bit k: the range spans the periodic box along k
  int nx, nxy, ncells;
  float hf[3], Rgf, deltaf, inv_nx, inv_nxy;
  int pad[1];
};
static_assert(sizeof(BuildPlan) % 16 == 0, "plans are read as 16-byte words");

struct ListDev {
  int* nbr;      // entries: sorted j indices
  int* cnt;      // per particle: entries found (> K: overflow, searched instead)
  int* base;     // per particle: group * kListSlots + slot (-1: not listed)
  float* reach;  // per particle: R = gamma h (1 + skin) at build (0: not listed)
  const float4* posf;  // per particle: x, y, z relative to its grid cell's corner, h
  int K;
  int KS;        // entries per slot in memory (list_ks(K))
  float skin1;   // 1 + skin
  const unsigned int* rwrap_bits;  // max R at build (float bits): particles farther than
                                   // this from every face need no periodic wrap
  int* ovf;      // overflow particles, count in *ovf_n
  unsigned int* ovf_n;
  const float* cell_R;  // per linear grid cell: max R of its particles (cell_reach_kernel);
                        // null on a uniform grid (no per-cell pruning)
  int diag;      // profiling only: 2 = the build writes no entries
  const unsigned int* mark;  // nullable: particles the walks leave to a search (ghost-grown H)
  const BuildPlan* plan;  // per group (group_prep_kernel), read by the build
};

__device__ __forceinline__ void box_init(GroupBox& b) {
  b.lo[0] = b.lo[1] = b.lo[2] = 1e300;
  b.hi[0] = b.hi[1] = b.hi[2] = -1e300;
  b.Rg = 0.;
  b.pad = 0.;
}
__device__ __forceinline__ void box_add(GroupBox& b, const double4& p, double R) {
  b.lo[0] = p.x < b.lo[0] ? p.x : b.lo[0];
  b.lo[1] = p.y < b.lo[1] ? p.y : b.lo[1];
  b.lo[2] = p.z < b.lo[2] ? p.z : b.lo[2];
  b.hi[0] = p.x > b.hi[0] ? p.x : b.hi[0];
  b.hi[1] = p.y > b.hi[1] ? p.y : b.hi[1];
  b.hi[2] = p.z > b.hi[2] ? p.z : b.hi[2];
  b.Rg = R > b.Rg ? R : b.Rg;
}


__device__ __forceinline__ void build_plan(const GridDev& g, const GroupBox& b, double Rmax,
                                           BuildPlan& p) {
  p.Rg = b.Rg;
  p.Rmax = Rmax;
  // r < max(R_i, R_j); cells are enumerated out to reach + dx (drift)
  const double reach = fmax(b.Rg, Rmax) + g.dx;
  double D2 = 0.;
  p.full = 0;
  for (int k = 0; k < 3; k++) {
    int lo = (int)floor((b.lo[k] - g.origin[k] - reach) * g.inv_w[k]);
    int hi = (int)floor((b.hi[k] - g.origin[k] + reach) * g.inv_w[k]);
    bool full = false;
    if (g.periodic) {
      full = (hi - lo + 1 >= g.cdim[k]);
      if (full) {
        lo = 0;
        hi = g.cdim[k] - 1;
      }
    } else {
      lo = max(lo, 0);
      hi = min(hi, g.cdim[k] - 1);
    }
    p.lo[k] = lo;
    p.hi[k] = hi;
    p.full |= full ? 1 << k : 0;
    p.ctr[k] = 0.5 * (b.lo[k] + b.hi[k]);
    p.half[k] = 0.5 * (b.hi[k] - b.lo[k]);
    const double ext = full ? g.dim[k] : p.half[k] + reach;
    D2 += ext * ext;
  }
  p.nx = p.hi[0] - p.lo[0] + 1;
  p.nxy = p.nx * (p.hi[1] - p.lo[1] + 1);
  p.ncells = p.nxy * (p.hi[2] - p.lo[2] + 1);
  // Rounding bound of the fp32 relative coordinates: a candidate is staged
  // as fl(local) + fl(cell offset) with |local| <= w, |offset| <= D + w and
  // |sum| <= D (kThrSlack's argument, swh_wave.h, with 2(D + w) in place of D).
  const double wmax = fmax(g.w[0], fmax(g.w[1], g.w[2]));
  p.delta = 16. * kUnitRound * (sqrt(D2) + wmax);
  p.deltaf = (float)p.delta;
  for (int k = 0; k < 3; k++) p.hf[k] = (float)(p.half[k] + p.delta);
  p.Rgf = (float)(b.Rg + p.delta);
  p.inv_nx = 1.f / (float)p.nx;
  p.inv_nxy = 1.f / (float)p.nxy;
}

// Per-cell maximum R = gamma h (1 + skin): the list build skips a cell whose
// box lies farther than max(R_group, R_cell) from the group box (SWIFT's
// per-cell h_max pruning of DOPAIR2, runner_doiact_functions_hydro.h:1424-1530).
// A particle counts for the cell whose sorted range holds it (pcell, from the
// rebuild): after a drift it may stand outside that cell's box, and the build
// stages it from there (the box gaps allow for g.dx); inhibited particles
// (pcell < 0) are in no cell.
__global__ void cell_reach_kernel(const double4* __restrict__ pos, const int* __restrict__ pcell,
                                  int64_t n, float gs1, unsigned int* __restrict__ cell_R,
                                  const unsigned int* run_if) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || (run_if && *run_if == 0u)) return;
  const int lin = pcell[j];
  if (lin < 0) return;
  // positive floats order as their bit patterns
  atomicMax(&cell_R[lin], __float_as_uint((float)(pos[j].w * (double)gs1) * 1.0000005f));
}

// Candidates per lane per staging pass. Two: a 256-slot region then takes
// two passes before its consume (four filled it in one pass, so every pass
// consumed a part-full region); EAGLE's density loop 1.65 -> 1.60 ms, Sedov
// unchanged (profiles/r05y_stage_units_ab.txt).
#ifndef SWH_STAGE_U
#define SWH_STAGE_U 2
#endif

// A build wave's LDS: its staged candidate region and its i's pending hits.
// REGION: staged candidates per region; ICAP: LDS hits per i before a flush.
template <int LPI, int REGION, int ICAP, typename HitT_ = unsigned short>
struct ListLdsT {
  using HitT = HitT_;  // a hit: its slot in the region
  static_assert(REGION <= 256 || sizeof(HitT_) >= 2, "8-bit hits address 256 slots");
  static constexpr int GS = 64 / LPI;
  static constexpr int kRegion = REGION;
  static constexpr int kICap = ICAP;
  static_assert(kICap >= kListBlk * LPI, "one consume block must fit i's LDS hits");
  static constexpr int kStride = kICap + 2;  // odd dword stride: lists start on different banks
  // candidates per lane per staging pass (a pass must fit the region)
  static constexpr int kStageU = SWH_STAGE_U * 64 <= REGION ? SWH_STAGE_U : REGION / 64;
  static_assert(kStageU >= 1 && REGION >= 64 * kStageU, "a staging pass must fit the region");
  // staged candidates (SoA, so a lane's run of candidates reads as float4s and
  // pairs of them feed the packed fp32 tests): x, y, z relative to the box
  // centre, w = inflated R_j^2
  alignas(16) float cx[REGION];
  alignas(16) float cy[REGION];
  alignas(16) float cz[REGION];
  alignas(16) float cw[REGION];
  int candj[REGION];
  HitT hits[GS * kStride + 64];  // [i slot][entry] region slots; + per-lane dummies
};
template <int LPI>
using ListLds = ListLdsT<LPI, kListRegion, SWH_LIST_ICAP>;

// The per-group staging's cell table (one batch of up to 64 cells).
struct CellTab {
  int mark[64];    // staging pass: 4 x int8 per lane -- the cell whose range starts at
                   // each of the pass's 256 candidate positions, -1 elsewhere
  int j0[64];      // first sorted index of the cell minus its prefix
  float4 off[64];  // cell corner relative to the group centre (fp32)
};

// Inclusive max-scan over the 64 lanes by DPP (as wave_incl_scan; -1 is the
// identity: every value scanned is >= -1).
__device__ __forceinline__ int wave_incl_max(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}

// Positions relative to the lower corner of each particle's grid cell, in
// fp32, with h: the list build's staging loads 16 B per candidate and turns
// it into group-relative coordinates with three fp32 adds.
// The cell is the particle's sorted cell (pcell, from the rebuild), not the
// one its current position falls in: after a drift the offset may leave
// [0, w) by up to g.dx, and staging adds the sorted cell's corner back.
__device__ __forceinline__ float4 cell_local(const GridDev& g, const double4& p, int lin) {
  const double xs[3] = {p.x, p.y, p.z};
  const int ck[3] = {lin % g.cdim[0], (lin / g.cdim[0]) % g.cdim[1],
                     lin / (g.cdim[0] * g.cdim[1])};
  float l[3];
  for (int k = 0; k < 3; k++) l[k] = (float)(xs[k] - (g.origin[k] + ck[k] * g.w[k]));
  return make_float4(l[0], l[1], l[2], (float)p.w);
}

// Copy i's pending LDS hits to its global list (the LPI lanes of i split them).
template <int LPI, class LDS>
__device__ __forceinline__ void list_flush(const ListDev& ld, LDS& L, int& nq, int& wr, int il,
                                           int s, int gbase, TileStats& ts) {
  wave_sync();  // list entries were written by the other lanes of i
#ifndef SWH_DIAG_CELLS
  ts.bsteps += (unsigned int)(nq > s ? (nq - s + LPI - 1) / LPI : 0);  // this lane's entries
#endif
  const typename LDS::HitT* list = &L.hits[il * LDS::kStride];

  if (ld.diag != 2) {
    // four entries per lane per step: their slot and index reads are
    // independent, so a step costs two LDS round trips, not eight
    const int nk = min(nq, ld.K - wr);  // entries past K are not stored
    for (int t = s; t < nk; t += 4 * LPI) {
      int sl[4], jv[4];
#pragma unroll
      for (int q = 0; q < 4; q++) sl[q] = t + q * LPI < nk ? list[t + q * LPI] : 0;
#pragma unroll
      for (int q = 0; q < 4; q++) jv[q] = L.candj[sl[q]];
      if (LPI == 4 && kWalkLpi == 4 && (wr & 15) == 0 && t + 3 * LPI < nk) {
        // an i's first flush (wr = 0, the usual case) puts a lane's four
        // entries wr + t + 4q in one 16-byte word of the walk layout
        // (list_off4: entry k -> column k % 4, row k / 4, rows 4w..4w+3 of
        // window w together): one store
        *reinterpret_cast<int4*>(&ld.nbr[list_at(gbase + il, ld.KS, wr + t)]) =
            make_int4(jv[0], jv[1], jv[2], jv[3]);
      } else if (LPI == 4 && kWalkLpi == 8 && (wr & 31) == 0 && t + 3 * LPI < nk) {
        // eight walk lanes: entries wr + t + {0, 8} are rows m, m + 1 of walk
        // lane t % 8 (m even), wr + t + {4, 12} those of lane t % 8 + 4
        *reinterpret_cast<int2*>(&ld.nbr[list_at(gbase + il, ld.KS, wr + t)]) =
            make_int2(jv[0], jv[2]);
        *reinterpret_cast<int2*>(&ld.nbr[list_at(gbase + il, ld.KS, wr + t + 4)]) =
            make_int2(jv[1], jv[3]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (t + q * LPI < nk) ld.nbr[list_at(gbase + il, ld.KS, wr + t + q * LPI)] = jv[q];
      }
    }
  }
  wr += nq;
  nq = 0;
  wave_sync();
}

// Pad the staged region [nst, next multiple of kListBlk * LPI) with
// candidates that never hit (the consume blocks then need no bound check).
template <int LPI = 4, class LDS>
__device__ __forceinline__ void list_pad(LDS& L, int nst) {
  const int lane = threadIdx.x & 63;
  constexpr int B = kListBlk * LPI;
  const int end = min((nst + B - 1) / B * B, LDS::kRegion);
  for (int k = nst + lane; k < end; k += 64) {
    L.cx[k] = 3e30f;
    L.cy[k] = 3e30f;
    L.cz[k] = 3e30f;
    L.cw[k] = -1.f;
  }
}

// Phase A over the staged region [0, nst) for the list criterion, then flush.
template <int LPI, bool WRAP, class LDS>
__device__ __forceinline__ void list_consume(const GridDev& g, const ListDev& ld,
                                             const CellRange& c, float xi, float yi, float zi,
                                             float thr_i, bool act, int nst, LDS& L, int& nq,
                                             int& wr, int il, int s, int gbase, TileStats& ts) {
  constexpr int GS = 64 / LPI;
  const int dummy = GS * LDS::kStride + il * LPI + s;
  const int nblk = (nst + kListBlk * LPI - 1) / (kListBlk * LPI);
#ifndef SWH_DIAG_CELLS
  ts.asteps += (unsigned int)(nblk * kListBlk);
#endif
  const float bx = (float)g.dim[0], by = (float)g.dim[1], bz = (float)g.dim[2];
  for (int b = 0; b < nblk; b++) {
    if (__any(nq > LDS::kICap - kListBlk * LPI)) list_flush<LPI>(ld, L, nq, wr, il, s, gbase, ts);
    // lane s of i tests the contiguous run c0 .. c0 + kListBlk - 1 (its hits
    // come out in candidate order), two candidates per packed fp32 op
    const int c0 = (b * LPI + s) * kListBlk;
    static_assert(kListBlk == 8, "two float4 reads per coordinate");
    float4 qx[2], qy[2], qz[2], qw[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      qx[h] = *reinterpret_cast<const float4*>(&L.cx[c0 + 4 * h]);
      qy[h] = *reinterpret_cast<const float4*>(&L.cy[c0 + 4 * h]);
      qz[h] = *reinterpret_cast<const float4*>(&L.cz[c0 + 4 * h]);
      qw[h] = *reinterpret_cast<const float4*>(&L.cw[c0 + 4 * h]);
    }
    bool hit[kListBlk];
    int cnt = 0;
    const f32x2 xi2 = {xi, xi}, yi2 = {yi, yi}, zi2 = {zi, zi};
#pragma unroll
    for (int p = 0; p < kListBlk / 2; p++) {
      const float4& X = qx[p >> 1];
      const float4& Y = qy[p >> 1];
      const float4& Z = qz[p >> 1];
      const float4& W = qw[p >> 1];
      const bool hi2 = p & 1;
      f32x2 dx = xi2 - (hi2 ? f32x2{X.z, X.w} : f32x2{X.x, X.y});
      f32x2 dy = yi2 - (hi2 ? f32x2{Y.z, Y.w} : f32x2{Y.x, Y.y});
      f32x2 dz = zi2 - (hi2 ? f32x2{Z.z, Z.w} : f32x2{Z.x, Z.y});
      const f32x2 w2 = hi2 ? f32x2{W.z, W.w} : f32x2{W.x, W.y};
      if (WRAP) {
        if (c.full[0]) dx = f32x2{wrap_nearest_sel(dx.x, bx), wrap_nearest_sel(dx.y, bx)};
        if (c.full[1]) dy = f32x2{wrap_nearest_sel(dy.x, by), wrap_nearest_sel(dy.y, by)};
        if (c.full[2]) dz = f32x2{wrap_nearest_sel(dz.x, bz), wrap_nearest_sel(dz.y, bz)};
      }
      f32x2 r2 = dx * dx;
      r2 = __builtin_elementwise_fma(dy, dy, r2);
      r2 = __builtin_elementwise_fma(dz, dz, r2);
      // slots past nst hold far-away padding (list_pad), which never hits.
      // r2 < max(thr_i, w_j) on the bit patterns: r2 and the staged w_j are
      // >= 0 (w = -1 of the padding, or thr_i = -1 of an inactive i, orders
      // below every r2), so signed-integer order is float order and the max
      // needs no canonicalisation (fmaxf costs three instructions here)
      const int ti = __float_as_int(thr_i);
      hit[2 * p] = act & (__float_as_int(r2.x) < max(ti, __float_as_int(w2.x)));
      hit[2 * p + 1] = act & (__float_as_int(r2.y) < max(ti, __float_as_int(w2.y)));
      cnt += (hit[2 * p] ? 1 : 0) + (hit[2 * p + 1] ? 1 : 0);
    }
    // this lane's first position in i's list: i's count + earlier sub-lanes' hits
    int inc, tot;
    if constexpr (LPI == 4) {  // quad scan by DPP quad permutes (no LDS round trip)
      inc = cnt;
      int tt = __builtin_amdgcn_mov_dpp(inc, 0x90, 0xF, 0xF, false);  // quad_perm [0,0,1,2]
      inc += s >= 1 ? tt : 0;
      tt = __builtin_amdgcn_mov_dpp(inc, 0x40, 0xF, 0xF, false);  // quad_perm [0,0,0,1]
      inc += s >= 2 ? tt : 0;
      tot = __builtin_amdgcn_mov_dpp(inc, 0xFF, 0xF, 0xF, false);  // quad_perm [3,3,3,3]
    } else if constexpr (LPI == 8) {  // 8-lane segments: DPP row shifts, masked by s
      inc = cnt;
      int tt = __builtin_amdgcn_mov_dpp(inc, 0x111, 0xF, 0xF, false);  // row_shr:1
      inc += s >= 1 ? tt : 0;
      tt = __builtin_amdgcn_mov_dpp(inc, 0x112, 0xF, 0xF, false);  // row_shr:2
      inc += s >= 2 ? tt : 0;
      tt = __builtin_amdgcn_mov_dpp(inc, 0x114, 0xF, 0xF, false);  // row_shr:4
      inc += s >= 4 ? tt : 0;
      // the segment's last lane to all 8: each quad's last, then lanes 0-3
      // take lane 7's through the half-row mirror
      const int qb = __builtin_amdgcn_mov_dpp(inc, 0xFF, 0xF, 0xF, false);  // quad_perm [3,3,3,3]
      const int mb = __builtin_amdgcn_mov_dpp(qb, 0x141, 0xF, 0xF, false);  // row_half_mirror
      tot = s < 4 ? mb : qb;
    } else {
      inc = cnt;
      for (int o = 1; o < LPI; o <<= 1) {
        const int tt = __shfl_up(inc, o, LPI);
        if (s >= o) inc += tt;
      }
      tot = __shfl(inc, LPI - 1, LPI);
    }
    // (byte offsets: no scaling per candidate)
    using HitT = typename LDS::HitT;
    char* hb = reinterpret_cast<char*>(L.hits);
    int pos = (il * LDS::kStride + nq + inc - cnt) * (int)sizeof(HitT);
    const int dpos = dummy * (int)sizeof(HitT);
#pragma unroll
    for (int kk = 0; kk < kListBlk; kk++) {
      *reinterpret_cast<HitT*>(hb + (hit[kk] ? pos : dpos)) = (HitT)(c0 + kk);
      pos += hit[kk] ? (int)sizeof(HitT) : 0;
    }
    nq += tot;
  }
  list_flush<LPI>(ld, L, nq, wr, il, s, gbase, ts);
}

// A build wave's epilogue for its i-slot: list length, base and reach of i
// (an overflowing list queues i for the wave search), the launch's counters.
__device__ __forceinline__ void list_finish(const ListDev& ld, int i, bool act, double Ri, int wr,
                                            int lb, int s, unsigned long long* counter,
                                            const TileStats& ts) {
  if (i >= 0 && s == 0) {
    ld.cnt[i] = act ? wr : 0;
    ld.base[i] = act ? lb : -1;
    ld.reach[i] = act ? (float)Ri : 0.f;
    if (act && wr > ld.K) ld.ovf[atomicAdd(ld.ovf_n, 1u)] = i;
  }
  if (counter) {
    unsigned long long v = (unsigned long long)((act && s == 0) ? wr : 0);
    unsigned long long ld_ = ts.loaded, sg = ts.staged, fl = ts.bsteps;
    for (int o = 32; o > 0; o >>= 1) {
      v += __shfl_xor(v, o);
      ld_ += __shfl_xor(ld_, o);
      sg += __shfl_xor(sg, o);
      fl += __shfl_xor(fl, o);
    }
    if ((threadIdx.x & 63) == 0) {
      unsigned long long* cs = counter_stripe(counter);
      atomicAdd(cs + 3, v);  // list entries
      atomicAdd(cs + 4, ld_);
      atomicAdd(cs + 5, sg);
      atomicAdd(cs + 6, (unsigned long long)ts.asteps);
      atomicAdd(cs + 7, fl);  // lane flush steps
    }
  }
}

// What a build wave knows about its i-slot when the group's lists are done
// (the fused density walk continues from it).
struct BuildSlot {
  int i;        // sorted index (-1: empty slot)
  bool act;     // active i with a list
  int nl;       // its entries (> K: overflow)
  int lb;       // its list base (group * kListSlots + slot)
  double4 pi;   // position, h
};

// Build the pair lists of one i-group (one wave).
template <int LPI, class LDS>
__device__ __forceinline__ BuildSlot list_build(const GridDev& g, const SoA& a, const ListDev ld,
                                           const int2* __restrict__ groups, int gid, int ngroups,
                                           int max_active_bin,
                                           const unsigned int* __restrict__ hmax_bits,
                                           unsigned long long* counter, int diag, LDS& L,
                                           CellTab& T) {
  constexpr int kStageU = LDS::kStageU;
  // one int8 start mark per candidate of a staging pass
  static_assert(64 * kStageU <= (int)sizeof(CellTab::mark), "a pass's marks must fit CellTab::mark");
  const int lane = threadIdx.x & 63;
  const int il = lane / LPI, s = lane % LPI;
  const int2 gr = gid < ngroups ? groups[gid] : make_int2(0, 0);
  const int i = il < gr.y ? gr.x + il : -1;
  const bool act = i >= 0 && active_part(a, i, max_active_bin);
  const double skin1 = (double)ld.skin1;
  double4 pi = make_double4(0., 0., 0., 0.);
  if (act) pi = a.pos[i];
  const double Ri = act ? pi.w * (double)kGamma * skin1 : 0.;
  // the group's build plan (wave-uniform: scalar loads)
  const BuildPlan& P = ld.plan[gid < ngroups ? gid : 0];
  const double Rg = gid < ngroups ? P.Rg : 0.;
  TileStats ts;
  const int gbase = gid * kListSlots;
  int nq = 0, wr = 0;
  if (Rg > 0.) {
    const double Rmax = P.Rmax;
    CellRange c;
    double ctr[3], half[3];
    for (int k = 0; k < 3; k++) {
      c.lo[k] = P.lo[k];
      c.hi[k] = P.hi[k];
      c.full[k] = (P.full >> k) & 1;
      ctr[k] = P.ctr[k];
      half[k] = P.half[k];
    }
    const int nx = P.nx;
    const int nxy = P.nxy;
#ifdef SWH_DIAG_NOENUM  // profiling only (diag 1): no cell enumerated
    const int ncells = diag == 1 ? 0 : P.ncells;
#else
    const int ncells = P.ncells;
#endif
    const double delta = P.delta;
    const float deltaf = P.deltaf;
    const float xi = (float)(pi.x - ctr[0]);
    const float yi = (float)(pi.y - ctr[1]);
    const float zi = (float)(pi.z - ctr[2]);
    const float thr_i = act ? (float)((Ri + delta) * (Ri + delta)) * kThrSlack : -1.f;
    const float hxf = P.hf[0], hyf = P.hf[1], hzf = P.hf[2];
    const float Rgf = P.Rgf;
    const float gs1 = (float)((double)kGamma * skin1);
    const bool wrap = P.full != 0;
    const float bx = (float)g.dim[0], by = (float)g.dim[1], bz = (float)g.dim[2];
    const float inv_nx = P.inv_nx, inv_nxy = P.inv_nxy;
    // Staging, in batches of up to 64 cells (one lane per cell: its sorted
    // range and the offset of its lower corner from the group centre go to
    // LDS with a prefix sum of the counts). Candidates are then streamed
    // kStageU per lane per pass: each lane finds the cell of its candidate by
    // a binary search over the prefix sums and issues its 16-byte cell-local
    // position load; the kStageU searches and loads are independent, so a
    // lane keeps kStageU loads in flight.
    int nst = 0;
    for (int cb = 0; cb < ncells; cb += 64) {
      int cnt = 0, j0 = 0;
      float ox = 0.f, oy = 0.f, oz = 0.f;
      const int cl = cb + lane;
      if (cl < ncells) {
        const int iz = (int)(((float)cl + 0.5f) * inv_nxy);
        const int rxy = cl - iz * nxy;
        const int iy = (int)(((float)rxy + 0.5f) * inv_nx);
        const int ix = rxy - iy * nx;
        double sx, sy, sz;
        const int wx = wrap_cell(g, c, 0, c.lo[0] + ix, sx);
        const int wy = wrap_cell(g, c, 1, c.lo[1] + iy, sy);
        const int wz = wrap_cell(g, c, 2, c.lo[2] + iz, sz);
        const int2 sp = cell_range_of(g, wx, wy, wz);
        j0 = sp.x;
        cnt = sp.y - sp.x;
        // lower corner of this image of the cell, relative to the group centre
        const double dox = g.origin[0] + wx * g.w[0] + sx - ctr[0];
        const double doy = g.origin[1] + wy * g.w[1] + sy - ctr[1];
        const double doz = g.origin[2] + wz * g.w[2] + sz - ctr[2];
        ox = (float)dox;
        oy = (float)doy;
        oz = (float)doz;
        if (cnt > 0 && ld.cell_R && Rmax > Rg) {
          // prune by the cell's own reach: box gap group <-> cell (an axis
          // spanning the whole periodic box has no gap)
          // (the cell's particles may stand g.dx outside its box after a drift)
          const double gx = c.full[0] ? 0. : fmax(fmax(dox - half[0], -half[0] - dox - g.w[0]) - g.dx, 0.);
          const double gy = c.full[1] ? 0. : fmax(fmax(doy - half[1], -half[1] - doy - g.w[1]) - g.dx, 0.);
          const double gz = c.full[2] ? 0. : fmax(fmax(doz - half[2], -half[2] - doz - g.w[2]) - g.dx, 0.);
          const double Rc = fmax(Rg, (double)ld.cell_R[(wz * g.cdim[1] + wy) * g.cdim[0] + wx]) +
                            delta;
          if (gx * gx + gy * gy + gz * gz > Rc * Rc * (1. + 1e-6)) cnt = 0;
        }
      }
#ifdef SWH_DIAG_ENUM  // profiling only (diag 1): enumerate and prune the cells, stage nothing
      if (diag == 1) cnt = 0;
#endif
#ifdef SWH_DIAG_CELLS  // profiling only: asteps / bsteps count cells enumerated / staged from
      if (lane == 0) ts.asteps += (unsigned int)min(64, ncells - cb);
      ts.bsteps += cnt > 0 ? 1u : 0u;
#endif
      const int inc = wave_incl_scan(cnt);
      const int total = __builtin_amdgcn_readlane(inc, 63);
      const int cpre = inc - cnt;  // this lane's cell: first position in the batch
      wave_sync();
      T.j0[lane] = j0 - cpre;
      T.off[lane] = make_float4(ox, oy, oz, 0.f);
      int cur = -1;  // the cell of the last candidate of the previous pass
      for (int base = 0; base < total; base += 64 * kStageU) {
        if (nst > LDS::kRegion - 64 * kStageU) {  // no room for this pass: consume the region
          list_pad<LPI>(L, nst);
          wave_sync();
          if (diag != 1) {
            if (wrap)
              list_consume<LPI, true>(g, ld, c, xi, yi, zi, thr_i, act, nst, L, nq, wr, il, s,
                                      gbase, ts);
            else
              list_consume<LPI, false>(g, ld, c, xi, yi, zi, thr_i, act, nst, L, nq, wr, il, s,
                                       gbase, ts);
          }
          nst = 0;
          wave_sync();
        }
        int jj[kStageU];
        float4 q[kStageU];
        float4 off[kStageU];
        bool val[kStageU];
        // the cell of candidate qq: the last cell starting at or before qq.
        // Each non-empty cell marks its first position within the pass; a
        // max-scan over the lanes carries the marks forward (no per-candidate
        // search over the prefix sums)
        int kc[kStageU];
        wave_sync();  // the previous pass's marks are read
        T.mark[lane] = -1;  // (four int8 marks per lane)
        wave_sync();
        {
          const int rel = cpre - base;
          if (cnt > 0 && rel >= 0 && rel < 64 * kStageU)
            reinterpret_cast<signed char*>(T.mark)[rel] = (signed char)lane;
        }
        wave_sync();
#pragma unroll
        for (int u = 0; u < kStageU; u++)
          kc[u] = reinterpret_cast<const signed char*>(T.mark)[64 * u + lane];
#pragma unroll
        for (int u = 0; u < kStageU; u++) {
          kc[u] = max(wave_incl_max(kc[u]), cur);
          cur = __builtin_amdgcn_readlane(kc[u], 63);
        }
#pragma unroll
        for (int u = 0; u < kStageU; u++) kc[u] = max(kc[u], 0);  // (lanes past total)
#pragma unroll
        for (int u = 0; u < kStageU; u++) {
          const int qq = base + 64 * u + lane;
          val[u] = qq < total;
          jj[u] = val[u] ? T.j0[kc[u]] + qq : 0;
          off[u] = T.off[kc[u]];
        }
#pragma unroll
        for (int u = 0; u < kStageU; u++)
          q[u] = val[u] ? ld.posf[jj[u]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < kStageU; u++) {
          bool keep = false;
          float4 cf = make_float4(0.f, 0.f, 0.f, 0.f);
          if (val[u]) {
            cf.x = q[u].x + off[u].x;  // x, y, z relative to its cell's corner; h
            cf.y = q[u].y + off[u].y;
            cf.z = q[u].z + off[u].z;
            if (c.full[0]) cf.x = wrap_nearest_f(cf.x, bx);
            if (c.full[1]) cf.y = wrap_nearest_f(cf.y, by);
            if (c.full[2]) cf.z = wrap_nearest_f(cf.z, bz);
            const float ex = c.full[0] ? 0.f : fmaxf(fabsf(cf.x) - hxf, 0.f);
            const float ey = c.full[1] ? 0.f : fmaxf(fabsf(cf.y) - hyf, 0.f);
            const float ez = c.full[2] ? 0.f : fmaxf(fabsf(cf.z) - hzf, 0.f);
            const float Rj = q[u].w * gs1 + deltaf;
            cf.w = Rj * Rj * kThrSlack;
            const float rj = fmaxf(Rgf, Rj);
            keep = ex * ex + ey * ey + ez * ez <= rj * rj * kThrSlack;
          }
          const unsigned long long m = __ballot(keep);
          if (keep) {
            const int slot = nst + __popcll(m & ((1ull << lane) - 1ull));
            L.cx[slot] = cf.x;
            L.cy[slot] = cf.y;
            L.cz[slot] = cf.z;
            L.cw[slot] = cf.w;
            L.candj[slot] = jj[u];
          }
          nst += __popcll(m);
          ts.loaded += val[u] ? 1u : 0u;
          ts.staged += keep ? 1u : 0u;
        }
      }
      wave_sync();  // the next batch rewrites the cell table
    }
    list_pad<LPI>(L, nst);
    wave_sync();
    if (diag != 1 && nst > 0) {
      if (wrap)
        list_consume<LPI, true>(g, ld, c, xi, yi, zi, thr_i, act, nst, L, nq, wr, il, s, gbase,
                                ts);
      else
        list_consume<LPI, false>(g, ld, c, xi, yi, zi, thr_i, act, nst, L, nq, wr, il, s, gbase,
                                 ts);
    }
  }
  list_finish(ld, i, act, Ri, wr, gbase + il, s, counter, ts);
  BuildSlot b;
  b.i = i;
  b.act = act;
  b.nl = act ? wr : 0;
  b.lb = gbase + il;
  b.pi = pi;
  return b;
}

// Does particle x need the nearest-image wrap (within R of a periodic face)?
__device__ __forceinline__ bool near_face(const GridDev& g, const double4& p, double R) {
  return (p.x < R) | (p.x > g.dim[0] - R) | (p.y < R) | (p.y > g.dim[1] - R) | (p.z < R) |
         (p.z > g.dim[2] - R);
}

// Walk entries s, s+LPI, ... of i's list (nl entries from list base lb),
// four at a time: one 16-byte load gives a window's four indices (the next
// window's is loaded ahead), then the four entries' particle data are loaded
// together (only lanes that have them issue loads) and evaluated.
template <int LPI, bool WRAP, typename T, class S>
__device__ __forceinline__ void walk_entries(const GridDev& g, const SoA& a, const ListDev& ld,
                                             const double4& pi, int nl, int lb, int s, S& st) {
  static_assert(LPI == kWalkLpi, "the list layout gives each walk lane of an i its own windows");
  const int nme = nl > s ? (nl - s + LPI - 1) / LPI : 0;  // this lane's entries
  const int nw = (nme + 3) >> 2;
  if (nw == 0) return;
  const int* __restrict__ lanep = ld.nbr + list_lane(lb, ld.KS) + s * 4;
  auto step = [&](int j, const double4& pj, const JRec<S::kPay>& rj) {
    double dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
    if (WRAP) {
      dx = wrap_nearest(dx, g.dim[0]);
      dy = wrap_nearest(dy, g.dim[1]);
      dz = wrap_nearest(dz, g.dim[2]);
    }
    const T tdx = (T)dx, tdy = (T)dy, tdz = (T)dz;
    const T r2 = tdx * tdx + tdy * tdy + tdz * tdz;
    if (st.accept(j, pj, r2)) st.interact_staged(rj.p, rj.meta, pj, tdx, tdy, tdz, r2);
  };
  int4 wv = *reinterpret_cast<const int4*>(lanep);
  if constexpr (S::kPay > 1) {
    // heavy records (gradient, force): one entry at a time, its record loaded
    // at its entry (one record live: 4 waves/SIMD)
    int4 cur = wv;
#pragma unroll 1
    for (int m = 0; m < nme; m++) {
      const int q = m & 3;
      if (q == 0) {
        cur = wv;
        if (m + 4 < nme) wv = *reinterpret_cast<const int4*>(lanep + ((m >> 2) + 1) * kWinInts);
      }
      const int j = q == 0 ? cur.x : q == 1 ? cur.y : q == 2 ? cur.z : cur.w;
      const double4 pj = a.pos[j];
      const JRec<S::kPay> rj = S::load_j(a, j);
      step(j, pj, rj);
    }
    return;
  }
  for (int w = 0; w < nw; w++) {
    const int jv[4] = {wv.x, wv.y, wv.z, wv.w};
    if (w + 1 < nw) wv = *reinterpret_cast<const int4*>(lanep + (w + 1) * kWinInts);
    const int mrem = nme - 4 * w;  // entries of this window (>= 1)
    {
      double4 pj[4];
      JRec<S::kPay> rj[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (q < mrem) {
          pj[q] = a.pos[jv[q]];
          rj[q] = S::load_j(a, jv[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; q++)
        if (q < mrem) step(jv[q], pj[q], rj[q]);
    }
  }
}

// One loop over every active, listed particle: LPI lanes per i, 256/LPI
// consecutive sorted particles per workgroup.
// Threads per block of the list walks: the waves of one block share a CU's
// L1, so a larger block walks a contiguous run of sorted i's whose
// neighbours overlap.
#ifndef SWH_WALK_BLOCK
#define SWH_WALK_BLOCK 256
#endif
constexpr int kWalkBlock = SWH_WALK_BLOCK;

template <int LOOP, typename T, int LPI>
__device__ __forceinline__ void list_walk(const GridDev& g, SoA& a, const ListDev ld, int i0, int n,
                                          int max_active_bin, T a2H,
                                          const unsigned int* __restrict__ hmax_bits,
                                          unsigned long long* counter, int* __restrict__ ncount) {
  using S = LoopState<LOOP, T>;
  constexpr int PPB = kWalkBlock / LPI;
  const int i = i0 + xcd_block_id() * PPB + (int)threadIdx.x / LPI;
  const int s = (int)threadIdx.x % LPI;
  bool act = i < n && active_part(a, i, max_active_bin);
  int nl = 0, lb = 0;
  if (act) {
    nl = ld.cnt[i];
    lb = ld.base[i];
    if (nl > ld.K || lb < 0) act = false;  // overflow: the search walks it
    if (ld.mark && ld.mark[i]) act = false;  // grown past the lists: searched
  }
  S st;
  st.n = 0;
  double4 pi = make_double4(0., 0., 0., 0.);
  if (act) {
    st.load_i(a, i, a2H, hmax_bits);
    pi = a.pos[i];
  }
  if (!act) nl = 0;
  const double rwrap = (double)__uint_as_float(*ld.rwrap_bits);
  if (__any(act && g.periodic && near_face(g, pi, rwrap)))
    walk_entries<LPI, true, T>(g, a, ld, pi, nl, lb, s, st);
  else
    walk_entries<LPI, false, T>(g, a, ld, pi, nl, lb, s, st);
  reduce_lanes<LPI, T>(st);
  if (act && s == 0) {
    st.store(a, i);
    if (ncount) ncount[i] = st.n;
  }
  if (counter) {
    unsigned long long v = (unsigned long long)((act && s == 0) ? st.n : 0);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(counter_stripe(counter), v);
  }
}

}  // namespace swh
