// swh_hydro.hip — batch hydro loops of libswifthip on a device-resident
// swh_space: one launch per loop replaces every density / gradient / force
// task of a step (src/runner_doiact_functions_hydro.h DOSELF*/DOPAIR*/DOSUB*),
// plus the ghost h-iteration (src/runner_ghost.c:1085-1596), the extra ghost
// (:992-1083) and runner_do_end_hydro_force (src/runner_others.c:618).
//
// Gather formulation: every directed pair (i <- j) is evaluated exactly once,
// by the owner of i, with the non-symmetric iact (hydro_iact.h:130,276,488),
// so the sums are deterministic and need no atomics. The loops walk the
// step's pair lists (swh_list.h); particles the lists do not cover (list
// overflow, ghost reruns whose h outgrew the list reach) take a
// wave-per-particle search of the grid cells around them.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "swh_gather.h"
#include "swh_internal.h"
#include "swh_list.h"
#include "swh_wave.h"

namespace swh {

// Sum the counter stripes (counter_stripe) into the counter slots and clear
// them: one block of kCounterStripes threads, thread t owning stripe t.
__global__ __launch_bounds__(kCounterStripes) void stripe_reduce_kernel(
    unsigned long long* __restrict__ stripes, unsigned long long* __restrict__ out) {
  const int t = threadIdx.x;
  for (int k = 0; k < 8; k++) {
    if (k == 1 || k == 2) continue;  // slots 1-2 hold other state (swh_hydro.hip counter map)
    unsigned long long v = stripes[t * 8 + k];
    stripes[t * 8 + k] = 0ull;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((t & 63) == 0 && v) atomicAdd(out + k, v);
  }
}

// ---------------------------------------------------------------------------
// The step's pair lists (swh_list.h).
// ---------------------------------------------------------------------------
// (kWalkLpi, the lanes per i of the list walks: swh_list.h)

// `run_if` (nullable): the list-build kernels of a kept-list step run only
// when the device check (list_check_kernel) found the kept lists stale, so
// the host decides nothing and never waits.
__device__ __forceinline__ bool skip_build(const unsigned int* run_if) {
  return run_if && *run_if == 0u;
}

// The periodic-wrap radius: a particle within R_max + dx of a periodic face
// may have neighbours across it (dx: the displacement bound since the
// rebuild -- particles may have drifted out of the box); rwrap_base is its
// R_max part at the list build.
__device__ __forceinline__ unsigned int rwrap_of(float base, float dx) {
  return __float_as_uint(base + dx * (1.f + 1e-4f));
}

// The list build's preparation in one pass over the i-groups (16 lanes per
// group, four groups per wave; the groups partition every particle in a
// cell): each particle's cell-local fp32 position for the staging (posf) and
// the displacement record at build time (xd0 = xdiff: a kept list measures
// drifts from here; null when nothing drifted since the re-bin, xdiff = 0), and each group's box over its active particles
// (GroupBox), reduced across the group's 16 lanes, turned into the group's
// BuildPlan (cell range, centre, rounding bound) that the build's waves read
// with scalar loads. Thread 0 resets the build's device counters.
__global__ __launch_bounds__(256) void group_prep_kernel(
    GridDev g, SoA a, const int* __restrict__ pcell, const float4* __restrict__ xdiff,
    const int2* __restrict__ groups, int ngroups, int max_active_bin, double gs1,
    float4* __restrict__ posf, float4* __restrict__ xd0, BuildPlan* __restrict__ plan,
    const unsigned int* hmax_bits, float rgs1, float dx,
    unsigned int* rwrap,
    unsigned int* rwrap_base, unsigned int* ovf_n, unsigned int* nbuilds,
    const unsigned int* run_if) {
  if (skip_build(run_if)) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const float base = __uint_as_float(*hmax_bits) * rgs1 * (1.f + 1e-4f) + 1e-30f;
    *rwrap_base = __float_as_uint(base);
    *rwrap = rwrap_of(base, dx);
    *ovf_n = 0u;
    *nbuilds += 1u;
  }
  const int gidx = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 4);
  const int r = (int)(threadIdx.x & 15);
  const int2 gr = gidx < ngroups ? groups[gidx] : make_int2(0, 0);
  GroupBox b;
  box_init(b);
  for (int k = r; k < gr.y; k += 16) {
    const int i = gr.x + k;
    const double4 p = a.pos[i];
    const int pc = pcell[i];
    posf[i] = pc >= 0 ? cell_local(g, p, pc) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (xd0) xd0[i] = xdiff[i];
    if (active_part(a, i, max_active_bin)) box_add(b, p, p.w * (double)kGamma * gs1);
  }
  for (int o = 8; o > 0; o >>= 1) {
    for (int d = 0; d < 3; d++) {
      b.lo[d] = fmin(b.lo[d], __shfl_xor(b.lo[d], o, 16));
      b.hi[d] = fmax(b.hi[d], __shfl_xor(b.hi[d], o, 16));
    }
    b.Rg = fmax(b.Rg, __shfl_xor(b.Rg, o, 16));
  }
  if (gidx < ngroups && r == 0) {
    BuildPlan p;
    build_plan(g, b, (double)__uint_as_float(*hmax_bits) * (double)kGamma * gs1, p);
    plan[gidx] = p;
  }
}

__global__ void zero_u32_kernel(unsigned int* __restrict__ p, int64_t n,
                                const unsigned int* run_if) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !skip_build(run_if)) p[i] = 0u;
}

// Kept lists after drifts (SWIFT keeps a cell's sorts until its particles
// have moved too far: dx_max_sort against space_maxreldx, space.h:66,
// runner_doiact_functions_hydro.h:1357-1400). A list holds every j with
// r_build < max(R_i, R_j), R = gamma h (1 + skin) at the build. With D the
// largest displacement since the build, r_now >= r_build - 2D, so a pair it
// lacks can enter r < max(H_i, H_j) only if some particle has H_now + 2D >
// R_build. Pass 1: D (float bits) from the displacement record.
__global__ __launch_bounds__(256) void list_disp_kernel(const float4* __restrict__ xdiff,
                                                        const float4* __restrict__ xd0,
                                                        const int8_t* __restrict__ tb, int64_t n,
                                                        unsigned int* __restrict__ disp_bits) {
  __shared__ float sm[4];
  float d = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (tb[i] == kTimeBinInhibited) continue;
    const float4 a = xdiff[i], b = xd0 ? xd0[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
    d = fmaxf(d, sqrtf(dx * dx + dy * dy + dz * dz) * (1.f + 1e-5f));
  }
  block_max_bits(disp_bits, d, sm);
}

// Pass 2: stale if an active particle is unlisted, or the H_now + 2D of ANY
// particle in a cell (active or not) exceeds its build reach. The j side of
// the list criterion used R_j of every candidate, and the drift grows h of
// inactive particles too (drift_part's h_dt term), so an inactive j whose H
// outgrew R_j - 2D would lose force pairs r < H_j (DOPAIR2's max(H_i, H_j)).
// Every candidate's build h is the w of its staging copy (posf, rewritten by
// every build): R_j,build >= fl(h) gamma (1 + skin), taken 1e-6 low for the
// float product the build rounded.
__global__ __launch_bounds__(256) void list_check_kernel(SoA a, ListDev ld, int64_t n,
                                                         int max_active_bin,
                                                         const int* __restrict__ pcell,
                                                         const unsigned int* __restrict__ disp_bits,
                                                         unsigned int* __restrict__ stale) {
  __shared__ float sm[4];
  const double D = (double)__uint_as_float(*disp_bits);
  const double gs1 = (double)kGamma * (double)ld.skin1 * (1. - 1e-6);
  float bad = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (a.tb[i] == kTimeBinInhibited || pcell[i] < 0) continue;
    const double H = a.pos[i].w * (double)kGamma;
    if (H + 2. * D > (double)ld.posf[i].w * gs1) bad = 1.f;
    if (!active_part(a, i, max_active_bin)) continue;
    if (ld.base[i] < 0 || H + 2. * D > (double)ld.reach[i]) bad = 1.f;
  }
  block_max_bits(stale, bad, sm);  // 1.0f's bits: nonzero = stale
}

// Kept lists: the wrap radius follows the displacement bound dx of the drifts.
__global__ void list_rwrap_kernel(unsigned int* rwrap, const unsigned int* rwrap_base,
                                  float dx) {
  if (threadIdx.x == 0) *rwrap = rwrap_of(__uint_as_float(*rwrap_base), dx);
}

#ifndef SWH_BUILD_WPE
#define SWH_BUILD_WPE 0
#endif
__global__ __launch_bounds__(64)
#if SWH_BUILD_WPE > 0
__attribute__((amdgpu_waves_per_eu(SWH_BUILD_WPE)))
#endif
void list_build_kernel(GridDev g, SoA a, ListDev ld,
                                                       const int2* __restrict__ groups, int g0,
                                                       int ngroups, int max_active_bin,
                                                       const unsigned int* __restrict__ hmax_bits,
                                                       unsigned long long* counter, int diag,
                                                       const unsigned int* run_if) {
  __shared__ ListLds<kListLpiBuild> lds;
  __shared__ CellTab tab;
  if (skip_build(run_if)) return;
  (void)list_build<kListLpiBuild>(g, a, ld, groups, g0 + xcd_block_id(), ngroups, max_active_bin,
                                  hmax_bits, counter, diag, lds, tab);
}

#ifndef SWH_WALK_WPE
#define SWH_WALK_WPE 0
#endif
#ifndef SWH_WALK_WPE_DENS
#define SWH_WALK_WPE_DENS 4
#endif
template <int LOOP, typename T>
__global__ __launch_bounds__(kWalkBlock)
#if SWH_WALK_WPE > 0
__attribute__((amdgpu_waves_per_eu(SWH_WALK_WPE)))
#endif
void walk_kernel(GridDev g, SoA a, ListDev ld, int i0, int n,
                                                   int max_active_bin, T a2H,
                                                   const unsigned int* __restrict__ hmax_bits,
                                                   unsigned long long* counter,
                                                   int* __restrict__ ncount) {
  list_walk<LOOP, T, kWalkLpi>(g, a, ld, i0, n, max_active_bin, a2H, hmax_bits, counter, ncount);
}

// The density walk held to 4 waves/SIMD (its four entries in flight per lane
// want 132 VGPRs, i.e. 3 waves; at <= 128 it runs 1.157 -> 1.10 ms per loop
// at 128^3; the force walk already fits 128 and does not gain).
template <typename T>
__global__ __launch_bounds__(kWalkBlock)
#if SWH_WALK_WPE_DENS > 0
__attribute__((amdgpu_waves_per_eu(SWH_WALK_WPE_DENS)))
#endif
void density_walk_kernel(GridDev g, SoA a, ListDev ld, int i0, int n, int max_active_bin, T a2H,
                         const unsigned int* __restrict__ hmax_bits, unsigned long long* counter,
                         int* __restrict__ ncount) {
  list_walk<LOOP_DENSITY, T, kWalkLpi>(g, a, ld, i0, n, max_active_bin, a2H, hmax_bits, counter,
                                       ncount);
}

// The list's overflow particles (more than K hits: a large H in a dense
// region): one wave per particle searches the cells around it, the 64 lanes
// striding over each cell's particles, cells farther than max(H_i, the
// cell's own max H) (force) or H_i (density, gradient) skipped; the lane
// partial sums are combined at the end. The count is read on the device, so
// the launch needs no host round trip.
template <int LOOP, typename T>
__global__ __launch_bounds__(256) void overflow_kernel(GridDev g, SoA a, ListDev ld,
                                                       const int* __restrict__ queue,
                                                       const unsigned int* __restrict__ qn,
                                                       int max_active_bin, T a2H,
                                                       const unsigned int* __restrict__ hmax_bits,
                                                       unsigned long long* counter,
                                                       int* __restrict__ ncount) {
  const int nov = (int)*qn;
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * (blockDim.x / 64);
  for (int w = blockIdx.x * (blockDim.x / 64) + (int)(threadIdx.x / 64); w < nov; w += nwaves) {
    const int i = queue[w];
    if (!active_part(a, i, max_active_bin)) continue;  // wave-uniform
    LoopState<LOOP, T> st;
    st.n = 0;
    st.load_i(a, i, a2H, hmax_bits);
    const double4 pi = a.pos[i];
    const double Hi = pi.w * (double)kGamma;
    CellRange c;
    cell_range(g, pi.x, pi.y, pi.z, st.reach, c);
    // The cells of the range are tested 64 at a time, one per lane (a large
    // reach spans many cells, most of them pruned), then the accepted ones
    // are walked by all lanes in the range's order (z, y, x).
    const int nx = c.hi[0] - c.lo[0] + 1, ny = c.hi[1] - c.lo[1] + 1;
    const int ncr = nx * ny * (c.hi[2] - c.lo[2] + 1);
    for (int base = 0; base < ncr; base += 64) {
      const int q = base + lane;
      bool ok = false;
      int2 r = make_int2(0, 0);
      double sx = 0., sy = 0., sz = 0.;
      if (q < ncr) {
        const int wx = wrap_cell(g, c, 0, c.lo[0] + q % nx, sx);
        const int wy = wrap_cell(g, c, 1, c.lo[1] + (q / nx) % ny, sy);
        const int wz = wrap_cell(g, c, 2, c.lo[2] + q / (nx * ny), sz);
        r = cell_range_of(g, wx, wy, wz);
        if (r.y > r.x) {
          // box gap between i and this image of the cell (its particles may
          // stand g.dx outside it after a drift)
          const double cl[3] = {g.origin[0] + wx * g.w[0] + sx, g.origin[1] + wy * g.w[1] + sy,
                                g.origin[2] + wz * g.w[2] + sz};
          const double xs[3] = {pi.x, pi.y, pi.z};
          double gap2 = 0.;
          for (int k = 0; k < 3; k++) {
            if (c.full[k]) continue;
            const double gk = fmax(fmax(cl[k] - xs[k], xs[k] - cl[k] - g.w[k]) - g.dx, 0.);
            gap2 += gk * gk;
          }
          const int lin = (wz * g.cdim[1] + wy) * g.cdim[0] + wx;
          const double Rc = LOOP != LOOP_FORCE ? Hi
                            : ld.cell_R           ? fmax(Hi, (double)ld.cell_R[lin])
                                                  : st.reach;
          ok = gap2 <= Rc * Rc * (1. + 1e-6) + 1e-300;
        }
      }
      for (unsigned long long m = __ballot(ok); m; m &= m - 1) {
        const int b = __ffsll((long long)m) - 1;
        const int j0 = __shfl(r.x, b), j1 = __shfl(r.y, b);
        const double bx = __shfl(sx, b), by = __shfl(sy, b), bz = __shfl(sz, b);
        for (int j = j0 + lane; j < j1; j += 64) {
          const double4 pj = a.pos[j];
          T dx, dy, dz;
          const T r2 = separation<T>(g, c, pi, pj, bx, by, bz, dx, dy, dz);
          if (st.accept(j, pj, r2)) st.interact(a, j, pj, dx, dy, dz, r2);
        }
      }
    }
    reduce_lanes<64, T>(st);
    if (lane == 0) {
      st.store(a, i);
      if (ncount) ncount[i] = st.n;
      if (counter) atomicAdd(counter_stripe(counter), (unsigned long long)st.n);
    }
  }
}

// The ghost's rerun lists, compacted into kSegs segments: workgroup b of a
// ghost pass appends to segment b % kSegs (capacity cap each), so the
// returning atomics of a pass spread over kSegs counters instead of all
// ~2,000 workgroups queueing on one (device-scope atomics on one address
// serialise at ~60 ns: 0.12 ms per pass over 2M particles). Entry t of the
// list is entry t - (earlier segments' counts) of its segment.
constexpr int kSegs = 8;
struct SegList {
  const int* idx;
  const unsigned int* cnt;  // kSegs counts
  int cap;
};
__device__ __forceinline__ int seg_total(const SegList& l) {
  int c = 0;
#pragma unroll
  for (int q = 0; q < kSegs; q++) c += (int)l.cnt[q];
  return c;
}
__device__ __forceinline__ int seg_at(const SegList& l, int t) {
#pragma unroll
  for (int q = 0; q < kSegs; q++) {
    const int c = (int)l.cnt[q];
    if (t < c) return l.idx[(size_t)q * l.cap + t];
    t -= c;
  }
  return -1;
}

// Density on a subset (the ghost's reruns, runner_ghost.c:1503-1546): LPI
// lanes per rerun particle walk its list while its H still fits the list
// reach; any other one (H grown past its reach, list overflow, no lists) is
// queued for the wave-per-particle search (overflow_kernel). The subset is the
// ghost's redo list, in (nearly) sorted order.
template <typename T>
__global__ __launch_bounds__(256)
#if SWH_WALK_WPE_DENS > 0
__attribute__((amdgpu_waves_per_eu(SWH_WALK_WPE_DENS)))
#endif
void walk_subset_kernel(GridDev g, SoA a, ListDev ld,
                                                          int list_ok,
                                                          SegList subset,
                                                          unsigned int* __restrict__ zero_next,
                                                          int max_active_bin,
                                                          const unsigned int* __restrict__ hmax_bits,
                                                          unsigned long long* counter,
                                                          int* __restrict__ searchq,
                                                          unsigned int* nsearch) {
  constexpr int LPI = kWalkLpi;
  // the next ghost pass's output counters (not read by this rerun or the
  // pass before it): cleared here instead of by a separate launch
  if (zero_next && blockIdx.x == 0 && threadIdx.x <= kSegs) zero_next[threadIdx.x] = 0u;
  // the grid may be an upper bound: the count is the device's
  const int nitems = seg_total(subset);
  const int t = (int)blockIdx.x * (256 / LPI) + (int)threadIdx.x / LPI;
  const int s = (int)threadIdx.x % LPI;
  const int i = t < nitems ? seg_at(subset, t) : -1;
  bool act = i >= 0 && active_part(a, i, max_active_bin);
  int nl = 0, lb = -1;
  double4 pi = make_double4(0., 0., 0., 0.);
  bool search = false;
  if (act) {
    pi = a.pos[i];
    if (list_ok) {
      nl = ld.cnt[i];
      lb = ld.base[i];
    }
    const bool listed = list_ok && lb >= 0 && nl <= ld.K &&
                        pi.w * (double)kGamma <= (double)ld.reach[i];
    if (!listed) {
      search = true;
      act = false;
    }
  }
  const bool q = search && s == 0;
  const int slot = block_append(q, nsearch);
  if (q) searchq[slot] = i;
  LoopState<LOOP_DENSITY, T> st;
  st.n = 0;
  if (act) st.load_i(a, i, (T)0, hmax_bits);
  if (!act) nl = 0;
  const double rwrap = list_ok ? (double)__uint_as_float(*ld.rwrap_bits) : 0.;
  if (__any(act && g.periodic && near_face(g, pi, rwrap)))
    walk_entries<LPI, true, T>(g, a, ld, pi, nl, lb, s, st);
  else
    walk_entries<LPI, false, T>(g, a, ld, pi, nl, lb, s, st);
  reduce_lanes<LPI, T>(st);
  if (act && s == 0) st.store(a, i);
  if (counter) {
    unsigned long long v = (unsigned long long)((act && s == 0) ? st.n : 0);
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(counter_stripe(counter), v);
  }
}

// hydro_init_part (src/hydro/SPHENIX/hydro.h:553-566) on active particles.
__global__ void init_kernel(SoA a, int64_t n, int max_active_bin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !active_part(a, i, max_active_bin)) return;
  a.th[i].y = 0.f;
  a.dens[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  a.rot[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// ---------------------------------------------------------------------------
// Ghost (runner_ghost.c:1085-1596, EXTRA_HYDRO_LOOP branch, non-cosmological
// time-steps). One thread per particle still iterating; particles whose h
// moved by more than h_tolerance are re-initialised and appended to the redo
// list (the subset reruns of runner_ghost.c:1503-1546 become one subset launch
// per iteration: list walks, or searches where h outgrew the list reach).
// ---------------------------------------------------------------------------
struct GhostParams {
  float h_max, h_min, eta_dim, eps;
  int use_mass_weighted;
  double a2_inv, H, fac_B;
};

// One particle of the ghost: redo (h updated, queued for a rerun), or
// converged (final fields written); hf_out = its h, stale = H outgrew its
// list reach.
template <typename T>
__device__ __forceinline__ void ghost_part(SoA& a, int i, bool first, float* left, float* right,
                                           const GhostParams& gp,
                                           const float* __restrict__ list_reach, bool& redo_out,
                                           float& hf_out, bool& stale) {
  double4 pos = a.pos[i];
  const T h_old = (T)(float)pos.w;
  const T h_old_dim = h_old * h_old * h_old;
  const T h_old_dim_minus_one = h_old * h_old;
  float4 th = a.th[i];
  float4 d = a.dens[i];   // rho_dh, wcount, wcount_dh, div_v
  float4 r = a.rot[i];    // rot_v, laplace_u
  const float4 vm = a.vm[i];
  T rho = th.y, rho_dh = d.x, wcount = d.y, wcount_dh = d.z, div_v = d.w;
  T rot_x = r.x, rot_y = r.y, rot_z = r.z;
  T h_new;
  bool has_no_neighbours = false;
  bool tidy = false;  // converged-by-clamp branch (runner_ghost.c:1272-1300)
  // the bisection bounds: [0, h_max] on the first pass, else the last pass's
  float lft = first ? 0.f : left[i], rgt = first ? gp.h_max : right[i];
  if (wcount < (T)(1.e-5 * kRoot)) {
    has_no_neighbours = true;
    h_new = (T)2 * h_old;
  } else {
    // hydro_end_density (hydro.h:599-630)
    const T h_inv = (T)1 / h_old;
    const T h_inv_dim = h_inv * h_inv * h_inv;
    const T h_inv_dim_plus_one = h_inv_dim * h_inv;
    const T m = vm.w;
    rho += m * (T)kRoot;
    rho_dh -= (T)kDim * m * (T)kRoot;
    wcount += (T)kRoot;
    wcount_dh -= (T)kDim * (T)kRoot;
    rho *= h_inv_dim;
    rho_dh *= h_inv_dim_plus_one;
    wcount *= h_inv_dim;
    wcount_dh *= h_inv_dim_plus_one;
    const T rho_inv = (T)1 / rho;
    const T a_inv2 = (T)gp.a2_inv;
    rot_x *= h_inv_dim_plus_one * a_inv2 * rho_inv;
    rot_y *= h_inv_dim_plus_one * a_inv2 * rho_inv;
    rot_z *= h_inv_dim_plus_one * a_inv2 * rho_inv;
    div_v *= h_inv_dim_plus_one * rho_inv * a_inv2;
    div_v += (T)gp.H * (T)kDim;
    if (gp.use_mass_weighted) {
      const T inv_mass = (T)1 / m;
      wcount = rho * inv_mass;
      wcount_dh = rho_dh * inv_mass;
    }
    const T n_sum = wcount * h_old_dim;
    const T n_target = (T)gp.eta_dim;
    const T f = n_sum - n_target;
    const T f_prime = wcount_dh * h_old_dim + (T)kDim * wcount * h_old_dim_minus_one;
    if (n_sum < n_target) lft = (float)tmax((T)lft, h_old);
    else if (n_sum > n_target) rgt = (float)tmin((T)rgt, h_old);
    if ((h_old >= (T)gp.h_max && f < (T)0) || (h_old <= (T)gp.h_min && f > (T)0)) {
      tidy = true;
      h_new = h_old;
    } else {
      h_new = h_old - f / (f_prime + (T)FLT_MIN);
      h_new = tmin(h_new, (T)2 * h_old);
      h_new = tmax(h_new, (T)0.5 * h_old);
      h_new = tmax(h_new, (T)lft);
      h_new = tmin(h_new, (T)rgt);
    }
  }
  T h_final = h_old;
  if (!tidy && fabs(h_new - h_old) > (T)gp.eps * h_old) {
    T hset;
    if ((h_new == (T)lft && h_old == (T)rgt) || (h_old == (T)lft && h_new == (T)rgt)) {
      const T l3 = (T)lft * (T)lft * (T)lft, r3 = (T)rgt * (T)rgt * (T)rgt;
      hset = cbrt((T)0.5 * (l3 + r3));
    } else {
      hset = h_new;
    }
    const float hf = (float)hset;
    if (hf < gp.h_max && hf > gp.h_min) {
      // redo: store h, re-initialise (hydro_init_part), queue for the rerun
      pos.w = (double)hf;
      a.pos[i] = pos;
      th.y = 0.f;
      a.th[i] = th;  // (a whole-record store, not a 4-byte one into it)
      a.dens[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      a.rot[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      left[i] = lft;
      right[i] = rgt;
      redo_out = true;
      hf_out = hf;
      // the rerun walks i's list only while the new H fits its reach
      stale = list_reach && (double)hf * (double)kGamma > (double)list_reach[i];
      return;
    } else if (hf <= gp.h_min) {
      h_final = (T)gp.h_min;
    } else {
      h_final = (T)gp.h_max;
      if (has_no_neighbours) {
        // hydro_part_has_no_neighbours (hydro.h:774-802)
        const T hinv = (T)1 / h_final;
        const T hid = hinv * hinv * hinv;
        rho = (T)vm.w * (T)kRoot * hid;
        wcount = (T)kRoot * hid;
        rho_dh = wcount_dh = rot_x = rot_y = rot_z = div_v = (T)0;
        r.w = 0.f;  // laplace_u
      }
    }
  }
  const float hf = (float)h_final;
  pos.w = (double)hf;
  a.pos[i] = pos;
  hf_out = hf;
  // the step's pair lists cover this particle's loops only while H <= its R
  stale = list_reach && (double)hf * (double)kGamma > (double)list_reach[i];
  // converged: hydro_prepare_gradient + hydro_reset_gradient (hydro.h:654-733)
  const T hh = (T)hf;
  const T curl_v = tsqrt(rot_x * rot_x + rot_y * rot_y + rot_z * rot_z);
  const T abs_div_v = fabs(div_v);
  const T pressure = (T)kHydroGammaMinusOne * (T)th.x * rho;
  const T soundspeed = tsqrt((T)kHydroGamma * pressure / rho);
  const T balsara =
      abs_div_v / (abs_div_v + curl_v + (T)0.0001f * soundspeed * (T)gp.fac_B / hh);
  const T common_factor = hh * (T)kDimInv / wcount;
  T grad_h_term;
  if (hh > (T)0.9999f * (T)gp.h_max) {
    grad_h_term = (T)0;
  } else {
    const T grad_W_term = common_factor * wcount_dh;
    grad_h_term = (grad_W_term < (T)-0.9999f)
                      ? (T)0
                      : common_factor * rho_dh / ((T)1 + grad_W_term);
  }
  th.y = (float)rho;
  th.z = (float)pressure;
  th.w = (float)soundspeed;
  a.th[i] = th;
  a.dens[i] = make_float4((float)rho_dh, (float)wcount, (float)wcount_dh, (float)div_v);
  r.x = (float)rot_x; r.y = (float)rot_y; r.z = (float)rot_z;
  a.rot[i] = r;
  float4 fc = a.fc[i];
  fc.x = (float)grad_h_term;
  fc.y = (float)balsara;
  a.fc[i] = fc;
  float4 g = a.grad[i];
  g.x = (float)((T)2 * soundspeed);  // v_sig
  g.y = fc.z;                        // alpha_visc_max_ngb = alpha_visc
  a.grad[i] = g;
}

// One pass of the ghost: over every active particle (the first, whose
// bisection bounds start at [0, h_max]) or the previous pass's `list`; the
// particles it queues for a rerun are appended to segmented `redo` (one
// atomic per workgroup on its segment's counter; nredo[kSegs] counts the
// reruns past their list reach).
template <typename T>
__global__ __launch_bounds__(1024) void ghost_kernel(
    SoA a, SegList list, int count, int max_active_bin, int* __restrict__ redo,
    unsigned int* __restrict__ nredo, int cap, unsigned int* __restrict__ nsearch,
    float* left, float* right, GhostParams gp, unsigned int* hmax_bits,
    const float* __restrict__ list_reach, unsigned int* ngrown, int* __restrict__ grown_q) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  // the rerun after this pass appends its searches from zero (the previous
  // rerun's search has run: same stream)
  if (t == 0) *nsearch = 0u;
  // a list pass's grid may be an upper bound: its count is the device's
  if (list.idx) count = seg_total(list);
  bool rd = false, stale = false;
  float hf = 0.f;
  int i = -1;
  bool first = false;
  if (t < count) {
    if (list.idx) {
      i = seg_at(list, t);
    } else if (active_part(a, t, max_active_bin)) {
      i = t;
      first = true;
    }
  }
  if (i >= 0) ghost_part<T>(a, i, first, left, right, gp, list_reach, rd, hf, stale);
  const int seg = (int)(blockIdx.x & (kSegs - 1));
  const int slot = block_append(rd, nredo + seg);
  if (rd) redo[(size_t)seg * cap + slot] = i;
  // reruns whose new H outgrew their list reach (they would need the
  // wave-per-particle search): one conditional atomic per wave
  const unsigned long long ms = __ballot(rd && stale);
  if ((threadIdx.x & 63) == 0 && ms) atomicAdd(nredo + kSegs, (unsigned int)__popcll(ms));
  // converged particles whose H outgrew their list reach: queued (few; one
  // atomic per wave that has any) for the gradient / force loops' searches
  stale = stale && !rd;
  const int gs = wave_append(stale, ngrown);
  if (stale) grown_q[gs] = i;
  // h max: an atomic only when it changes something (all blocks hitting one
  // address serialise at ~10 ns per atomic)
  float m = hf;
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0 && m > 0.f) atomic_max_bits_if(hmax_bits, __float_as_uint(m));
}

// The lists after a ghost that grew some converged H past its list reach R
// (grown_q): the gradient loop (r < H_i) searches those particles; the force
// loop (r < max(H_i, H_j)) also every i within H_j of a grown j, whose list may
// lack j (it holds the j with r < max(R_i, R_j) at the build). One wave per
// grown particle marks them (mark: u32 per particle, zero between loops) and
// queues each once; particles already searched as list overflow are left to
// that search.
__global__ __launch_bounds__(256) void grown_mark_kernel(GridDev g, SoA a, ListDev ld,
                                                         const int* __restrict__ grown_q,
                                                         int ngrown, int force,
                                                         const int* __restrict__ pcell,
                                                         unsigned int* __restrict__ cell_R,
                                                         unsigned int* __restrict__ mark,
                                                         int* __restrict__ q,
                                                         unsigned int* __restrict__ qn) {
  const int lane = (int)threadIdx.x & 63;
  const int w = (int)blockIdx.x * 4 + (int)threadIdx.x / 64;
  if (w >= ngrown) return;  // wave-uniform
  const int j = grown_q[w];
  auto queue = [&](int i) {
    if (ld.cnt[i] > ld.K) return;  // list overflow: searched anyway
    if (atomicExch(&mark[i], 1u) == 0u) q[atomicAdd(qn, 1u)] = i;
  };
  if (lane == 0) queue(j);
  if (!force) return;
  const double4 pj = a.pos[j];
  const double Hj = pj.w * (double)kGamma;
  // the per-cell reach the force searches prune by (adaptive grid) must
  // cover the grown H too
  if (cell_R && lane == 0 && pcell[j] >= 0)
    atomicMax(&cell_R[pcell[j]], __float_as_uint((float)Hj * 1.0000005f));
  CellRange c;
  cell_range(g, pj.x, pj.y, pj.z, Hj, c);
  for (int cz = c.lo[2]; cz <= c.hi[2]; cz++) {
    double sz;
    const int wz = wrap_cell(g, c, 2, cz, sz);
    for (int cy = c.lo[1]; cy <= c.hi[1]; cy++) {
      double sy;
      const int wy = wrap_cell(g, c, 1, cy, sy);
      for (int cx = c.lo[0]; cx <= c.hi[0]; cx++) {
        double sx;
        const int wx = wrap_cell(g, c, 0, cx, sx);
        const int2 r = cell_range_of(g, wx, wy, wz);
        for (int i = r.x + lane; i < r.y; i += 64) {
          double dx, dy, dz;
          const double r2 = separation<double>(g, c, pj, a.pos[i], sx, sy, sz, dx, dy, dz);
          if (r2 < Hj * Hj * (1. + 1e-6)) queue(i);
        }
      }
    }
  }
}

__global__ void grown_clear_kernel(const int* __restrict__ q, const unsigned int* __restrict__ qn,
                                   unsigned int* __restrict__ mark) {
  const int n = (int)*qn;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x)
    mark[q[t]] = 0u;
}

// runner_do_extra_ghost (runner_ghost.c:992-1083): hydro_end_gradient,
// hydro_prepare_force (hydro.h:823-934), timestep_limiter_prepare_force,
// hydro_reset_acceleration.
struct ForcePrepParams {
  double a, a_factor_sound_speed, a2_inv, time_base;
  float visc_alpha_max, visc_alpha_min, visc_length;
  float diff_beta, diff_alpha_max, diff_alpha_min;
  int use_bins;                     // cosmological dt_alpha per time bin (swh_hydro_params)
  double dt_bin[kNumTimeBins + 1];  // runner_ghost.c:1038-1046
};

template <typename T>
__global__ void extra_ghost_kernel(SoA a, int64_t n, int max_active_bin, ForcePrepParams fp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int tb = a.tb[i];
  if (!active_part(a, i, max_active_bin)) return;
  const T h = (T)(float)a.pos[i].w;
  const T h_inv = (T)1 / h;
  const T h_inv_dim = h_inv * h_inv * h_inv;
  const T h_inv_dim_plus_one = h_inv_dim * h_inv;
  float4 r = a.rot[i];
  const T laplace_u = (T)r.w * (T)2 * h_inv_dim_plus_one;
  r.w = (float)laplace_u;
  a.rot[i] = r;
  // get_timestep (timeline.h:91-95), or the caller's cosmological table
  const T dt_alpha = (T)(fp.use_bins ? ((tb >= 0 && tb <= kNumTimeBins) ? fp.dt_bin[tb] : 0.)
                                     : ((tb <= 0) ? 0. : (double)(1LL << (tb + 1)) * fp.time_base));
  const float4 th = a.th[i];
  float4 g = a.grad[i];     // v_sig, avmn, div_v_prev, div_v_dt
  float4 fc = a.fc[i];      // f, balsara, alpha_visc, alpha_diff
  const T div_v = (T)a.dens[i].w;
  const T kernel_support_physical = h * (T)fp.a * (T)kGamma;
  const T kernel_support_physical_inv = (T)1 / kernel_support_physical;
  const T v_sig_physical = (T)g.x * (T)fp.a_factor_sound_speed;
  const T pressure = (T)kHydroGammaMinusOne * (T)th.x * (T)th.y;
  const T soundspeed_physical =
      tsqrt((T)kHydroGamma * pressure / (T)th.y) * (T)fp.a_factor_sound_speed;
  const T sound_crossing_time_inverse = soundspeed_physical * kernel_support_physical_inv;
  const T div_v_dt = dt_alpha == (T)0 ? (T)0 : (div_v - (T)g.z) / dt_alpha;
  const T S = div_v < (T)0 ? kernel_support_physical * kernel_support_physical *
                                 tmax((T)0, (T)-1 * div_v_dt)
                           : (T)0;
  const T soundspeed_square = soundspeed_physical * soundspeed_physical;
  const T alpha_loc = (T)fp.visc_alpha_max * S / (soundspeed_square + S);
  T alpha = fc.z;
  if (alpha_loc > alpha) {
    alpha = alpha_loc;
  } else {
    const T timescale_ratio = dt_alpha * sound_crossing_time_inverse * (T)fp.visc_length;
    alpha += alpha_loc * timescale_ratio;
    alpha /= ((T)1 + timescale_ratio);
  }
  alpha = tmax(alpha, (T)fp.visc_alpha_min);
  g.z = (float)div_v;
  g.w = (float)div_v_dt;
  const T diffusion_timescale_physical_inverse = v_sig_physical * kernel_support_physical_inv;
  const T sqrt_u_inv = (T)1 / tsqrt((T)th.x);
  T alpha_diff_dt = (T)fp.diff_beta * kernel_support_physical * laplace_u *
                    (T)fp.a_factor_sound_speed * sqrt_u_inv * (T)fp.a2_inv;
  alpha_diff_dt -= ((T)fc.w - (T)fp.diff_alpha_min) * diffusion_timescale_physical_inverse;
  T new_diffusion_alpha = (T)fc.w;
  new_diffusion_alpha += alpha_diff_dt * dt_alpha;
  new_diffusion_alpha = tmax(new_diffusion_alpha, (T)fp.diff_alpha_min);
  const T viscous_diffusion_limit =
      (T)fp.diff_alpha_max * ((T)1 - (T)g.y / (T)fp.visc_alpha_max);
  new_diffusion_alpha = tmin(new_diffusion_alpha, viscous_diffusion_limit);
  fc.z = (float)alpha;
  fc.w = (float)new_diffusion_alpha;
  a.fc[i] = fc;
  a.grad[i] = g;
  a.mintb[i] = (int8_t)(kNumTimeBins + 1);
  a.acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  a.hdt[i] = 0.f;
}

// hydro_reset_acceleration (hydro.h:944-955) + timestep_limiter_prepare_force.
__global__ void reset_acc_kernel(SoA a, int64_t n, int max_active_bin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !active_part(a, i, max_active_bin)) return;
  a.acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  a.hdt[i] = 0.f;
  a.mintb[i] = (int8_t)(kNumTimeBins + 1);
}

__global__ void end_force_kernel(SoA a, int64_t n, int max_active_bin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !active_part(a, i, max_active_bin)) return;
  a.hdt[i] = a.hdt[i] * ((float)a.pos[i].w * kDimInv);  // hydro.h:1080-1084
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
static swh_status check_built(swh_space* s) {
  if (!s) return SWH_ERR_ARG;
  if (!s->built) {
    swh::set_error("swh_space_rebuild must precede the loops");
    return SWH_ERR_STATE;
  }
  return SWH_OK;
}

static unsigned long long* counter_slot(swh_space* s) {
  return s->counters.as<unsigned long long>();  // slot 0: interactions
}
static unsigned int* hmax_slot(swh_space* s) { return s->counters.as<unsigned int>() + 2; }
// The stripes the counted kernels add into (kCounterStripes x 8 u64, zero
// between counted loops: stripe_reduce_kernel clears them).
static swh_status stripes_slot(swh_space* s, unsigned long long** out) {
  if (!s->ctr_stripes.ptr) {
    const size_t b = (size_t)kCounterStripes * 8 * sizeof(unsigned long long);
    SWH_TRY(s->ctr_stripes.reserve(b));
    SWH_HIP(hipMemsetAsync(s->ctr_stripes.ptr, 0, b, s->stream));
  }
  *out = s->ctr_stripes.as<unsigned long long>();
  return SWH_OK;
}

// Counter slots (s->counters, 128 bytes): u64[0] interactions, u32[2] max h
// (float bits), u32[4..5] ghost list counts, u64[3] list entries, u64[4..7]
// loop work counters, u32[16] list overflow count, u32[17] list-stale flag,
// u32[18] list wrap radius (float bits).
static unsigned int* ovf_slot(swh_space* s) { return s->counters.as<unsigned int>() + 16; }
static unsigned int* stale_slot(swh_space* s) { return s->counters.as<unsigned int>() + 17; }
static unsigned int* rwrap_slot(swh_space* s) { return s->counters.as<unsigned int>() + 18; }
// u32[20]: the ghost reruns' search-queue length
constexpr float kGhostListSkin = 0.01f;
// u32[17]: converged particles the ghost grew past their list reach (grown_q);
// up to n / kGrownSearchMax of them are searched instead of a list rebuild
constexpr int kGrownSearchMax = 256;
// u32[28]: the grown particles' search queue (grown_mark_kernel)
static unsigned int* grown_qn_slot(swh_space* s) { return s->counters.as<unsigned int>() + 28; }
static unsigned int* search_slot(swh_space* s) { return s->counters.as<unsigned int>() + 20; }

// (u32[19]: the drift's displacement, u32[21]: max |v_full|, swh_space.hip)
// u32[24]: kept lists found stale by the device check; u32[25]: displacement
// since the list build (float bits); u32[26]: list builds run on the device;
// u32[27]: the wrap radius's R_max part
static unsigned int* keep_stale_slot(swh_space* s) { return s->counters.as<unsigned int>() + 24; }
static unsigned int* disp_slot(swh_space* s) { return s->counters.as<unsigned int>() + 25; }
static unsigned int* nbuild_slot(swh_space* s) { return s->counters.as<unsigned int>() + 26; }
static unsigned int* rwrap_base_slot(swh_space* s) { return s->counters.as<unsigned int>() + 27; }

static ListDev list_dev(swh_space* s) {
  // skin of the lists in use (the ghost may rebuild them with a wider one)
  ListDev d;
  d.nbr = s->nbr.as<int>();
  d.cnt = s->nbr_cnt.as<int>();
  d.base = s->nbr_base.as<int>();
  d.reach = s->nbr_reach.as<float>();
  d.K = s->list_K;
  d.KS = list_ks(s->list_K);
  d.skin1 = 1.f + s->list_skin_cur;
  d.rwrap_bits = rwrap_slot(s);
  d.ovf = s->nbr_ovf.as<int>();
  d.posf = s->posf.as<const float4>();
  d.diag = s->tuning.diag_mode;
  d.plan = s->gplan.as<const BuildPlan>();
  d.ovf_n = ovf_slot(s);
  // per-cell reach pruning only pays on an adaptive (clustered) grid
  d.cell_R = s->grid.adaptive ? s->cell_hreach.as<const float>() : nullptr;
  d.mark = nullptr;
  return d;
}

// Build the step's pair lists for the active particles. run_if (nullable):
// a device flag; the build kernels do nothing unless it is set (kept lists
// that the device check found stale).
static swh_status build_lists(swh_space* s, const swh_hydro_params* P, bool count,
                              float skin, const unsigned int* run_if = nullptr) {
  const int K = s->tuning.list_capacity > 0 ? s->tuning.list_capacity : 128;
  unsigned long long* stripes = nullptr;
  if (count) SWH_TRY(stripes_slot(s, &stripes));
  s->list_skin_cur = skin;
  SWH_TRY(s->nbr.reserve((size_t)std::max(1, s->ngroups) * list_ks(K) * kListSlots *
                         sizeof(int)));
  if (K % 4 != 0) {
    set_error("list_capacity must be a multiple of 4");
    return SWH_ERR_ARG;
  }
  SWH_TRY(s->nbr_cnt.reserve((size_t)s->n * sizeof(int)));
  SWH_TRY(s->nbr_base.reserve((size_t)s->n * sizeof(int)));
  SWH_TRY(s->nbr_reach.reserve((size_t)s->n * sizeof(float)));
  SWH_TRY(s->nbr_ovf.reserve((size_t)s->n * sizeof(int)));
  SWH_TRY(s->posf.reserve((size_t)s->n * sizeof(float4)));
  SWH_TRY(s->list_xd0.reserve((size_t)s->n * sizeof(float4)));
  // The displacement record: with no drift since the re-bin (xdiff = 0) the
  // build's record is zero and is not written (s->xd0_zero); before a build
  // after a drift, which the device may skip, the record is made real.
#ifndef SWH_XD0_SKIP
#define SWH_XD0_SKIP 1
#endif
  const bool no_drift = SWH_XD0_SKIP && s->grid.dx == 0.;
  if (!no_drift && s->xd0_zero) {
    SWH_HIP(hipMemsetAsync(s->list_xd0.ptr, 0, (size_t)s->n * sizeof(float4), s->stream));
    s->xd0_zero = false;
  }
  if (no_drift) s->xd0_zero = true;
  SWH_TRY(s->cell_hreach.reserve((size_t)std::max(1, s->grid.ncell) * sizeof(float)));
  s->list_K = K;
  const ListDev ld = list_dev(s);
  if (ld.cell_R) {
    hipLaunchKernelGGL(zero_u32_kernel, dim3((s->grid.ncell + 255) / 256), dim3(256), 0,
                       s->stream, s->cell_hreach.as<unsigned int>(), (int64_t)s->grid.ncell,
                       run_if);
    hipLaunchKernelGGL(cell_reach_kernel, dim3((int)((s->n + 255) / 256)), dim3(256), 0,
                       s->stream, s->pos.as<const double4>(), s->pcell.as<const int>(), s->n,
                       (float)(kGamma * ld.skin1), s->cell_hreach.as<unsigned int>(), run_if);
  }
  SWH_TRY(s->gplan.reserve((size_t)std::max(1, s->ngroups) * sizeof(BuildPlan)));
  ListDev ldb = list_dev(s);
  hipLaunchKernelGGL(group_prep_kernel, dim3(std::max(1, (s->ngroups + 15) / 16)), dim3(256), 0,
                     s->stream, grid_dev(s), soa_of(s), s->pcell.as<const int>(),
                     s->xdiff.as<const float4>(), s->groups.as<const int2>(), s->ngroups,
                     P->max_active_bin, (double)ld.skin1, s->posf.as<float4>(),
                     no_drift ? nullptr : s->list_xd0.as<float4>(), s->gplan.as<BuildPlan>(),
                     hmax_slot(s),
                     (float)(kGamma * ld.skin1), (float)s->grid.dx, rwrap_slot(s),
                     rwrap_base_slot(s), ovf_slot(s), nbuild_slot(s), run_if);
  hipLaunchKernelGGL(list_build_kernel, dim3(s->ngroups), dim3(64), 0, s->stream, grid_dev(s),
                     soa_of(s), ldb, s->groups.as<const int2>(), 0, s->ngroups,
                     P->max_active_bin, hmax_slot(s), count ? stripes : nullptr,
                     s->tuning.diag_mode, run_if);
  SWH_HIP(hipGetLastError());
  s->list_valid = true;
  s->list_check = false;
  s->list_mab = P->max_active_bin;
  s->grown_n = 0;  // the new lists cover every current H
  return SWH_OK;
}

// Kept lists after a drift: the device decides whether they still cover
// every pair (list_disp_kernel, list_check_kernel) and rebuilds them if not,
// all on the stream (no host round trip).
static swh_status check_kept_lists(swh_space* s, const swh_hydro_params* P, bool count) {
  const int nb = (int)((s->n + 255) / 256);
  SWH_HIP(hipMemsetAsync(keep_stale_slot(s), 0, 2 * sizeof(unsigned int), s->stream));
  hipLaunchKernelGGL(list_disp_kernel, dim3(std::min(nb, kReduceBlocks)), dim3(256), 0, s->stream,
                     s->xdiff.as<const float4>(),
                     s->xd0_zero ? nullptr : s->list_xd0.as<const float4>(),
                     s->tb.as<const int8_t>(), s->n, disp_slot(s));
  hipLaunchKernelGGL(list_check_kernel, dim3(std::min(nb, kReduceBlocks)), dim3(256), 0, s->stream, soa_of(s), list_dev(s),
                     s->n, P->max_active_bin, s->pcell.as<const int>(), disp_slot(s),
                     keep_stale_slot(s));
  hipLaunchKernelGGL(list_rwrap_kernel, dim3(1), dim3(64), 0, s->stream, rwrap_slot(s),
                     rwrap_base_slot(s), (float)s->grid.dx);
  SWH_HIP(hipGetLastError());
  // a device-side rebuild (stale) resets the record: xd0 = xdiff
  return build_lists(s, P, count, s->tuning.list_skin, keep_stale_slot(s));
}

template <int LOOP, typename T>
static void launch_typed(swh_space* s, const GridDev& gd, const SegList* subset, int nitems,
                         int max_active_bin, T a2H, unsigned long long* ctr, int* ncount,
                         const unsigned int* mark = nullptr) {
  const int block = 256;
  ListDev ld = list_dev(s);
  ld.mark = mark;
  constexpr int ppb = block / kWalkLpi;
  if (subset) {  // density reruns of the ghost: list walks, then the queued searches
    // (nitems: an upper bound of the device's count; the ghost pass cleared
    // the search counter)
    hipLaunchKernelGGL((walk_subset_kernel<T>), dim3((nitems + ppb - 1) / ppb), dim3(block), 0,
                       s->stream, gd, soa_of(s), ld, s->list_valid ? 1 : 0, *subset,
                       s->ghost_zero_next, max_active_bin, hmax_slot(s), ctr,
                       s->ghost_search.as<int>(), search_slot(s));
    // one wave per queued particle; the queue length is read on the device
    const int sblocks = std::max(1, std::min(2048, (nitems + 3) / 4));
    hipLaunchKernelGGL((overflow_kernel<LOOP_DENSITY, T>), dim3(sblocks), dim3(block), 0,
                       s->stream, gd, soa_of(s), ld, s->ghost_search.as<const int>(),
                       search_slot(s), max_active_bin, a2H, hmax_slot(s), ctr, ncount);
    return;
  }
  constexpr int wppb = kWalkBlock / kWalkLpi;
  if (LOOP == LOOP_DENSITY && sizeof(T) == 8)  // (the fp32 walk would spill)
    hipLaunchKernelGGL((density_walk_kernel<T>), dim3((nitems + wppb - 1) / wppb),
                       dim3(kWalkBlock), 0, s->stream, gd, soa_of(s), ld, 0, nitems,
                       max_active_bin, a2H, hmax_slot(s), ctr, ncount);
  else
    hipLaunchKernelGGL((walk_kernel<LOOP, T>), dim3((nitems + wppb - 1) / wppb),
                       dim3(kWalkBlock), 0, s->stream, gd, soa_of(s), ld, 0, nitems,
                       max_active_bin, a2H, hmax_slot(s), ctr, ncount);
  hipLaunchKernelGGL((overflow_kernel<LOOP, T>), dim3(64), dim3(block), 0, s->stream, gd,
                     soa_of(s), ld, ld.ovf, ld.ovf_n, max_active_bin, a2H, hmax_slot(s), ctr,
                     ncount);
}

template <int LOOP>
static swh_status launch_loop(swh_space* s, const swh_hydro_params* P, const SegList* subset,
                              int nitems, bool count) {
  if (nitems <= 0) return SWH_OK;
  if (!subset && s->ngroups <= 0) return SWH_OK;
  if (!subset) {
    // The density loop builds the step's lists; gradient and force reuse them
    // while no particle's H has outgrown its list reach (ghost: stale flag).
    // list_keep (or diag_mode 7): a density loop keeps lists that are still
    // valid, as SWIFT keeps its sort lists -- after a drift the device checks
    // the displacement against the lists' skin and rebuilds only if needed.
    const bool keep = (s->tuning.list_keep || s->tuning.diag_mode == 7) &&
                      s->list_mab == P->max_active_bin;
    const bool fresh = s->list_valid && s->list_mab == P->max_active_bin;
    if (keep && fresh && s->list_check) {
      SWH_TRY(check_kept_lists(s, P, count));
    } else if ((LOOP == LOOP_DENSITY && !(keep && fresh)) || !fresh) {
      SWH_TRY(build_lists(s, P, count, s->tuning.list_skin));
    } else if (s->list_check) {  // gradient / force right after a drift
      SWH_TRY(check_kept_lists(s, P, count));
    }
    if (s->tuning.diag_mode != 0 && s->tuning.diag_mode != 3 && s->tuning.diag_mode != 4 &&
        s->tuning.diag_mode != 7)
      return SWH_OK;
  }
  const GridDev gd = grid_dev(s);
  const double a2H = P->a * P->a * P->H;
  unsigned long long* ctr = nullptr;
  if (count) SWH_TRY(stripes_slot(s, &ctr));
  int* ncount = count ? s->ncount.as<int>() : nullptr;
  const bool f64 = s->ctx->precision == SWH_PRECISION_F64;
  // gradient / force after a ghost that grew a few H past the lists: those
  // particles (force: and their neighbours within H) are searched
  const bool grown = !subset && LOOP != LOOP_DENSITY && s->grown_n > 0 && s->list_valid;
  unsigned int* mark = nullptr;
  unsigned int* qn = grown_qn_slot(s);
  if (grown) {
    // the marks stay zero between uses (grown_clear_kernel); a (re)allocation
    // -- first use, or an upload that raised n since -- starts them zeroed
    const size_t mark_bytes = (size_t)s->n * sizeof(unsigned int);
    if (s->grown_mark.bytes < mark_bytes) {
      SWH_TRY(s->grown_mark.reserve(mark_bytes));
      SWH_HIP(hipMemsetAsync(s->grown_mark.ptr, 0, s->grown_mark.bytes, s->stream));
    }
    SWH_TRY(s->grown_search.reserve((size_t)s->n * sizeof(int)));
    mark = s->grown_mark.as<unsigned int>();
    SWH_HIP(hipMemsetAsync(qn, 0, sizeof(unsigned int), s->stream));
    hipLaunchKernelGGL(grown_mark_kernel, dim3((s->grown_n + 3) / 4), dim3(256), 0, s->stream,
                       gd, soa_of(s), list_dev(s), s->grown_q.as<const int>(), s->grown_n,
                       LOOP == LOOP_FORCE ? 1 : 0, s->pcell.as<const int>(),
                       s->grid.adaptive ? s->cell_hreach.as<unsigned int>() : nullptr, mark,
                       s->grown_search.as<int>(), qn);
  }
  if (f64)
    launch_typed<LOOP, double>(s, gd, subset, nitems, P->max_active_bin, a2H, ctr, ncount, mark);
  else
    launch_typed<LOOP, float>(s, gd, subset, nitems, P->max_active_bin, (float)a2H, ctr,
                              ncount, mark);
  if (grown) {
    const ListDev ld = list_dev(s);
    const int* q = s->grown_search.as<const int>();
    if (f64)
      hipLaunchKernelGGL((overflow_kernel<LOOP, double>), dim3(256), dim3(256), 0, s->stream,
                         gd, soa_of(s), ld, q, qn, P->max_active_bin, a2H, hmax_slot(s), ctr,
                         ncount);
    else
      hipLaunchKernelGGL((overflow_kernel<LOOP, float>), dim3(256), dim3(256), 0, s->stream,
                         gd, soa_of(s), ld, q, qn, P->max_active_bin, (float)a2H,
                         hmax_slot(s), ctr, ncount);
    hipLaunchKernelGGL(grown_clear_kernel, dim3(64), dim3(256), 0, s->stream, q, qn, mark);
  }
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

template <int LOOP>
static swh_status run_loop(swh_space* s, const swh_hydro_params* P, int64_t* n_out) {
  SWH_TRY(check_built(s));
  if (!P) return SWH_ERR_ARG;
  if (s->n == 0) {  // nothing to interact (the counters are not even reserved)
    if (n_out) *n_out = 0;
    return SWH_OK;
  }
  SWH_HIP(hipSetDevice(s->ctx->device));
  // counted launch: slot 0 = interactions, 3 = list entries, 4-7 = work counters
  unsigned long long* ctr = counter_slot(s);
  if (n_out) SWH_HIP(hipMemsetAsync(ctr + 3, 0, 5 * sizeof(unsigned long long), s->stream));
  if (n_out) SWH_HIP(hipMemsetAsync(ctr, 0, sizeof(unsigned long long), s->stream));
  const bool keep = (s->tuning.list_keep || s->tuning.diag_mode == 7) &&
                    s->list_mab == P->max_active_bin;
  const bool fresh = s->list_valid && s->list_mab == P->max_active_bin;
  const bool rebuilds = (LOOP == LOOP_DENSITY && !(keep && fresh)) || !fresh;
  SWH_TRY(launch_loop<LOOP>(s, P, nullptr, (int)s->n, n_out != nullptr));
  if (n_out) {
    unsigned long long* stripes = nullptr;
    SWH_TRY(stripes_slot(s, &stripes));
    hipLaunchKernelGGL(stripe_reduce_kernel, dim3(1), dim3(kCounterStripes), 0, s->stream,
                       stripes, ctr);
    SWH_HIP(hipGetLastError());
    unsigned long long h[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    SWH_HIP(hipMemcpyAsync(h, ctr, sizeof(h), hipMemcpyDeviceToHost, s->stream));
    SWH_HIP(hipStreamSynchronize(s->stream));
    *n_out = (int64_t)h[0];
    for (int k = 0; k < 4; k++) s->loop_stats[k] = (int64_t)h[4 + k];
    if (rebuilds) {
      s->list_entries = (int64_t)h[3];
      s->list_overflow = (int32_t)(h[8] & 0xffffffffull);
    }
  }
  return SWH_OK;
}

}  // namespace swh

using namespace swh;

extern "C" {

swh_status swh_space_init_parts(swh_space* s, const swh_hydro_params* P) {
  if (!s || !P) return SWH_ERR_ARG;
  if (s->n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  const int block = 256;
  hipLaunchKernelGGL(init_kernel, dim3((int)((s->n + block - 1) / block)), dim3(block), 0,
                     s->stream, soa_of(s), s->n, P->max_active_bin);
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

swh_status swh_density_loop(swh_space* s, const swh_hydro_params* P, int64_t* n) {
  return run_loop<LOOP_DENSITY>(s, P, n);
}
swh_status swh_gradient_loop(swh_space* s, const swh_hydro_params* P, int64_t* n) {
  return run_loop<LOOP_GRADIENT>(s, P, n);
}
swh_status swh_force_loop(swh_space* s, const swh_hydro_params* P, int64_t* n) {
  return run_loop<LOOP_FORCE>(s, P, n);
}

swh_status swh_ghost(swh_space* s, const swh_hydro_params* P, int32_t* iterations,
                     int64_t* n_unconverged) {
  SWH_TRY(check_built(s));
  if (!P) return SWH_ERR_ARG;
  if (iterations) *iterations = 0;
  if (n_unconverged) *n_unconverged = 0;
  const int64_t n = s->n;
  if (n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->stream;
  SWH_TRY(s->ghost_left.reserve(n * sizeof(float)));
  SWH_TRY(s->ghost_right.reserve(n * sizeof(float)));
  // segmented rerun lists: segment capacity = the workgroups a pass over n
  // particles sends to one segment, x 1024
  const int cap = (int)(((n + 1023) / 1024 + kSegs - 1) / kSegs) * 1024;
  SWH_TRY(s->ghost_list.reserve((size_t)kSegs * cap * sizeof(int)));
  SWH_TRY(s->ghost_list2.reserve((size_t)kSegs * cap * sizeof(int)));
  SWH_TRY(s->ghost_search.reserve(n * sizeof(int)));
  SWH_TRY(s->grown_q.reserve(n * sizeof(int)));
  constexpr int kCnt = kSegs + 1;  // a pass's segment counts + its reruns past reach
  SWH_TRY(s->ghost_seg.reserve(2 * kCnt * sizeof(unsigned int)));
  SWH_TRY(s->ghost_host.reserve(64 * kCnt * sizeof(unsigned int)));
  const int block = 1024;
  GhostParams gp;
  gp.h_max = P->h_max;
  gp.h_min = P->h_min;
  gp.eta_dim = P->eta_neighbours * P->eta_neighbours * P->eta_neighbours;
  gp.eps = P->h_tolerance;
  gp.use_mass_weighted = P->use_mass_weighted_num_ngb;
  gp.a2_inv = P->a2_inv;
  gp.H = P->H;
  gp.fac_B = P->a_factor_Balsara_eps;
  // Pass k writes rerun list L[k % 2] with counts C[k % 2]; its rerun walks
  // them and clears C[(k + 1) % 2] for pass k + 1. The first pass is
  // synchronous (its count of reruns past their list reach decides a list
  // rebuild); later passes are pipelined: pass k, the copy of its counts,
  // and its rerun (grid sized by pass k - 1's count, the device reading the
  // real one) are queued before the host waits for pass k's count, so the
  // GPU runs the rerun while the host reads -- a pass with no reruns costs
  // an empty rerun launch, not a host round trip per pass.
  int* L[2] = {s->ghost_list.as<int>(), s->ghost_list2.as<int>()};
  unsigned int* Cn[2] = {s->ghost_seg.as<unsigned int>(), s->ghost_seg.as<unsigned int>() + kCnt};
  unsigned int* hc = static_cast<unsigned int*>(s->ghost_host.ptr);
  const bool lists = true;
  SWH_HIP(hipMemsetAsync(stale_slot(s), 0, sizeof(unsigned int), st));
  SWH_HIP(hipMemsetAsync(Cn[0], 0, 2 * kCnt * sizeof(unsigned int), st));
  // profiling only (SWH_GHOST_DEBUG): per pass the rerun count, the reruns
  // past their list reach, and the ghost / host + rebuild / rerun times (the
  // passes then run synchronously)
  static const bool dbg = std::getenv("SWH_GHOST_DEBUG") != nullptr;
  hipEvent_t dev[4] = {nullptr, nullptr, nullptr, nullptr};
  if (dbg)
    for (auto& e : dev) SWH_HIP(hipEventCreate(&e));
  // the copies of the passes' counts (the host waits on these, not the stream)
  struct CountEvents {
    hipEvent_t e[2] = {nullptr, nullptr};
    ~CountEvents() {
      for (auto& x : e)
        if (x) (void)hipEventDestroy(x);
    }
    hipEvent_t& operator[](int k) { return e[k]; }
  } ev_cnt;
  for (int k = 0; k < 2; k++) SWH_HIP(hipEventCreateWithFlags(&ev_cnt.e[k], hipEventDisableTiming));
  auto launch_pass = [&](int k, const SegList& in, int grid_items) -> swh_status {
    const float* lreach = (lists && s->list_valid) ? s->nbr_reach.as<const float>() : nullptr;
    const int g = (grid_items + block - 1) / block;
    if (s->ctx->precision == SWH_PRECISION_F64)
      hipLaunchKernelGGL(ghost_kernel<double>, dim3(g), dim3(block), 0, st, soa_of(s), in,
                         grid_items, P->max_active_bin, L[k & 1], Cn[k & 1], cap,
                         search_slot(s), s->ghost_left.as<float>(), s->ghost_right.as<float>(),
                         gp, hmax_slot(s), lreach, stale_slot(s), s->grown_q.as<int>());
    else
      hipLaunchKernelGGL(ghost_kernel<float>, dim3(g), dim3(block), 0, st, soa_of(s), in,
                         grid_items, P->max_active_bin, L[k & 1], Cn[k & 1], cap,
                         search_slot(s), s->ghost_left.as<float>(), s->ghost_right.as<float>(),
                         gp, hmax_slot(s), lreach, stale_slot(s), s->grown_q.as<int>());
    SWH_HIP(hipGetLastError());
    SWH_HIP(hipMemcpyAsync(hc + (k % 64) * kCnt, Cn[k & 1], kCnt * sizeof(unsigned int),
                           hipMemcpyDeviceToHost, st));
    SWH_HIP(hipEventRecord(ev_cnt[k & 1], st));
    return SWH_OK;
  };
  auto rerun = [&](int k, int grid_items) -> swh_status {
    const SegList list{L[k & 1], Cn[k & 1], cap};
    s->ghost_zero_next = Cn[(k + 1) & 1];
    const swh_status r = launch_loop<LOOP_DENSITY>(s, P, &list, grid_items, false);
    s->ghost_zero_next = nullptr;
    return r;
  };
  auto total = [&](int k) {
    int c = 0;
    for (int q = 0; q < kSegs; q++) c += (int)hc[(k % 64) * kCnt + q];
    return c;
  };
  auto debug_line = [&](int k, int in, int out, bool rebuilt) {
    if (!dbg) return;
    (void)hipEventSynchronize(dev[3]);
    float ms[3] = {0.f, 0.f, 0.f};
    for (int q = 0; q < 3; q++) (void)hipEventElapsedTime(&ms[q], dev[q], dev[q + 1]);
    std::fprintf(stderr,
                 "[swh ghost] it %d: in %d, rerun %d, past reach %u, rebuilt %d | ghost %.3f "
                 "ms, host + rebuild %.3f ms, rerun %.3f ms\n",
                 k, in, out, hc[(k % 64) * kCnt + kSegs], (int)rebuilt, ms[0], ms[1], ms[2]);
  };
  // pass 0 (synchronous)
  int it = 0, count = 0;
  if (P->max_smoothing_iterations > 0) {
    if (dbg) SWH_HIP(hipEventRecord(dev[0], st));
    SWH_TRY(launch_pass(0, SegList{nullptr, Cn[1], cap}, (int)n));
    if (dbg) SWH_HIP(hipEventRecord(dev[1], st));
    SWH_HIP(hipStreamSynchronize(st));
    count = total(0);
    const unsigned int nstale = hc[kSegs];
    it = 1;
    const bool many = s->list_valid ? (int64_t)nstale * 8 >= n : (int64_t)count * 8 >= n;
    if (count > 0 && lists && many) {
      // Many reruns whose new H outgrew their list reach (the first pass after
      // a drift with exact lists: every growing h): rebuild the lists for the
      // new h, with a 1% skin so the few later passes' changes stay within
      // reach and the gradient / force loops keep them, then walk. Lists built
      // with a skin (swh_tuning.list_skin, 2% by default) cover the reruns:
      // they walk the lists, the few outgrown ones are searched.
      SWH_TRY(build_lists(s, P, false, std::max(s->tuning.list_skin, kGhostListSkin)));
      SWH_HIP(hipMemsetAsync(stale_slot(s), 0, sizeof(unsigned int), st));
    }
    if (dbg) SWH_HIP(hipEventRecord(dev[2], st));
    if (count > 0) SWH_TRY(rerun(0, count));
    if (dbg) SWH_HIP(hipEventRecord(dev[3], st));
    debug_line(0, (int)n, count, count > 0 && lists && many);
  }
  // passes 1, 2, ... (pipelined)
  while (count > 0 && it < P->max_smoothing_iterations) {
    const int k = it;
    const SegList in{L[(k - 1) & 1], Cn[(k - 1) & 1], cap};
    if (dbg) SWH_HIP(hipEventRecord(dev[0], st));
    SWH_TRY(launch_pass(k, in, count));
    if (dbg) {
      SWH_HIP(hipEventRecord(dev[1], st));
      SWH_HIP(hipEventRecord(dev[2], st));
    }
    SWH_TRY(rerun(k, count));  // (pass k's reruns are at most its input)
    if (dbg) SWH_HIP(hipEventRecord(dev[3], st));
    // the counts of pass k: their copy follows pass k on the stream, ahead
    // of the rerun just queued, which the GPU runs meanwhile
    SWH_HIP(hipEventSynchronize(ev_cnt[k & 1]));
    const int in_count = count;
    count = total(k);
    it = k + 1;
    debug_line(k, in_count, count, false);
  }
  if (dbg)
    for (auto& e : dev) (void)hipEventDestroy(e);
  {
    // slots 2 (max h) .. 17 (list-stale flag) in one read
    unsigned int c[18];
    SWH_HIP(hipMemcpyAsync(c, s->counters.ptr, sizeof(c), hipMemcpyDeviceToHost, st));
    SWH_HIP(hipStreamSynchronize(st));
    // converged particles grown past their list reach: a few are searched by
    // the gradient / force loops (grown_mark_kernel); many -> those loops
    // rebuild the lists
    s->grown_n = 0;
    if (lists && s->list_valid && c[17]) {
      if ((int64_t)c[17] * kGrownSearchMax > n) s->list_valid = false;
      else s->grown_n = (int32_t)c[17];
    }
    if (dbg)
      std::fprintf(stderr, "[swh ghost] converged past their list reach: %u (%s)\n", c[17],
                   !c[17] ? "-" : s->grown_n ? "searched" : "lists rebuilt");
    float hmax;
    std::memcpy(&hmax, &c[2], sizeof(hmax));
    // a kernel reach of half the periodic box or more would need more than
    // the nearest image (runner_doiact_functions_hydro.h:2283, "Cell smaller
    // than smoothing length")
    if (s->grid.periodic &&
        (double)hmax * kGamma >= 0.5 * std::min(s->grid.dim[0], std::min(s->grid.dim[1],
                                                                         s->grid.dim[2]))) {
      swh::set_error("Cell smaller than smoothing length: gamma*h_max=%g, box %g", hmax * kGamma,
                     std::min(s->grid.dim[0], std::min(s->grid.dim[1], s->grid.dim[2])));
      return SWH_ERR_CELL_SMALL;
    }
  }
  if (iterations) *iterations = it;
  if (n_unconverged) *n_unconverged = count;
  if (count > 0) {
    swh::set_error("Smoothing length failed to converge on %d particles.", count);
    return SWH_ERR_NOT_CONVERGED;
  }
  return SWH_OK;
}

swh_status swh_extra_ghost(swh_space* s, const swh_hydro_params* P) {
  SWH_TRY(check_built(s));
  if (!P) return SWH_ERR_ARG;
  if (s->n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  ForcePrepParams fp;
  fp.a = P->a;
  fp.a_factor_sound_speed = P->a_factor_sound_speed;
  fp.a2_inv = P->a2_inv;
  fp.time_base = P->time_base;
  fp.visc_alpha_max = P->visc_alpha_max;
  fp.visc_alpha_min = P->visc_alpha_min;
  fp.visc_length = P->visc_length;
  fp.diff_beta = P->diff_beta;
  fp.diff_alpha_max = P->diff_alpha_max;
  fp.diff_alpha_min = P->diff_alpha_min;
  fp.use_bins = P->dt_alpha_bins != nullptr;
  for (int b = 0; b <= kNumTimeBins; b++) fp.dt_bin[b] = fp.use_bins ? P->dt_alpha_bins[b] : 0.;
  const int block = 256;
  const int g = (int)((s->n + block - 1) / block);
  if (s->ctx->precision == SWH_PRECISION_F64)
    hipLaunchKernelGGL(extra_ghost_kernel<double>, dim3(g), dim3(block), 0, s->stream,
                       soa_of(s), s->n, P->max_active_bin, fp);
  else
    hipLaunchKernelGGL(extra_ghost_kernel<float>, dim3(g), dim3(block), 0, s->stream,
                       soa_of(s), s->n, P->max_active_bin, fp);
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

swh_status swh_space_reset_acceleration(swh_space* s, const swh_hydro_params* P) {
  if (!s || !P) return SWH_ERR_ARG;
  if (s->n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  const int block = 256;
  hipLaunchKernelGGL(reset_acc_kernel, dim3((int)((s->n + block - 1) / block)), dim3(block),
                     0, s->stream, soa_of(s), s->n, P->max_active_bin);
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

swh_status swh_end_force(swh_space* s, const swh_hydro_params* P) {
  SWH_TRY(check_built(s));
  if (!P) return SWH_ERR_ARG;
  if (s->n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  const int block = 256;
  hipLaunchKernelGGL(end_force_kernel, dim3((int)((s->n + block - 1) / block)), dim3(block),
                     0, s->stream, soa_of(s), s->n, P->max_active_bin);
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

}  // extern "C"
