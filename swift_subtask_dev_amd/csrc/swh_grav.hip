// swh_grav.hip — batch leaf-leaf P2P gravity (runner_doself_grav_pp /
// runner_dopair_grav_pp, src/runner_doiact_grav.c:1500-1871 and 584-760) on a
// device-resident gpart set.
//
// One 256-thread workgroup per i-leaf (leaves in XCD-contiguous order, so the
// leaves one XCD works on are neighbours and share its L2); each thread keeps
// up to kIPer i-particle accumulators in registers (fp64). Source leaves of
// the i-leaf's CSR list are streamed through LDS in 256-particle tiles
// (x, y, z, softening and its reciprocal in fp64, mass); every lane reads
// the same tile entry (LDS broadcast), so the inner loop is pure fp64 FMA
// work: the compute-bound P2P roofline (fp64 vector, no MFMA: a gather/FMA
// path, not a dense contraction). Per pair: 1/sqrt(r^2) by the hardware
// reciprocal square root refined by Newton steps, 1/max(eps_i, eps_j) as
// min(1/eps_i, 1/eps_j) from per-particle reciprocals (no division), and the
// i == j term of a self tile removed by a zero mass instead of a branch.
//
// Pairs flagged allow_mpole (runner_dopair_grav_pp's allow_mpole, the
// recursive pair task's M2P branch, runner_doiact_grav.c:1273-1400): an
// i-particle that passes gravity_M2P_accept against the source leaf's
// multipole (float test, swh_mpole.h) skips that leaf's P2P tiles (zero mass)
// and takes M2P instead, in m2p_kernel; leaf multipoles come from p2m_kernel.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "swh_internal.h"
#include "swh_mpole.h"
#include "swh_physics.h"
#include "swh_wave.h"

namespace swh {

constexpr int kGravBlock = 256;
#ifndef SWH_GRAV_IPER
#define SWH_GRAV_IPER 2
#endif
constexpr int kIPer = SWH_GRAV_IPER;  // i-particles per thread per pass

struct GSoA {
  double4* pos;  // x, y, z, epsilon
  double* hinv;  // 1 / epsilon
  float* mass;   // 0 for inhibited
  int8_t* active;
  double4* acc;  // a_x, a_y, a_z, potential
  float* oagn;   // old_a_grav_norm (adaptive MAC)
  const swh_multipole* mp;  // per leaf (p2m_kernel)
};

__global__ void gunpack_kernel(GLayout L, const char* __restrict__ aos, int64_t n, GSoA g,
                               int max_active_bin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const char* r = aos + i * L.stride;
  const double* x = reinterpret_cast<const double*>(r + L.x);
  const float eps = *reinterpret_cast<const float*>(r + L.epsilon);
  g.pos[i] = make_double4(x[0], x[1], x[2], (double)eps);
  g.hinv[i] = 1.0 / (double)eps;
  const int tb = *reinterpret_cast<const int8_t*>(r + L.time_bin);
  const bool inhibited = tb == kTimeBinInhibited;
  g.mass[i] = inhibited ? 0.f : *reinterpret_cast<const float*>(r + L.mass);
  g.active[i] = (!inhibited && tb <= max_active_bin) ? 1 : 0;
  g.acc[i] = make_double4(0., 0., 0., 0.);
  g.oagn[i] = L.old_a_grav_norm >= 0 ? *reinterpret_cast<const float*>(r + L.old_a_grav_norm)
                                     : 0.f;
}

// gravity_P2M + gravity_multipole_compute_power (multipole.h:878-1266), one
// wave per cell (ids[w], or cell w). Leaves hold ~10-400 gparts, so the wave
// splits over the moments, not the gparts: lane (h, tt) takes term 4 + tt and
// the gparts of parity h, in order; the halves combine with one shuffle.
// Mass, CoM, r_max, the largest softening and the smallest old |a| are
// summed the same way (every lane of a half holds the same partials). Terms
// are stored as the reference stores them (float); the power of the float
// terms follows in lane 0.
constexpr int kP2MWaves = 4;
// (a, b, c) of term t packed as a | b << 4 | c << 8, for lane-indexed lookups
__constant__ unsigned short kMpABC[SWH_MPOLE_TERMS] = {
#define SWH_ABC(t) (unsigned short)(kMpA[t] | kMpB[t] << 4 | kMpC[t] << 8)
    SWH_ABC(0),  SWH_ABC(1),  SWH_ABC(2),  SWH_ABC(3),  SWH_ABC(4),  SWH_ABC(5),  SWH_ABC(6),
    SWH_ABC(7),  SWH_ABC(8),  SWH_ABC(9),  SWH_ABC(10), SWH_ABC(11), SWH_ABC(12), SWH_ABC(13),
    SWH_ABC(14), SWH_ABC(15), SWH_ABC(16), SWH_ABC(17), SWH_ABC(18), SWH_ABC(19), SWH_ABC(20),
    SWH_ABC(21), SWH_ABC(22), SWH_ABC(23), SWH_ABC(24), SWH_ABC(25), SWH_ABC(26), SWH_ABC(27),
    SWH_ABC(28), SWH_ABC(29), SWH_ABC(30), SWH_ABC(31), SWH_ABC(32), SWH_ABC(33), SWH_ABC(34)};
#undef SWH_ABC
__device__ __forceinline__ double fact4(int n) {  // n! for a run-time n <= 4
  return n <= 1 ? 1. : n == 2 ? 2. : n == 3 ? 6. : 24.;
}
__device__ __forceinline__ double ipow4(double x, int n) {
  const double x2 = x * x;
  return n == 0 ? 1. : n == 1 ? x : n == 2 ? x2 : n == 3 ? x2 * x : x2 * x2;
}
__global__ __launch_bounds__(64 * kP2MWaves) void p2m_kernel(GLayout L, const char* __restrict__ aos,
                                                             const swh_leaf* __restrict__ leaves,
                                                             const int* __restrict__ ids, int nids,
                                                             swh_multipole* __restrict__ out) {
  __shared__ double sP[kP2MWaves][SWH_MPOLE_TERMS - 4];
  const int wv = (int)threadIdx.x / 64;
  const int w = (int)blockIdx.x * kP2MWaves + wv;
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5, tt = lane & 31;
  const bool live = w < nids;  // wave-uniform; no early exit before the barrier
  int c = 0;
  swh_leaf lf{0, 0};
  if (live) {
    c = ids ? ids[w] : w;
    lf = leaves[c];
  }
  auto rec = [&](int k) { return aos + (size_t)(lf.start + k) * L.stride; };
  // pass 1: mass and mass-weighted position
  double m0 = 0., mx = 0., my = 0., mz = 0.;
  float eps_max = 0.f, oag_min = FLT_MAX;
  for (int k = h; k < lf.count; k += 2) {
    const char* r = rec(k);
    const double* x = reinterpret_cast<const double*>(r + L.x);
    const double m = *reinterpret_cast<const float*>(r + L.mass);
    m0 += m;
    mx += x[0] * m;
    my += x[1] * m;
    mz += x[2] * m;
    eps_max = fmaxf(eps_max, *reinterpret_cast<const float*>(r + L.epsilon));
    if (L.old_a_grav_norm >= 0)
      oag_min = fminf(oag_min, *reinterpret_cast<const float*>(r + L.old_a_grav_norm));
  }
  m0 += __shfl_xor(m0, 32);
  mx += __shfl_xor(mx, 32);
  my += __shfl_xor(my, 32);
  mz += __shfl_xor(mz, 32);
  eps_max = fmaxf(eps_max, __shfl_xor(eps_max, 32));
  oag_min = fminf(oag_min, __shfl_xor(oag_min, 32));
  const double imass = 1.0 / m0;
  const double com[3] = {mx * imass, my * imass, mz * imass};
  // pass 2: this lane's moment about the CoM, and r_max^2
  const int t = 4 + tt;
  const bool term = tt < SWH_MPOLE_TERMS - 4;
  const int abc = term ? (int)kMpABC[t] : 0;
  const int ta = abc & 15, tb = (abc >> 4) & 15, tc = abc >> 8;
  double v = 0., rmax2 = 0.;
  for (int k = h; k < lf.count; k += 2) {
    const char* r = rec(k);
    const double* x = reinterpret_cast<const double*>(r + L.x);
    const double m = *reinterpret_cast<const float*>(r + L.mass);
    const double d0 = x[0] - com[0], d1 = x[1] - com[1], d2 = x[2] - com[2];
    rmax2 = fmax(rmax2, d0 * d0 + d1 * d1 + d2 * d2);
    v += m * (ipow4(d0, ta) * ipow4(d1, tb) * ipow4(d2, tc));
  }
  v += __shfl_xor(v, 32);
  rmax2 = fmax(rmax2, __shfl_xor(rmax2, 32));
  // M_n = (-1)^|n| sum m d^n / n!, stored by its lane; the power terms
  // (mpole_power's weights and float/double mix) summed in term order by lane 0
  const int ord = ta + tb + tc;
  const double coef = ((ord & 1) ? -1. : 1.) / (fact4(ta) * fact4(tb) * fact4(tc));
  const float Mf = (float)(v * coef);
  const double wgt = fact4(ta) * fact4(tb) * fact4(tc) / fact4(ord);
  if (live && h == 0 && term) {
    sP[wv][tt] = wgt == 1. ? (double)(Mf * Mf) : wgt * (double)Mf * (double)Mf;
    out[c].M[t] = Mf;
  }
  __syncthreads();
  if (live && lane == 0) {
    double p[5] = {0., 0., 0., 0., 0.};
#pragma unroll
    for (int q = 4; q < SWH_MPOLE_TERMS; q++) p[mp_order(q)] += sP[wv][q - 4];
    swh_multipole& M = out[c];
    for (int k = 0; k < 3; k++) M.CoM[k] = com[k];
    M.r_max = sqrt(rmax2);
    M.M[0] = (float)m0;
    M.M[1] = M.M[2] = M.M[3] = 0.f;
    M.power[0] = M.M[0];
    M.power[1] = 0.f;
    for (int o = 2; o <= 4; o++) M.power[o] = (float)sqrt(p[o]);
    M.max_softening = eps_max;
    M.min_old_a_grav_norm = oag_min;
  }
}

// One depth of the upward pass (src/space_split.c:340-440), one thread per
// split cell: the progeny's mass-weighted CoM, gravity_M2M of each child to
// it summed in double (the reference adds float copies), r_max = min(max_k
// (r_max_k + |CoM - CoM_k|), the CoM's distance to the farthest corner), the
// largest softening and smallest old |a| of the progeny, the power.
__global__ __launch_bounds__(64) void m2m_kernel(const int* __restrict__ list, int n,
                                                 const swh_gcell* __restrict__ cells,
                                                 swh_multipole* __restrict__ mp) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int c = list[k];
  const swh_gcell C = cells[c];
  double mass = 0., com[3] = {0., 0., 0.};
  for (int q = 0; q < 8; q++) {
    if (C.progeny[q] < 0) continue;
    const swh_multipole& B = mp[C.progeny[q]];
    const double m = (double)B.M[0];
    mass += m;
    for (int d = 0; d < 3; d++) com[d] += B.CoM[d] * m;
  }
  const double imass = 1. / mass;
  for (int d = 0; d < 3; d++) com[d] *= imass;
  double Mt[SWH_MPOLE_TERMS];
#pragma unroll
  for (int t = 0; t < SWH_MPOLE_TERMS; t++) Mt[t] = 0.;
  float eps_max = 0.f, oag_min = FLT_MAX;
  double r_max = 0.;
  for (int q = 0; q < 8; q++) {
    if (C.progeny[q] < 0) continue;
    const swh_multipole& B = mp[C.progeny[q]];
    const double dx = com[0] - B.CoM[0], dy = com[1] - B.CoM[1], dz = com[2] - B.CoM[2];
    double X[SWH_MPOLE_TERMS];
    xpowers<double>(dx, dy, dz, X);
    float Mb[SWH_MPOLE_TERMS];
#pragma unroll
    for (int t = 0; t < SWH_MPOLE_TERMS; t++) Mb[t] = B.M[t];
    m2m_t<0>(Mb, X, Mt);
    eps_max = fmaxf(eps_max, B.max_softening);
    oag_min = fminf(oag_min, B.min_old_a_grav_norm);
    r_max = fmax(r_max, B.r_max + sqrt(dx * dx + dy * dy + dz * dz));
  }
  double c2 = 0.;
  for (int d = 0; d < 3; d++) {
    const double e = com[d] > C.loc[d] + C.width[d] / 2. ? com[d] - C.loc[d]
                                                         : C.loc[d] + C.width[d] - com[d];
    c2 += e * e;
  }
  swh_multipole M;
  for (int d = 0; d < 3; d++) M.CoM[d] = com[d];
  M.r_max = fmin(r_max, sqrt(c2));
#pragma unroll
  for (int t = 0; t < SWH_MPOLE_TERMS; t++) M.M[t] = (float)Mt[t];
  M.M[0] = (float)mass;
  M.M[1] = M.M[2] = M.M[3] = 0.f;
  M.max_softening = eps_max;
  M.min_old_a_grav_norm = oag_min;
  mpole_power(M);
  mp[c] = M;
}

__global__ void gpack_kernel(GLayout L, char* __restrict__ aos, int64_t n, GSoA g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !g.active[i]) return;
  char* r = aos + i * L.stride;
  float* a = reinterpret_cast<float*>(r + L.a_grav);
  const double4 ac = g.acc[i];
  a[0] += (float)ac.x;
  a[1] += (float)ac.y;
  a[2] += (float)ac.z;
  *reinterpret_cast<float*>(r + L.potential) += (float)ac.w;
  g.acc[i] = make_double4(0., 0., 0., 0.);  // a second download adds nothing
}


// runner_iact_grav_pp_full / _truncated (gravity_iact.h:47-135) for one
// pair, fp64: h2 = max(eps_i^2, eps_j^2), h_inv = min(1/eps_i, 1/eps_j).
//
// Split in three so the common case runs branch-free: p2p_newton gives the
// unsoftened terms of every pair; p2p_soften replaces them for the pairs
// inside the larger softening (h2 = max(eps_i^2, eps_j^2), h_inv =
// min(1/eps_i, 1/eps_j)), which the callers reach only when a lane of the
// wave has r2 below the tile's largest h2 (emax = max(h2_i, max_j h2_j): one
// compare per pair instead of two, no divergent branch); p2p_trunc applies
// the long-range truncation. FLT_MIN joins the r2 sum (r2 + FLT_MIN == r2 in
// fp64 for every r2 above 1e-22, so the softening test is unchanged).
__device__ __forceinline__ void p2p_newton(double dx, double dy, double dz, double mass,
                                           double& r2, double& r_inv, double& f_ij,
                                           double& pot_ij) {
  r2 = fma(dx, dx, fma(dy, dy, fma(dz, dz, (double)FLT_MIN)));
  r_inv = rsqrt1_f64(r2);
  const double mr = mass * r_inv;
  f_ij = mr * (r_inv * r_inv);
  pot_ij = -mr;
}
__device__ __forceinline__ void p2p_soften(double r2, double r_inv, double e2i, double e2j,
                                           double hvi, double hvj, double mass, double& f_ij,
                                           double& pot_ij) {
  if ((r2 >= e2i) & (r2 >= e2j)) return;
  const double h_inv = hvj < hvi ? hvj : hvi;
  const double ui = r2 * r_inv * h_inv;
  const double mh = mass * h_inv;
  f_ij = mh * (h_inv * h_inv) * grav_force_eval(ui);
  pot_ij = mh * grav_pot_eval(ui);
}
// The long-range truncation of kernel_long_grav_eval (kernel_long_gravity.h:
// 160-190): with alpha = 1 / (1 + e^x), x = 2 r / r_s, the reference's
// corr_pot = 2 (1 - alpha e^x) and corr_f = 2 (1 + alpha ((1 - alpha) x -
// e^x)) are, since alpha e^x = 1 - alpha, 2 alpha and 2 alpha (1 + (1 -
// alpha) x); from E = e^-x (never overflows), alpha = E r and 1 - alpha = r
// with r = 1 / (1 + E). tworsi = 2 / r_s.
template <bool FMA3 = false>
__device__ __forceinline__ void p2p_trunc(double r2, double r_inv, double tworsi, double& f_ij,
                                          double& pot_ij) {
  const double x = r2 * r_inv * tworsi;
  const double E2 = exp_neg_f64_x2<FMA3>(x);      // 2 E
  const double r = rcp1_f64(fma(E2, 0.5, 1.));     // 1 - alpha
  const double a2 = E2 * r;                         // 2 alpha
  pot_ij *= a2;
  f_ij *= fma(a2 * r, x, a2);
}

// Nearest periodic image of a separation (|d| < 1.5 box): d - box rint(d /
// box), the same image as nearestf's branches (periodic.h:84-90) but three
// fp64 operations instead of two compares, two adds and four selects.
__device__ __forceinline__ double nearest_rint(double d, double box, double ibox) {
  return fma(-box, __builtin_rint(d * ibox), d);
}

// One LDS tile against this thread's IPER i-particles: every j entry is read
// once and used IPER times. SELF: the tile may hold an i itself (the
// i-leaf's own leaf), whose term is removed by a zero mass. MASK: the
// per-source activity act[k] (M2P takers) zeroes masses; without it every
// lane computes and the caller discards inactive i's. emax[k] = max(h2_i,
// the tile's largest h2_j): pairs at or beyond it are unsoftened.
template <bool TRUNC, bool PERIODIC, bool SELF, bool MASK, int IPER>
__device__ __forceinline__ void p2p_tile(const double* sx, const double* sy, const double* sz,
                                         const double* se2, const double* sh, const double* sm,
                                         int nt, const int* self_local, const double* xi,
                                         const double* yi, const double* zi, const double* hi2,
                                         const double* emax, const double* hv, const bool* act,
                                         double dimx, double dimy, double dimz, double tworsi,
                                         double* ax, double* ay, double* az, double* pot) {
  const double idimx = 1. / dimx, idimy = 1. / dimy, idimz = 1. / dimz;
  for (int t = 0; t < nt; t++) {
    const double xj = sx[t], yj = sy[t], zj = sz[t];
    const double mj = sm[t];
#pragma unroll
    for (int k = 0; k < IPER; k++) {
      double dx = xj - xi[k], dy = yj - yi[k], dz = zj - zi[k];
      if (PERIODIC) {
        dx = nearest_rint(dx, dimx, idimx);
        dy = nearest_rint(dy, dimy, idimy);
        dz = nearest_rint(dz, dimz, idimz);
      }
      double ms = mj;
      if (MASK) ms = act[k] ? ms : 0.;
      if (SELF) ms = t == self_local[k] ? 0. : ms;  // j == i: no term
      double r2, ri, f, pt;
      p2p_newton(dx, dy, dz, ms, r2, ri, f, pt);
      if (__builtin_expect(__any(r2 < emax[k]), 0))
        if (r2 < emax[k]) p2p_soften(r2, ri, hi2[k], se2[t], hv[k], sh[t], ms, f, pt);
      if (TRUNC) p2p_trunc(r2, ri, tworsi, f, pt);
      ax[k] = fma(f, dx, ax[k]);
      ay[k] = fma(f, dy, ay[k]);
      az[k] = fma(f, dz, az[k]);
      pot[k] += pt;
    }
  }
}

// Largest value over a wave (lanes without one pass 0).
__device__ __forceinline__ double wave_max_f64(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

// Per pair: which of this thread's i-particles take the source leaf's
// multipole instead (allow_mpole pairs only; block-uniform branch).
template <int IPER>
__device__ __forceinline__ void mpole_mask(const GSoA& g, const MacParams& P,
                                           const swh_leaf_pair& pr, const swh_leaf& J,
                                           const bool* act, const int* gi, bool* actp) {
  const bool mp = pr.allow_mpole && J.count > 1;
  if (!mp) {
#pragma unroll
    for (int k = 0; k < IPER; k++) actp[k] = act[k];
    return;
  }
  const MacSource B = mac_source(g.mp[pr.j]);
#pragma unroll
  for (int k = 0; k < IPER; k++) {
    bool use = false;
    if (act[k]) {
      const double4 p = g.pos[gi[k]];
      use = m2p_accept(P, B, (float)p.x, (float)p.y, (float)p.z, (float)p.w, g.oagn[gi[k]]);
    }
    actp[k] = act[k] && !use;
  }
}

// BLK threads per i-leaf workgroup, IPER i-particles per thread: 256 x 2 for
// the ~400-particle leaves of space_splitsize, 64 x 1 for the small leaves of
// a deep tree (cell_split_size 50), so the lanes are not left idle.
template <bool MPOLE, int BLK, int IPER>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(MPOLE ? 3 : 4))) void p2p_kernel(
    GSoA g, const swh_leaf* __restrict__ leaves, const int* __restrict__ pair_off,
    const swh_leaf_pair* __restrict__ pairs, int periodic, double dimx, double dimy,
    double dimz, double r_s_inv, MacParams mac, unsigned long long* counter) {
  __shared__ double sx[BLK], sy[BLK], sz[BLK], se2[BLK],
      sh[BLK];
  __shared__ double sm[BLK];  // (fp64: no conversion per pair)
  __shared__ double swmax[BLK / 64];  // per wave: the largest staged h2
  const int li = xcd_block_id();
  const swh_leaf L = leaves[li];
  const int p0 = pair_off[li], p1 = pair_off[li + 1];
  // no sources: leave acc alone (a tree's inner cells overlap their leaves,
  // whose blocks update the same particles)
  if (p0 == p1) return;
  unsigned long long nint = 0;
  for (int ibase = 0; ibase < L.count; ibase += BLK * IPER) {
    int gi[IPER], self_local[IPER];
    double xi[IPER], yi[IPER], zi[IPER], hi2[IPER], hv[IPER];
    double ax[IPER], ay[IPER], az[IPER], pot[IPER];
    bool act[IPER];
#pragma unroll
    for (int k = 0; k < IPER; k++) {
      const int local = ibase + k * BLK + (int)threadIdx.x;
      gi[k] = L.start + local;
      act[k] = local < L.count && g.active[gi[k]];
      const double4 p = act[k] ? g.pos[gi[k]] : make_double4(0., 0., 0., 1.);
      xi[k] = p.x; yi[k] = p.y; zi[k] = p.z;
      hi2[k] = p.w * p.w;
      hv[k] = act[k] ? g.hinv[gi[k]] : 1.;
      ax[k] = ay[k] = az[k] = pot[k] = 0.;
    }
    bool anyk = false;  // an i-slot past the first occupied in this wave
#pragma unroll
    for (int k = 1; k < IPER; k++) anyk = anyk || act[k];
    const bool full = __any(anyk);
    for (int q = p0; q < p1; q++) {
      const swh_leaf_pair pr = pairs[q];
      const swh_leaf J = leaves[pr.j];
      bool actp[IPER];  // act minus the particles taking this leaf's multipole
      if (MPOLE) {
        mpole_mask<IPER>(g, mac, pr, J, act, gi, actp);
      } else {
#pragma unroll
        for (int k = 0; k < IPER; k++) actp[k] = act[k];
      }
      for (int jbase = 0; jbase < J.count; jbase += BLK) {
        const int nt = min(BLK, J.count - jbase);
        __syncthreads();
        double e2 = 0.;
        if ((int)threadIdx.x < nt) {
          const int gj = J.start + jbase + (int)threadIdx.x;
          const double4 p = g.pos[gj];
          sx[threadIdx.x] = p.x;
          sy[threadIdx.x] = p.y;
          sz[threadIdx.x] = p.z;
          e2 = p.w * p.w;
          se2[threadIdx.x] = e2;
          sh[threadIdx.x] = g.hinv[gj];
          sm[threadIdx.x] = g.mass[gj];
        }
        e2 = wave_max_f64(e2);
        if ((threadIdx.x & 63) == 0) swmax[threadIdx.x / 64] = e2;
        __syncthreads();
        double tmax = swmax[0];
#pragma unroll
        for (int w = 1; w < BLK / 64; w++) tmax = fmax(tmax, swmax[w]);
        double emax[IPER];
        // the i-leaf's own particles can only sit in a tile of a leaf range
        // overlapping it (block-uniform test)
        const bool self = J.start + jbase < L.start + L.count && L.start < J.start + jbase + nt;
#pragma unroll
        for (int k = 0; k < IPER; k++) {
          emax[k] = act[k] ? fmax(hi2[k], tmax) : 0.;  // (inactive lanes: discarded)
          self_local[k] = gi[k] - (J.start + jbase);
          if (actp[k])
            nint += (unsigned long long)(nt - ((self_local[k] >= 0 && self_local[k] < nt) ? 1 : 0));
        }
// (a wave none of whose i-slots past the first is occupied -- the last waves
// of a ~391-gpart leaf's 512 slots -- runs the one-slot tile: half the pairs;
// for the plain Newtonian tiles, which keep the kernel within 128 VGPRs)
#define SWH_P2P_TILE(TR, PE, SE)                                                             \
  do {                                                                                       \
    if (SE || TR || PE || full)                                                              \
      p2p_tile<TR, PE, SE, MPOLE, IPER>(sx, sy, sz, se2, sh, sm, nt, self_local, xi, yi, zi,  \
                                        hi2, emax, hv, actp, dimx, dimy, dimz, 2. * r_s_inv, \
                                        ax, ay, az, pot);                                    \
    else                                                                                     \
      p2p_tile<TR, PE, SE, MPOLE, 1>(sx, sy, sz, se2, sh, sm, nt, self_local, xi, yi, zi,     \
                                     hi2, emax, hv, actp, dimx, dimy, dimz, 2. * r_s_inv,    \
                                     ax, ay, az, pot);                                       \
  } while (0)
        if (self) {
          if (pr.truncated) {
            if (periodic) SWH_P2P_TILE(true, true, true);
            else SWH_P2P_TILE(true, false, true);
          } else {
            if (periodic) SWH_P2P_TILE(false, true, true);
            else SWH_P2P_TILE(false, false, true);
          }
        } else {
          if (pr.truncated) {
            if (periodic) SWH_P2P_TILE(true, true, false);
            else SWH_P2P_TILE(true, false, false);
          } else {
            if (periodic) SWH_P2P_TILE(false, true, false);
            else SWH_P2P_TILE(false, false, false);
          }
        }
#undef SWH_P2P_TILE
      }
    }
#pragma unroll
    for (int k = 0; k < IPER; k++) {
      if (!act[k]) continue;
      double4 a = g.acc[gi[k]];
      a.x += ax[k];
      a.y += ay[k];
      a.z += az[k];
      a.w += pot[k];
      g.acc[gi[k]] = a;
    }
  }
  if (counter) {
    for (int o = 32; o > 0; o >>= 1) nint += __shfl_xor(nint, o);
    if ((threadIdx.x & 63) == 0 && nint) atomicAdd(counter, nint);
  }
}

// Small i-leaves (every leaf <= 64 gparts: a deep tree, cell_split_size 50)
// with batched sources: one wave per i-leaf, LPI = floor(64 / count) lanes
// per i-particle (up to 8), lane s of i taking tile entries s, s + LPI, ...
// (the LPI partial sums combined by shuffles at the end, so a 12-gpart leaf
// keeps 60 lanes busy instead of 12). The gparts of
// up to 32 consecutive P-P entries (up to kPPBatch of them) are gathered into
// the LDS tile at once: the chain of dependent loads (entry -> source leaf ->
// its gparts) and the wave barriers are paid once per batch, not once per
// source leaf (a cosmological tree has ~16 gparts per leaf and ~300 source
// leaves per i-leaf under the adaptive MAC). Each entry's truncation and M2P
// acceptance become bits (tmask: truncated entries; mmask, per i: the entries
// whose multipole this i takes instead, m2p_accept as in mpole_mask, tested
// one (i, entry) pair per lane); entries every active i takes through the
// multipole are not staged, and the entries that need per-pair masks (a
// mixed M2P decision, the i-leaf's own gparts: the self term, by tile
// position) are staged at the tile's tail, so only the tail runs the masked
// loop. Sources larger than the tile (no-cache entries against a whole cell)
// are staged in tile-sized chunks, every LDS index stays below kPPBatch.
//
// Periodic boxes: the staging shifts each source gpart to its image nearest
// the i-leaf's first gpart c. With e the i-leaf's extent around c, a staged
// source within L/2 - e of c (every dimension) is then the nearest image for
// every i of the leaf, so the pair loop needs no wrap; a tile holding any
// source past that bound (a pair separation near L/2: top-level cells of a
// tiny box) wraps every pair (nearest_rint), as nearestf does.
constexpr int kPPBatch = 256;
#ifndef SWH_P2P_EXP
#define SWH_P2P_EXP 0
#endif

// The batch kernel's pair loop over one staged tile: lane s of its i takes
// entries s, s + lpi, ... MASKED: per pair, the entry's M2P bit (pmask) and
// the self term (gpart index) zero the mass, and the pairs are counted;
// otherwise the caller counted them. TR: 0 / 1 = no / every entry truncated,
// 2 = per entry (tmask).
struct PairCtx {
  double4 pi;
  double hi2, hv, emax, tworsi, dimx, dimy, dimz, idimx, idimy, idimz;
};
struct TileLds {
  const double *sx, *sy, *sz, *sm;  // one array, kPPBatch apart: one address per pair
  const float* seps;  // softening: h2 = eps^2 and 1 / eps are exact from the float
  const unsigned char* sb;
};
template <bool MASKED, int TR>
__device__ __forceinline__ void batch_pairs(const TileLds& tl, const PairCtx& c, int t0, int lpi,
                                            int tn, bool wrap, unsigned int pmask,
                                            unsigned int tmask, int self_t, double& ax, double& ay,
                                            double& az, double& pot, unsigned int& nint) {
  // one address per pair: the loop runs over x's slot, y, z and the mass sit
  // kPPBatch slots on; the slot index is derived only where it is needed
  const double* const end = tl.sx + tn;
  for (const double* px = tl.sx + t0; px < end; px += lpi) {
    double dx = px[0] - c.pi.x, dy = px[kPPBatch] - c.pi.y, dz = px[2 * kPPBatch] - c.pi.z;
    if (wrap) {
      dx = nearest_rint(dx, c.dimx, c.idimx);
      dy = nearest_rint(dy, c.dimy, c.idimy);
      dz = nearest_rint(dz, c.dimz, c.idimz);
    }
    int b = 0;
    if (MASKED || TR == 2) b = tl.sb[px - tl.sx];
    double mass;
    if (MASKED) {
      const bool use = ((pmask >> b) & 1u) & ((int)(px - tl.sx) != self_t);
      nint += use;
      mass = use ? px[3 * kPPBatch] : 0.;
    } else {
      mass = px[3 * kPPBatch];
    }
    double r2, r_inv, f_ij, pot_ij;
    p2p_newton(dx, dy, dz, mass, r2, r_inv, f_ij, pot_ij);
    if (__builtin_expect(__any(r2 < c.emax), 0))
      if (r2 < c.emax) {
        const double ej = (double)tl.seps[px - tl.sx];
        p2p_soften(r2, r_inv, c.hi2, ej * ej, c.hv, 1. / ej, mass, f_ij, pot_ij);
      }
    if (TR == 1 || (TR == 2 && ((tmask >> b) & 1u)))
      p2p_trunc<true>(r2, r_inv, c.tworsi, f_ij, pot_ij);
    ax = fma(f_ij, dx, ax);
    ay = fma(f_ij, dy, ay);
    az = fma(f_ij, dz, az);
    pot += pot_ij;
  }
}

// MPOLE: mbits[entry] = the lanes whose i takes the entry's multipole (its
// MAC passed), for m2p_kernel, which then tests nothing itself.
template <bool MPOLE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void p2p_batch_kernel(
    GSoA g, const swh_leaf* __restrict__ leaves, const int* __restrict__ pair_off,
    const swh_leaf_pair* __restrict__ pairs, int periodic, double dimx, double dimy,
    double dimz, double r_s_inv, MacParams mac, unsigned long long* counter,
    unsigned long long* __restrict__ mbits) {
  // 37 B per staged gpart (9.6 KB): four waves per SIMD
  __shared__ double stile[4 * kPPBatch];  // x, y, z, mass
  double* const sx = stile;
  double* const sy = stile + kPPBatch;
  double* const sz = stile + 2 * kPPBatch;
  double* const sm = stile + 3 * kPPBatch;
  __shared__ float seps[kPPBatch];
  __shared__ unsigned char sb[kPPBatch];
  __shared__ int boff[32], bstart[32], bent[32];  // per slot: position, gpart, entry
  // the MAC tests' scratch (1.5 KB) over sx: used between tiles only
  static_assert(32 * sizeof(MacSource) + 64 * 4 + 32 * 8 + 32 * 4 <= sizeof(double) * kPPBatch,
                "MAC scratch fits sx");
  MacSource* const mac_ms = reinterpret_cast<MacSource*>(sx);
  unsigned long long* const mac_qmask =
      reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(sx) + 32 * sizeof(MacSource));
  unsigned int* const mac_imask = reinterpret_cast<unsigned int*>(mac_qmask + 32);
  int* const mac_q = reinterpret_cast<int*>(mac_imask + 64);
  const int li = xcd_block_id();
  const swh_leaf L = leaves[li];
  const int p0 = pair_off[li], p1 = pair_off[li + 1];
  if (p0 == p1) return;  // (inner cells overlap their leaves: leave acc alone)
  const int lane = (int)threadIdx.x;
  // lanes per i: as many as fit (not only powers of two: a 20-gpart leaf
  // keeps 60 lanes busy with 3, not 40 with 2; 91% of the lanes of a
  // cosmological tree's leaves against 80%)
  const int lpi = L.count >= 64 ? 1 : min(8, 64 / max(L.count, 1));  // wave-uniform
  const int il = lane / lpi, s = lane % lpi;
  const int gi = L.start + il;
  const bool act = il < L.count && g.active[gi];
  const double4 pi = act ? g.pos[gi] : make_double4(0., 0., 0., 1.);
  const double hi2 = pi.w * pi.w;
  const double hv = act ? g.hinv[gi] : 1.;
  const double tworsi = 2. * r_s_inv;
  const double idimx = 1. / dimx, idimy = 1. / dimy, idimz = 1. / dimz;
  // the MAC's float view of i (gravity_cache_populate)
  const float4 pf = make_float4((float)pi.x, (float)pi.y, (float)pi.z, (float)pi.w);
  const float oag = MPOLE && act ? g.oagn[gi] : 0.f;
  const unsigned long long actmask = __ballot(act);  // the lanes of active i's
  // the MAC's test lanes: lane = kk * count + ii tests i-slot ii (its data
  // from lane ii * lpi), epr entries per round; ibits = the lanes of ii
  const int nI = max(L.count, 1), epr = max(1, 64 / nI);
  const int kk = lane / nI, ii = lane - kk * nI;
  const int tsrc = ii * lpi;  // < 64: count * lpi <= 64
  float4 t_pf = make_float4(0.f, 0.f, 0.f, 0.f);
  float t_oag = 0.f;
  bool t_act = false;
  if (MPOLE) {
    t_pf = make_float4(__shfl(pf.x, tsrc), __shfl(pf.y, tsrc), __shfl(pf.z, tsrc),
                       __shfl(pf.w, tsrc));
    t_oag = __shfl(oag, tsrc);
    t_act = __shfl((int)act, tsrc) != 0 && kk < epr && ii < L.count;
  }
  const unsigned long long ibits = ((1ull << lpi) - 1ull) << tsrc;
  // periodic: the i-leaf's first gpart c and the leaf's extent around it
  double cx = 0., cy = 0., cz = 0., lim_x = 0., lim_y = 0., lim_z = 0.;
  if (periodic) {
    const double4 c = g.pos[L.start];
    cx = c.x;
    cy = c.y;
    cz = c.z;
    double e = 0.;
    if (il < L.count) {
      const double4 q = g.pos[gi];
      e = fmax(fabs(q.x - cx), fmax(fabs(q.y - cy), fabs(q.z - cz)));
    }
    e = wave_max_f64(e);
    lim_x = 0.5 * dimx * (1. - 1e-12) - e;
    lim_y = 0.5 * dimy * (1. - 1e-12) - e;
    lim_z = 0.5 * dimz * (1. - 1e-12) - e;
  }
  double ax = 0., ay = 0., az = 0., pot = 0.;
  unsigned int nint = 0;
  for (int qb = p0; qb < p1;) {
    // lane q < 32 reads entry qb + q: its source leaf, flags, the batch prefix
    int cnt = 0, jst = 0, jl = 0;
    bool tr = false, am = false;
    if (lane < 32 && qb + lane < p1) {
      const swh_leaf_pair pr = pairs[qb + lane];
      const swh_leaf J = leaves[pr.j];
      cnt = J.count;
      jst = J.start;
      jl = pr.j;
      tr = pr.truncated != 0;
      am = pr.allow_mpole && J.count > 1;
    }
    // every lane loads its own entry's multipole fields at once (a chain of
    // one load per tested entry otherwise: the kernel's largest stall)
    MacSource msrc{};
    if (MPOLE && am) msrc = mac_source(g.mp[jl]);
    const int inc = wave_incl_scan(cnt);
    // the batch: the entries whose gparts fit the tile (a prefix). A source
    // larger than the tile (a split cell of a no-cache P-P entry: a
    // single-gpart cell against a whole cell) is a batch of its own, staged
    // in tile-sized chunks.
    const unsigned long long fit = __ballot(cnt > 0 && inc <= kPPBatch);
    const int B = fit ? __popcll(fit) : 1;
    const unsigned int tmask = (unsigned int)__ballot(lane < B && tr);
    unsigned int mmask = 0;  // the entries this i takes through their multipole
    unsigned long long mine = 0;  // lane q < B: entry q's accepting lanes
    if (MPOLE) {
      // The MAC tests of the batch, one (i, entry) test per lane: the entries
      // with allow_mpole are listed in LDS (scratch over the tile, whose last
      // readers are done) and lane (kk, ii) tests i-slot ii against entries
      // kk, kk + EPR, ...; the results gather by LDS OR into per-i entry masks
      // (mmask) and per-entry lane masks (mbits).
      const unsigned long long amb = __ballot(lane < B && am);
      if (amb) {
        const int nq = __popcll(amb);
        wave_sync();
        if (lane < B && am) {
          const int r = __popcll(amb & ((1ull << lane) - 1ull));
          mac_ms[r] = msrc;
          mac_q[r] = lane;
        }
        mac_imask[lane] = 0u;
        if (lane < 32) mac_qmask[lane] = 0ull;
        wave_sync();
        if (t_act && SWH_P2P_EXP != 3)
          for (int k = kk; k < nq; k += epr)
            if (m2p_accept(mac, mac_ms[k], t_pf.x, t_pf.y, t_pf.z, t_pf.w, t_oag)) {
              const int q = mac_q[k];
              atomicOr(&mac_imask[ii], 1u << q);
              atomicOr(&mac_qmask[q], ibits);
            }
        wave_sync();
        if (act) mmask = mac_imask[il];
        if (lane < B) mine = mac_qmask[lane];
      }
      if (lane < B) mbits[qb + lane] = mine;
    }
    // Entries every active i takes through the multipole are not staged at
    // all (the M2P acceptance is nearly always uniform over a small leaf);
    // only the mixed ones need per-pair masks.
    // (allm bit q: every active lane takes entry q's multipole; anym: some)
    const unsigned long long mact = mine & actmask;
    const unsigned int allm = (unsigned int)__ballot(mact == actmask);
    const unsigned int anym = (unsigned int)__ballot(mact != 0ull);
    const bool inb = lane < B;
    const int cnt2 = (inb && ((allm >> lane) & 1u)) ? 0 : (inb ? cnt : 0);
    // Staging order: first the entries every i takes alike (plain), then the
    // ones that need per-pair masks -- a multipole for some of the i's only
    // (mixed), or the i-leaf's own gparts (self terms to drop) -- so only the
    // tile's tail runs the masked pair loop. slot = an entry's place in that
    // order, pos = its first staged position.
    const bool ownq = cnt2 > 0 && jst < L.start + L.count && L.start < jst + cnt;
    const bool maskq = inb && (ownq || (((anym & ~allm) >> lane) & 1u));
    const int cA = maskq ? 0 : cnt2, cM = maskq ? cnt2 : 0;
    const unsigned long long ballA = __ballot(inb && !maskq), ballM = __ballot(maskq);
    const int incA = wave_incl_scan(cA), incM = ballM ? wave_incl_scan(cM) : 0;
    const int totalA = __builtin_amdgcn_readlane(incA, 63);
    const int total2 = SWH_P2P_EXP == 2 ? 0 : totalA + __builtin_amdgcn_readlane(incM, 63);
    const unsigned long long below = (1ull << lane) - 1ull;
    const int slot = maskq ? __popcll(ballA) + __popcll(ballM & below) : __popcll(ballA & below);
    const int posq = maskq ? totalA + incM - cM : incA - cA;
    // plain entries all / none / some truncated
    const unsigned int bA = (unsigned int)ballA, bM = (unsigned int)ballM;
    const int trA = (tmask & bA) == bA ? 1 : (tmask & bA) == 0u ? 0 : 2;
    const bool trM = (tmask & bM) == bM;  // every masked entry truncated
    // per i: the entries it takes by P2P (inactive i: none)
    const unsigned int pmask = act ? ~mmask : 0u;
    for (int jb = 0; jb < total2; jb += kPPBatch) {
      const int tn = min(kPPBatch, total2 - jb);
      wave_sync();  // the previous tile's readers are done
      if (inb) {
        boff[slot] = posq;  // (an unstaged entry: its successor's offset)
        bstart[slot] = jst;
        bent[slot] = lane;
      }
      wave_sync();
      double e2max = 0.;
      bool far = false;
      for (int k = lane; k < tn; k += 64) {
        const int e = jb + k;  // the batch's e-th gpart
        int b = 0;  // its entry's slot: the largest b with boff[b] <= e
        for (int st = 16; st > 0; st >>= 1)
          if (b + st < B && boff[b + st] <= e) b += st;
        const int gj = bstart[b] + (e - boff[b]);
        const double4 p = g.pos[gj];
        double px = p.x, py = p.y, pz = p.z;
        if (periodic) {
          // (no shift: the position itself, bit for bit)
          px = fma(-dimx, __builtin_rint((px - cx) * idimx), px);
          py = fma(-dimy, __builtin_rint((py - cy) * idimy), py);
          pz = fma(-dimz, __builtin_rint((pz - cz) * idimz), pz);
          far |= (fabs(px - cx) > lim_x) | (fabs(py - cy) > lim_y) | (fabs(pz - cz) > lim_z);
        }
        sx[k] = px;
        sy[k] = py;
        sz[k] = pz;
        seps[k] = (float)p.w;  // (the gpart's float epsilon, exactly)
        e2max = fmax(e2max, p.w * p.w);
        sm[k] = (double)g.mass[gj];
        sb[k] = (unsigned char)bent[b];
      }
      const double emax = act ? fmax(hi2, wave_max_f64(e2max)) : 0.;
      const bool wrap = periodic && __any(far);
      wave_sync();
      // The plain part [0, tA): no per-pair mask, the pairs counted per lane;
      // every or no entry truncated -> no per-pair truncation bit. The
      // masked part [tA, tn) tests each pair's entry bit and self index.
      const int tA = SWH_P2P_EXP == 4 ? tn : min(tn, max(0, totalA - jb));
      const PairCtx pc{pi, hi2, hv, emax, tworsi, dimx, dimy, dimz, idimx, idimy, idimz};
      const TileLds tl{sx, sy, sz, sm, seps, sb};
      // this i's own tile position (its self term), or -1
      int self_t = -1;
      for (unsigned long long m = __ballot(inb && ownq); m; m &= m - 1) {
        const int q = __ffsll((long long)m) - 1;
        const int js = __builtin_amdgcn_readlane(jst, q), jc = __builtin_amdgcn_readlane(cnt, q);
        const int t = __builtin_amdgcn_readlane(posq, q) + (gi - js) - jb;
        if (gi >= js && gi < js + jc && t >= 0 && t < tn) self_t = t;
      }
#if SWH_P2P_EXP == 1 || SWH_P2P_EXP == 3  // experiments (wrong results): 1 staging + MAC
// only, 2 entries + MAC only, 3 staging only
#define SWH_BATCH_PAIRS(M, T, T0, T1) (void)0
#else
#define SWH_BATCH_PAIRS(M, T, T0, T1)                                                          \
  batch_pairs<M, T>(tl, pc, (T0) + s, lpi, T1, wrap, pmask, tmask, self_t, ax, ay, az, pot, nint)
#endif
      if (tA > 0) {
        if (act) nint += (unsigned int)(tA > s ? (tA - s + lpi - 1) / lpi : 0);
        if (trA == 1) SWH_BATCH_PAIRS(false, 1, 0, tA);
        else if (trA == 0) SWH_BATCH_PAIRS(false, 0, 0, tA);
        else SWH_BATCH_PAIRS(false, 2, 0, tA);
      }
      if (tA < tn) {
        if (trM) SWH_BATCH_PAIRS(true, 1, tA, tn);
        else SWH_BATCH_PAIRS(true, 2, tA, tn);
      }
#undef SWH_BATCH_PAIRS
    }
    qb += B;
  }
  // combine the LPI lanes of each i into its first (lane il * lpi)
  {
    const double bx = ax, by = ay, bz = az, bp = pot;
    for (int o = 1; o < lpi; o++) {
      ax += __shfl(bx, lane + o);
      ay += __shfl(by, lane + o);
      az += __shfl(bz, lane + o);
      pot += __shfl(bp, lane + o);
    }
  }
  if (act && s == 0) {
    double4 a = g.acc[gi];
    a.x += ax;
    a.y += ay;
    a.z += az;
    a.w += pot;
    g.acc[gi] = a;
  }
  if (counter) {
    unsigned long long n = nint;
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if (lane == 0 && n) atomicAdd(counter, n);
  }
}

// fp32 mode (SWH_PRECISION_F32): the reference's own float arithmetic,
// operation by operation (gravity_iact.h), for parity with the float runner.
__global__ __launch_bounds__(kGravBlock) void p2p_kernel_f32(
    GSoA g, const swh_leaf* __restrict__ leaves, const int* __restrict__ pair_off,
    const swh_leaf_pair* __restrict__ pairs, int periodic, double dimx, double dimy,
    double dimz, float r_s_inv, MacParams mac, unsigned long long* counter) {
  using T = float;
  __shared__ double sx[kGravBlock], sy[kGravBlock], sz[kGravBlock];
  __shared__ float se[kGravBlock], sm[kGravBlock];
  const int li = xcd_block_id();
  const swh_leaf L = leaves[li];
  const int p0 = pair_off[li], p1 = pair_off[li + 1];
  // no sources: leave acc alone (a tree's inner cells overlap their leaves,
  // whose blocks update the same particles)
  if (p0 == p1) return;
  unsigned long long nint = 0;
  for (int ibase = 0; ibase < L.count; ibase += kGravBlock * kIPer) {
    int gi[kIPer];
    double xi[kIPer], yi[kIPer], zi[kIPer];
    T hi[kIPer], ax[kIPer], ay[kIPer], az[kIPer], pot[kIPer];
    bool act[kIPer];
#pragma unroll
    for (int k = 0; k < kIPer; k++) {
      const int local = ibase + k * kGravBlock + (int)threadIdx.x;
      gi[k] = L.start + local;
      act[k] = local < L.count && g.active[gi[k]];
      const double4 p = act[k] ? g.pos[gi[k]] : make_double4(0., 0., 0., 1.);
      xi[k] = p.x; yi[k] = p.y; zi[k] = p.z;
      hi[k] = (T)p.w;
      ax[k] = ay[k] = az[k] = pot[k] = (T)0;
    }
    for (int q = p0; q < p1; q++) {
      const swh_leaf_pair pr = pairs[q];
      const swh_leaf J = leaves[pr.j];
      bool actp[kIPer];
      mpole_mask<kIPer>(g, mac, pr, J, act, gi, actp);
      for (int jbase = 0; jbase < J.count; jbase += kGravBlock) {
        const int nt = min(kGravBlock, J.count - jbase);
        __syncthreads();
        if ((int)threadIdx.x < nt) {
          const int gj = J.start + jbase + (int)threadIdx.x;
          const double4 p = g.pos[gj];
          sx[threadIdx.x] = p.x;
          sy[threadIdx.x] = p.y;
          sz[threadIdx.x] = p.z;
          se[threadIdx.x] = (float)p.w;
          sm[threadIdx.x] = g.mass[gj];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kIPer; k++) {
          if (!actp[k]) continue;
          const int self_local = gi[k] - (J.start + jbase);
          for (int t = 0; t < nt; t++) {
            if (t == self_local) continue;
            double dxd = sx[t] - xi[k], dyd = sy[t] - yi[k], dzd = sz[t] - zi[k];
            if (periodic) {
              dxd = dxd > 0.5 * dimx ? dxd - dimx : (dxd < -0.5 * dimx ? dxd + dimx : dxd);
              dyd = dyd > 0.5 * dimy ? dyd - dimy : (dyd < -0.5 * dimy ? dyd + dimy : dyd);
              dzd = dzd > 0.5 * dimz ? dzd - dimz : (dzd < -0.5 * dimz ? dzd + dimz : dzd);
            }
            const T dx = (T)dxd, dy = (T)dyd, dz = (T)dzd;
            const T r2 = dx * dx + dy * dy + dz * dz;
            const T h = tmax(hi[k], se[t]);
            const T h_inv = (T)1 / h;
            T f, pt;
            if (pr.truncated)
              iact_grav_pp<T, true>(r2, h * h, h_inv, h_inv * h_inv * h_inv, (T)sm[t], r_s_inv,
                                    f, pt);
            else
              iact_grav_pp<T, false>(r2, h * h, h_inv, h_inv * h_inv * h_inv, (T)sm[t],
                                     r_s_inv, f, pt);
            ax[k] += f * dx; ay[k] += f * dy; az[k] += f * dz; pot[k] += pt;
          }
          nint += (unsigned long long)(nt - ((self_local >= 0 && self_local < nt) ? 1 : 0));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kIPer; k++) {
      if (!act[k]) continue;
      double4 a = g.acc[gi[k]];
      a.x += (double)ax[k];
      a.y += (double)ay[k];
      a.z += (double)az[k];
      a.w += (double)pot[k];
      g.acc[gi[k]] = a;
    }
  }
  if (counter) {
    for (int o = 32; o > 0; o >>= 1) nint += __shfl_xor(nint, o);
    if ((threadIdx.x & 63) == 0 && nint) atomicAdd(counter, nint);
  }
}

// Stats only (swh_grav_tree with stats, after the step): the P2P pairs of
// truncated entries, SURVEY 8d's 43-flop pairs. One wave per i-leaf, a lane
// per active i (64 at a time); an i that took an allow_mpole entry through
// its multipole (the batch kernel's MAC bits when it ran, m2p_accept as in
// mpole_mask otherwise) has no pairs with it; the self pair is not one.
__global__ __launch_bounds__(64) void pp_trunc_count_kernel(
    GSoA g, const swh_leaf* __restrict__ leaves, const int* __restrict__ pair_off,
    const swh_leaf_pair* __restrict__ pairs, MacParams mac, int any_mpole,
    const unsigned long long* __restrict__ mbits, unsigned long long* counter) {
  const int li = blockIdx.x;
  const swh_leaf L = leaves[li];
  const int p0 = pair_off[li], p1 = pair_off[li + 1];
  if (p0 == p1) return;
  const int lane = (int)threadIdx.x;
  // the batch kernel's lanes per i (its MAC bits are per lane)
  const int lpi = L.count >= 64 ? 1 : min(8, 64 / max(L.count, 1));
  unsigned long long n = 0;
  for (int ib = 0; ib < L.count; ib += 64) {
    const int il = ib + lane;
    const int gi = L.start + il;
    const bool act = il < L.count && g.active[gi];
    const double4 pi = act ? g.pos[gi] : make_double4(0., 0., 0., 1.);
    for (int q = p0; q < p1; q++) {
      const swh_leaf_pair pr = pairs[q];
      if (!pr.truncated) continue;
      const swh_leaf J = leaves[pr.j];
      bool m2p = false;
      if (any_mpole && pr.allow_mpole && J.count > 1 && act) {
        if (mbits)
          m2p = (mbits[q] >> (il * lpi)) & 1ull;
        else
          m2p = m2p_accept(mac, mac_source(g.mp[pr.j]), (float)pi.x, (float)pi.y, (float)pi.z,
                           (float)pi.w, g.oagn[gi]);
      }
      if (act && !m2p)
        n += (unsigned long long)(J.count - ((gi >= J.start && gi < J.start + J.count) ? 1 : 0));
    }
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  if (lane == 0 && n) atomicAdd(counter, n);
}

// M2P of the allow_mpole pairs (runner_dopair_grav_pm_full / _truncated,
// runner_doiact_grav.c:911-1200): every active i of the i-leaf that passes
// the MAC against source leaf j's multipole. Runs after p2p_kernel on the
// same stream (both add into acc).
// SMALL (every leaf <= 64 gparts, one wave per leaf): the accepted (i,
// entry) pairs are queued and evaluated 64 at a time; otherwise a thread per
// i walks the whole list.
// The pair's M2P terms {potential, a_x, a_y, a_z} for i-leaf gpart gi and
// the multipole of source leaf j.
template <typename T>
__device__ __forceinline__ void m2p_pair(const GSoA& g, int gi, int j, bool truncated,
                                         int periodic, double dimx, double dimy, double dimz,
                                         double r_s_inv, T* f) {
  const swh_multipole& M = g.mp[j];
  const double4 p = g.pos[gi];
  double dx = M.CoM[0] - p.x, dy = M.CoM[1] - p.y, dz = M.CoM[2] - p.z;
  if (periodic) {
    dx = dx > 0.5 * dimx ? dx - dimx : (dx < -0.5 * dimx ? dx + dimx : dx);
    dy = dy > 0.5 * dimy ? dy - dimy : (dy < -0.5 * dimy ? dy + dimy : dy);
    dz = dz > 0.5 * dimz ? dz - dimz : (dz < -0.5 * dimz ? dz + dimz : dz);
  }
  const T eps = (T)fmaxf((float)p.w, M.max_softening);
  m2p<T>(M.M, (T)dx, (T)dy, (T)dz, eps, truncated, (T)r_s_inv, f);
}

// Small leaves after p2p_batch_kernel<true> (fp64): one wave per leaf, the
// MAC already decided there (mbits: per entry, the accepting lanes, lpi per
// i). The entries are read 64 at a time; each lane expands its entry's
// accepting i's into an LDS queue at its scanned offset (entry-major, so a
// round's multipole reads are a few multipoles broadcast from their cache
// lines), and the queue is evaluated 64 pairs per round with every lane busy
// (the M2P, ~500 fp64 instructions; a chunk's last < 64 pairs wait for the
// next chunk's, so rounds run full), each lane adding its terms to its i's
// LDS accumulator with ds_add_f64. The MAC tests were ~55% of the wave time
// of a kernel that repeated them.
template <typename T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void m2p_bits_kernel(
    GSoA g, const swh_leaf* __restrict__ leaves, const int* __restrict__ pair_off,
    const swh_leaf_pair* __restrict__ pairs, const unsigned long long* __restrict__ mbits,
    int periodic, double dimx, double dimy, double dimz, double r_s_inv,
    unsigned long long* counter) {
  const int li = xcd_block_id();
  const swh_leaf L = leaves[li];
  const int p0 = pair_off[li], p1 = pair_off[li + 1];
  if (p0 == p1) return;  // no sources (a tree's inner cells)
  // the entries of the last two chunks that had any (halves of cj / ctr), and
  // the queue: pairs left from earlier chunks (< 64) at its front
  __shared__ int cj[128];
  __shared__ unsigned char ctr[128];
  __shared__ unsigned short q[64 * 64 + 64];  // i << 8 | entry slot
  __shared__ T accs[4][64];
  const int lane = (int)threadIdx.x;
  // the P2P kernel's lanes: lpi per i, i = lane / lpi (its lane s = 0 stands for it)
  const int lpi = L.count >= 64 ? 1 : min(8, 64 / max(L.count, 1));
  const unsigned long long smask = __ballot(lane % lpi == 0 && lane / lpi < L.count);
  const unsigned int inv = (65536u + (unsigned)lpi - 1u) / (unsigned)lpi;  // b / lpi, b < 64
  for (int c = 0; c < 4; c++) accs[c][lane] = (T)0;
  unsigned long long nm = 0;
  int nq = 0, half = 0, qb = p0;
  while (qb < p1 || nq > 0) {
    int n_eval = nq;  // (the list's end)
    if (qb < p1) {
      unsigned long long m = 0;
      int jl = 0;
      unsigned char tr = 0;
      if (qb + lane < p1) {
        m = mbits[qb + lane] & smask;
        if (m) {
          const swh_leaf_pair pr = pairs[qb + lane];
          jl = pr.j;
          tr = pr.truncated != 0;
        }
      }
      const int c = __popcll(m);
      const int inc = wave_incl_scan(c);
      const int tot = __builtin_amdgcn_readlane(inc, 63);
      wave_sync();  // the previous round's readers are done
      // left pairs naming the half this chunk would overwrite (two chunks
      // back) are evaluated first, and the chunk is read again
      if (!(tot > 0 && __any(lane < nq && ((q[lane] & 64u) != 0u) == (half != 0)))) {
        if (tot > 0) {
          cj[half * 64 + lane] = jl;
          ctr[half * 64 + lane] = tr;
          int at = nq + inc - c;
          for (unsigned long long mm = m; mm; mm &= mm - 1) {
            const unsigned int b = (unsigned int)(__ffsll((long long)mm) - 1);
            q[at++] = (unsigned short)(((b * inv) >> 16) << 8 | (unsigned int)(half * 64 + lane));
          }
          wave_sync();
          nm += (unsigned long long)tot;
          nq += tot;
          half ^= 1;
        }
        qb += 64;
        // full rounds; the rest (< 64) waits for the next chunk's pairs
        n_eval = qb < p1 ? (nq & ~63) : nq;
      }
    }
    if (n_eval > 0) {
      for (int r0 = 0; r0 < n_eval; r0 += 64) {
        if (r0 + lane < n_eval) {
          const unsigned int e = q[r0 + lane];
          const int il = (int)(e >> 8), k = (int)(e & 255u);
          T f[4];
          m2p_pair<T>(g, L.start + il, cj[k], ctr[k] != 0, periodic, dimx, dimy, dimz, r_s_inv,
                      f);
          for (int c2 = 0; c2 < 4; c2++) atomicAdd(&accs[c2][il], f[c2]);
        }
      }
      const int left = nq - n_eval;
      unsigned short v = 0;
      if (lane < left) v = q[n_eval + lane];
      wave_sync();
      if (lane < left) q[lane] = v;
      wave_sync();
      nq = left;
    }
  }
  wave_sync();
  const T F[4] = {accs[0][lane], accs[1][lane], accs[2][lane], accs[3][lane]};
  if (lane < L.count && (F[0] != (T)0 || F[1] != (T)0 || F[2] != (T)0 || F[3] != (T)0)) {
    const int gi = L.start + lane;
    double4 a = g.acc[gi];
    a.x += (double)F[1];
    a.y += (double)F[2];
    a.z += (double)F[3];
    a.w += (double)F[0];
    g.acc[gi] = a;
  }
  if (counter && lane == 0 && nm) atomicAdd(counter + 1, nm);
}

template <typename T, bool SMALL>
__global__ __launch_bounds__(kGravBlock) __attribute__((amdgpu_waves_per_eu(SMALL ? 3 : 1))) void m2p_kernel(
    GSoA g, const swh_leaf* __restrict__ leaves, const int* __restrict__ pair_off,
    const swh_leaf_pair* __restrict__ pairs, int periodic, double dimx, double dimy,
    double dimz, double r_s_inv, MacParams mac, unsigned long long* counter) {
  const int li = xcd_block_id();
  const swh_leaf L = leaves[li];
  const int p0 = pair_off[li], p1 = pair_off[li + 1];
  if (p0 == p1) return;  // no sources (a tree's inner cells)
  unsigned long long nm = 0;
  if (SMALL) {
    // One wave per leaf (<= 64 gparts). The P-P entries are read 64 at a
    // time (one per lane, loads in parallel) and their allow_mpole ones --
    // ~7% of a cosmological tree's entries -- compacted into LDS until 64
    // have gathered (or the list ends): one group. The wave then tests every
    // (entry, active i) pair of the group against the MAC, 64 pairs per
    // iteration in entry-major order (lane t of an iteration holds pair t0 +
    // t = entry * nact + i), and appends the accepted ones to a 128-slot LDS
    // ring; whenever 64 are queued (and once the tests are done) they are
    // evaluated together with every lane busy (the M2P, ~500 fp64
    // instructions, no longer runs with only the lanes whose pair passed
    // enabled). Entry-major keeps a round's multipole reads to a few
    // multipoles (broadcast from the cache lines) where i-major order read a
    // different one per lane; each lane adds its terms to its i's LDS
    // accumulator with ds_add_f64.
    __shared__ float4 spi[64];  // i: float position and softening (the MAC's inputs)
    __shared__ float soag[64];  // i: old |a|
    __shared__ unsigned char actl[64];  // the active i's, compacted
    __shared__ int cj[128];             // gathered allow_mpole entries: source leaf
    __shared__ unsigned char ctr[128];  //   and truncation flag
    __shared__ MacSource sb[64];        // the group's MAC inputs
    __shared__ unsigned short q[128];   // accepted pairs, a ring: i << 8 | entry
    __shared__ T accs[4][64];
    const int lane = (int)threadIdx.x;
    const unsigned long long below = (1ull << lane) - 1ull;
    const int gi = L.start + lane;
    const bool acti = lane < L.count && g.active[gi];
    const double4 pl = acti ? g.pos[gi] : make_double4(0., 0., 0., 1.);
    spi[lane] = make_float4((float)pl.x, (float)pl.y, (float)pl.z, (float)pl.w);
    soag[lane] = acti ? g.oagn[gi] : 0.f;
    for (int c = 0; c < 4; c++) accs[c][lane] = (T)0;
    const unsigned long long actm = __ballot(acti);
    const int nact = __popcll(actm);
    if (nact == 0) return;  // nothing active in this leaf
    if (acti) actl[__popcll(actm & below)] = (unsigned char)lane;
    int nbuf = 0;
    for (int qb = p0; qb < p1 || nbuf > 0; qb += 64) {
      if (qb < p1) {
        bool am = false;
        int jl = 0;
        unsigned char tr = 0;
        if (qb + lane < p1) {
          const swh_leaf_pair pr = pairs[qb + lane];
          am = pr.allow_mpole && leaves[pr.j].count > 1;
          jl = pr.j;
          tr = pr.truncated != 0;
        }
        const unsigned long long m = __ballot(am);
        wave_sync();  // the previous group's readers are done
        if (am) {
          const int r = nbuf + __popcll(m & below);
          cj[r] = jl;
          ctr[r] = tr;
        }
        nbuf += __popcll(m);
        wave_sync();
        if (nbuf < 64 && qb + 64 < p1) continue;  // gather more first
      }
      const int ne = nbuf < 64 ? nbuf : 64;
      if (ne == 0) continue;
      if (lane < ne) sb[lane] = mac_source(g.mp[cj[lane]]);
      wave_sync();
      const int ntest = nact * ne;
      int k = lane / nact, ii = lane - k * nact;  // this lane's pair: (actl[ii], k)
      const int dk = 64 / nact, di = 64 - dk * nact;
      int t0 = 0, qh = 0, qt = 0;  // tests done; ring head and tail
      while (t0 < ntest || qt > qh) {
        if (t0 < ntest && qt - qh < 64) {
          bool ok = false;
          int il = 0;
          if (t0 + lane < ntest) {
            il = actl[ii];
            const float4 p = spi[il];
            ok = m2p_accept(mac, sb[k], p.x, p.y, p.z, p.w, soag[il]);
          }
          const unsigned long long okm = __ballot(ok);
          if (ok) q[(qt + __popcll(okm & below)) & 127] = (unsigned short)(il << 8 | k);
          qt += __popcll(okm);
          t0 += 64;
          k += dk;
          ii += di;
          if (ii >= nact) {
            ii -= nact;
            k++;
          }
          wave_sync();
          continue;
        }
        const int nr = qt - qh < 64 ? qt - qh : 64;
        const bool valid = lane < nr;
        int il = -1;
        T f[4] = {(T)0, (T)0, (T)0, (T)0};
        if (valid) {
          const unsigned int e = q[(qh + lane) & 127];
          il = (int)(e >> 8);
          const int kk = (int)(e & 255u);
          m2p_pair<T>(g, L.start + il, cj[kk], ctr[kk] != 0, periodic, dimx, dimy, dimz,
                      r_s_inv, f);
        }
        if (valid)
          for (int c = 0; c < 4; c++) atomicAdd(&accs[c][il], f[c]);
        nm += (unsigned long long)nr;
        qh += nr;
        wave_sync();
      }
      // the entries past the group move to the front of the buffer
      const int rest = nbuf - ne;
      int jl = 0;
      unsigned char tr = 0;
      if (lane < rest) {
        jl = cj[64 + lane];
        tr = ctr[64 + lane];
      }
      wave_sync();
      if (lane < rest) {
        cj[lane] = jl;
        ctr[lane] = tr;
      }
      nbuf = rest;
      wave_sync();
    }
    wave_sync();
    const T F[4] = {accs[0][lane], accs[1][lane], accs[2][lane], accs[3][lane]};
    if (acti && (F[0] != (T)0 || F[1] != (T)0 || F[2] != (T)0 || F[3] != (T)0)) {
      double4 a = g.acc[gi];
      a.x += (double)F[1];
      a.y += (double)F[2];
      a.z += (double)F[3];
      a.w += (double)F[0];
      g.acc[gi] = a;
    }
    if (counter && lane == 0 && nm) atomicAdd(counter + 1, nm);
    return;
  }
  // large leaves: a thread per i over the leaf's whole entry list
  for (int local = (int)threadIdx.x; local < L.count; local += (int)blockDim.x) {
    const int i = L.start + local;
    const bool act = g.active[i];
    if (!act) continue;
    const double4 p = act ? g.pos[i] : make_double4(0., 0., 0., 1.);
    const float oag = act ? g.oagn[i] : 0.f;
    T F[4] = {(T)0, (T)0, (T)0, (T)0};
    for (int q = p0; q < p1; q++) {
      const swh_leaf_pair pr = pairs[q];
      if (!pr.allow_mpole || leaves[pr.j].count <= 1) continue;
      const swh_multipole& M = g.mp[pr.j];
      if (!m2p_accept(mac, mac_source(M), (float)p.x, (float)p.y, (float)p.z, (float)p.w, oag))
        continue;
      T f[4];
      m2p_pair<T>(g, i, pr.j, pr.truncated != 0, periodic, dimx, dimy, dimz, r_s_inv, f);
      for (int k = 0; k < 4; k++) F[k] += f[k];
      nm++;
    }
    if (F[0] != (T)0 || F[1] != (T)0 || F[2] != (T)0 || F[3] != (T)0) {
      double4 a = g.acc[i];
      a.x += (double)F[1];
      a.y += (double)F[2];
      a.z += (double)F[3];
      a.w += (double)F[0];
      g.acc[i] = a;
    }
  }
  if (counter) {
    for (int o = 32; o > 0; o >>= 1) nm += __shfl_xor(nm, o);
    if ((threadIdx.x & 63) == 0 && nm) atomicAdd(counter + 1, nm);
  }
}

swh_status launch_pp(swh_gspace* g, const swh_grav_params* G, const MacParams& mac,
                     unsigned long long* ctr, hipEvent_t m2p_start = nullptr);

static GSoA gsoa_of(swh_gspace* g) {
  GSoA s;
  s.pos = g->pos.as<double4>();
  s.hinv = g->hinv.as<double>();
  s.mass = g->mass.as<float>();
  s.active = g->active.as<int8_t>();
  s.acc = g->accel.as<double4>();
  s.oagn = g->oagn.as<float>();
  s.mp = g->mpoles.as<const swh_multipole>();
  return s;
}

}  // namespace swh

using namespace swh;

extern "C" {

swh_status swh_gspace_create(swh_context* ctx, swh_gspace** out) {
  if (!ctx || !out) return SWH_ERR_ARG;
  SWH_HIP(hipSetDevice(ctx->device));
  auto* g = new swh_gspace();
  g->ctx = ctx;
  // The gravity step is a chain of small, dependent launches (the walk's
  // levels, the P2P / M2P / M2L / down passes): its stream takes the highest
  // priority, so a concurrent hydro loop (SWIFT runs both in one step) fills
  // the CUs the chain leaves idle instead of delaying it. SWH_GRAV_STREAM_PRIORITY=0:
  // default priority.
  int least = 0, greatest = 0;
  const char* pe = std::getenv("SWH_GRAV_STREAM_PRIORITY");
  const bool high = !(pe && pe[0] == '0');
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e == hipSuccess)
    e = hipStreamCreateWithPriority(&g->stream, hipStreamNonBlocking, high ? greatest : least);
  if (e != hipSuccess) {
    delete g;
    return SWH_ERR_HIP;
  }
  *out = g;
  return SWH_OK;
}

swh_status swh_gspace_destroy(swh_gspace* g) {
  if (!g) return SWH_OK;
  (void)hipSetDevice(g->ctx->device);
  (void)hipStreamSynchronize(g->stream);
  DevBuf* bufs[] = {&g->aos,      &g->pos,      &g->hinv,    &g->mass,    &g->active,
                    &g->accel,    &g->oagn,     &g->mpoles,  &g->leaves,  &g->pair_off,
                    &g->pairs,    &g->counter,  &g->cell_act, &g->ftens,  &g->m2l_off,
                    &g->m2l_src,  &g->l2l_list, &g->leaf_ids, &g->leaf_of, &g->m2m_list, &g->tree_d, &g->wf0,
                    &g->wf1,      &g->pp_key,  &g->pp_val,  &g->pp_key2,
                    &g->pp_val2,  &g->mm_key,  &g->mm_val,  &g->mm_key2,
                    &g->mm_val2,  &g->wsort_tmp, &g->wrec, &g->wcnt, &g->wbase, &g->owned_d,
                    &g->m2p_bits};
  for (DevBuf* b : bufs) b->release();
  mesh_release(g);
  (void)hipStreamDestroy(g->stream);
  delete g;
  return SWH_OK;
}

// The activity mask needs max_active_bin: it is (re)derived in
// swh_grav_pp_batch from the AoS image, so upload only stages the records.
swh_status swh_gspace_upload(swh_gspace* g, const void* gparts, int64_t count,
                             const swh_gpart_layout* GL, int on_device) {
  if (!g || (count > 0 && !gparts) || count < 0 || count > INT32_MAX / 2 || !GL)
    return SWH_ERR_ARG;
  GLayout L;
  SWH_TRY(make_glayout(GL, &L));
  SWH_HIP(hipSetDevice(g->ctx->device));
  g->layout = L;
  g->n = count;
  if (count == 0) return SWH_OK;
  SWH_TRY(g->aos.reserve((size_t)count * L.stride));
  SWH_TRY(g->pos.reserve((size_t)count * sizeof(double4)));
  SWH_TRY(g->hinv.reserve((size_t)count * sizeof(double)));
  SWH_TRY(g->mass.reserve((size_t)count * sizeof(float)));
  SWH_TRY(g->active.reserve((size_t)count));
  SWH_TRY(g->accel.reserve((size_t)count * sizeof(double4)));
  SWH_TRY(g->oagn.reserve((size_t)count * sizeof(float)));
  g->mpoles_valid = false;
  // nothing accumulated yet: a download before any batch (e.g. after only
  // swh_gspace_pm_mesh) returns the records with their mesh fields alone
  SWH_HIP(hipMemsetAsync(g->active.ptr, 0, (size_t)count, g->stream));
  SWH_HIP(hipMemsetAsync(g->accel.ptr, 0, (size_t)count * sizeof(double4), g->stream));
  SWH_HIP(hipMemcpyAsync(g->aos.ptr, gparts, (size_t)count * L.stride,
                         on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                         g->stream));
  if (!on_device) SWH_HIP(hipStreamSynchronize(g->stream));
  return SWH_OK;
}

swh_status swh_gspace_set_leaves(swh_gspace* g, const swh_leaf* leaves, int32_t nleaves,
                                 const int32_t* pair_offset, const swh_leaf_pair* pairs,
                                 int32_t npairs) {
  if (!g || nleaves < 0 || npairs < 0 || (nleaves > 0 && (!leaves || !pair_offset)) ||
      (npairs > 0 && !pairs))
    return SWH_ERR_ARG;
  int32_t maxc = 0;
  for (int i = 0; i < nleaves; i++) {
    if (leaves[i].start < 0 || leaves[i].count < 0 || leaves[i].start + leaves[i].count > g->n) {
      set_error("leaf %d [%d,+%d) outside the gpart set of %lld", i, leaves[i].start,
                leaves[i].count, (long long)g->n);
      return SWH_ERR_ARG;
    }
  }
  if (nleaves > 0 && (pair_offset[0] != 0 || pair_offset[nleaves] != npairs)) {
    set_error("pair_offset must run 0..npairs");
    return SWH_ERR_ARG;
  }
  for (int q = 0; q < npairs; q++)
    if (pairs[q].j < 0 || pairs[q].j >= nleaves) {
      set_error("pair %d names leaf %d of %d", q, pairs[q].j, nleaves);
      return SWH_ERR_ARG;
    }
  // the largest i-leaf that has sources (sizes the P2P workgroups)
  for (int i = 0; i < nleaves; i++)
    if (pair_offset[i + 1] > pair_offset[i]) maxc = std::max(maxc, leaves[i].count);
  SWH_HIP(hipSetDevice(g->ctx->device));
  SWH_TRY(g->leaves.reserve((size_t)std::max(1, nleaves) * sizeof(swh_leaf)));
  SWH_TRY(g->pair_off.reserve((size_t)(nleaves + 1) * sizeof(int32_t)));
  SWH_TRY(g->pairs.reserve((size_t)std::max(1, npairs) * sizeof(swh_leaf_pair)));
  if (nleaves > 0) {
    SWH_HIP(hipMemcpyAsync(g->leaves.ptr, leaves, nleaves * sizeof(swh_leaf),
                           hipMemcpyHostToDevice, g->stream));
    SWH_HIP(hipMemcpyAsync(g->pair_off.ptr, pair_offset, (nleaves + 1) * sizeof(int32_t),
                           hipMemcpyHostToDevice, g->stream));
  }
  if (npairs > 0)
    SWH_HIP(hipMemcpyAsync(g->pairs.ptr, pairs, npairs * sizeof(swh_leaf_pair),
                           hipMemcpyHostToDevice, g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  g->nleaves = nleaves;
  g->npairs = npairs;
  g->max_leaf = maxc;
  g->mpoles_valid = false;
  g->any_mpole = false;
  for (int q = 0; q < npairs; q++) g->any_mpole = g->any_mpole || pairs[q].allow_mpole;
  return SWH_OK;
}

swh_status swh_gspace_make_multipoles(swh_gspace* g, swh_multipole* out) {
  if (!g) return SWH_ERR_ARG;
  if (g->nleaves == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(g->ctx->device));
  SWH_TRY(g->mpoles.reserve((size_t)g->nleaves * sizeof(swh_multipole)));
  hipLaunchKernelGGL(p2m_kernel, dim3((g->nleaves + kP2MWaves - 1) / kP2MWaves), dim3(64 * kP2MWaves), 0, g->stream, g->layout,
                     g->aos.as<const char>(), g->leaves.as<const swh_leaf>(), nullptr, g->nleaves,
                     g->mpoles.as<swh_multipole>());
  SWH_HIP(hipGetLastError());
  g->mpoles_valid = true;
  if (out) {
    SWH_HIP(hipMemcpyAsync(out, g->mpoles.ptr, (size_t)g->nleaves * sizeof(swh_multipole),
                           hipMemcpyDeviceToHost, g->stream));
    SWH_HIP(hipStreamSynchronize(g->stream));
  }
  return SWH_OK;
}

swh_status swh_grav_pp_batch(swh_gspace* g, const swh_grav_params* G, int64_t* n_int,
                             int64_t* n_m2p) {
  if (!g || !G) return SWH_ERR_ARG;
  if (n_m2p) *n_m2p = 0;
  if (g->n == 0 || g->nleaves == 0) {
    if (n_int) *n_int = 0;
    return SWH_OK;
  }
  if (g->any_mpole && !g->mpoles_valid) {
    set_error("allow_mpole pairs need swh_gspace_make_multipoles first");
    return SWH_ERR_STATE;
  }
  const MacParams mac = mac_params(G);
  const bool want = n_int || n_m2p;
  SWH_HIP(hipSetDevice(g->ctx->device));
  const int block = 256;
  hipLaunchKernelGGL(gunpack_kernel, dim3((int)((g->n + block - 1) / block)), dim3(block), 0,
                     g->stream, g->layout, g->aos.as<const char>(), g->n, gsoa_of(g),
                     G->max_active_bin);
  SWH_HIP(hipGetLastError());
  SWH_TRY(g->counter.reserve(2 * sizeof(unsigned long long)));
  unsigned long long* ctr = want ? g->counter.as<unsigned long long>() : nullptr;
  if (ctr) SWH_HIP(hipMemsetAsync(ctr, 0, 2 * sizeof(unsigned long long), g->stream));
  SWH_TRY(launch_pp(g, G, mac, ctr));
  if (want) {
    unsigned long long h[2] = {0, 0};
    SWH_HIP(hipMemcpyAsync(h, ctr, sizeof(h), hipMemcpyDeviceToHost, g->stream));
    SWH_HIP(hipStreamSynchronize(g->stream));
    if (n_int) *n_int = (int64_t)h[0];
    if (n_m2p) *n_m2p = (int64_t)h[1];
  }
  return SWH_OK;
}

}  // extern "C"

namespace swh {

// The P2P (+ M2P) launches over the gspace's i-leaf CSR lists.
swh_status launch_pp(swh_gspace* g, const swh_grav_params* G, const MacParams& mac,
                     unsigned long long* ctr, hipEvent_t m2p_start) {
  const bool f64 = g->ctx->precision == SWH_PRECISION_F64;
  if (f64) {
    // the multipole-free instance keeps the P2P kernel's register budget;
    // small leaves (a deep tree) take one wave per i-leaf
    const bool small = g->max_leaf <= 64;
    if (small) {
      if (g->any_mpole) SWH_TRY(g->m2p_bits.reserve((size_t)std::max(1, g->npairs) * 8));
      auto k = g->any_mpole ? p2p_batch_kernel<true> : p2p_batch_kernel<false>;
      hipLaunchKernelGGL(k, dim3(g->nleaves), dim3(64), 0, g->stream, gsoa_of(g),
                         g->leaves.as<const swh_leaf>(), g->pair_off.as<const int>(),
                         g->pairs.as<const swh_leaf_pair>(), G->periodic, (double)G->dim[0],
                         (double)G->dim[1], (double)G->dim[2], (double)G->r_s_inv, mac, ctr,
                         g->m2p_bits.as<unsigned long long>());
    } else {
      auto k = g->any_mpole ? p2p_kernel<true, kGravBlock, kIPer>
                            : p2p_kernel<false, kGravBlock, kIPer>;
      hipLaunchKernelGGL(k, dim3(g->nleaves), dim3(kGravBlock), 0, g->stream, gsoa_of(g),
                         g->leaves.as<const swh_leaf>(), g->pair_off.as<const int>(),
                         g->pairs.as<const swh_leaf_pair>(), G->periodic, (double)G->dim[0],
                         (double)G->dim[1], (double)G->dim[2], (double)G->r_s_inv, mac, ctr);
    }
  }
  else
    hipLaunchKernelGGL(p2p_kernel_f32, dim3(g->nleaves), dim3(kGravBlock), 0, g->stream,
                       gsoa_of(g), g->leaves.as<const swh_leaf>(), g->pair_off.as<const int>(),
                       g->pairs.as<const swh_leaf_pair>(), G->periodic, (double)G->dim[0],
                       (double)G->dim[1], (double)G->dim[2], (float)G->r_s_inv, mac, ctr);
  SWH_HIP(hipGetLastError());
  if (m2p_start) SWH_HIP(hipEventRecord(m2p_start, g->stream));
  if (g->any_mpole && f64 && g->max_leaf <= 64) {
    // the batch kernel's MAC results
    hipLaunchKernelGGL(m2p_bits_kernel<double>, dim3(g->nleaves), dim3(64), 0, g->stream,
                       gsoa_of(g), g->leaves.as<const swh_leaf>(), g->pair_off.as<const int>(),
                       g->pairs.as<const swh_leaf_pair>(),
                       g->m2p_bits.as<const unsigned long long>(), G->periodic,
                       (double)G->dim[0], (double)G->dim[1], (double)G->dim[2],
                       (double)G->r_s_inv, ctr);
    SWH_HIP(hipGetLastError());
  } else if (g->any_mpole) {
    const bool small = g->max_leaf <= 64;  // one wave per small leaf
    auto k = f64 ? (small ? m2p_kernel<double, true> : m2p_kernel<double, false>)
                 : (small ? m2p_kernel<float, true> : m2p_kernel<float, false>);
    hipLaunchKernelGGL(k, dim3(g->nleaves), dim3(small ? 64 : kGravBlock), 0, g->stream,
                       gsoa_of(g), g->leaves.as<const swh_leaf>(), g->pair_off.as<const int>(),
                       g->pairs.as<const swh_leaf_pair>(), G->periodic, (double)G->dim[0],
                       (double)G->dim[1], (double)G->dim[2], (double)G->r_s_inv, mac, ctr);
    SWH_HIP(hipGetLastError());
  }
  return SWH_OK;
}

}  // namespace swh

extern "C" {

swh_status swh_gspace_download(swh_gspace* g, void* gparts, const swh_gpart_layout* GL,
                               int on_device) {
  if (!g || (g->n > 0 && !gparts) || !GL) return SWH_ERR_ARG;
  if (g->n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(g->ctx->device));
  const int block = 256;
  hipLaunchKernelGGL(gpack_kernel, dim3((int)((g->n + block - 1) / block)), dim3(block), 0,
                     g->stream, g->layout, g->aos.as<char>(), g->n, gsoa_of(g));
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemcpyAsync(gparts, g->aos.ptr, (size_t)g->n * g->layout.stride,
                         on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                         g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  return SWH_OK;
}

swh_status swh_gspace_sync(swh_gspace* g) {
  if (!g) return SWH_ERR_ARG;
  SWH_HIP(hipStreamSynchronize(g->stream));
  return SWH_OK;
}

swh_status swh_gspace_query(swh_gspace* g) {
  if (!g) return SWH_ERR_ARG;
  const hipError_t e = hipStreamQuery(g->stream);
  if (e == hipErrorNotReady) return SWH_BUSY;
  SWH_HIP(e);
  return SWH_OK;
}

}  // extern "C"

// ===========================================================================
// Tree gravity: the recursive gravity tasks over a cell tree
// (runner_doself_recursive_grav / runner_dopair_recursive_grav,
// src/runner_doiact_grav.c:2208-2431), M2L (runner_dopair_grav_mm*,
// 1881-2095) and the down pass (runner_do_grav_down, 65-164).
//
// The walk is a host-side decision procedure over the cells' multipoles
// (their CoM, r_max, power and softening): it emits P-P entries (i-leaf <-
// source cell, truncation and allow_mpole flags, i.e. the leaf-pair CSR the
// batch P2P/M2P kernels already run) and M-M entries (target <- source,
// symmetric or not). All arithmetic runs on the device: P2M per cell,
// P2P + M2P, M2L (thread per target cell over its CSR of sources), L2L level
// by level from the roots, L2P per leaf.
// ===========================================================================
namespace swh {

__global__ void cell_active_kernel(const swh_leaf* __restrict__ cells,
                                   const int8_t* __restrict__ active, int8_t* __restrict__ out) {
  const swh_leaf c = cells[blockIdx.x];
  int any = 0;
  for (int k = threadIdx.x; k < c.count; k += blockDim.x) any |= active[c.start + k];
  any = __syncthreads_or(any);
  if (threadIdx.x == 0) out[blockIdx.x] = any ? 1 : 0;
}

__device__ __forceinline__ double wrap_box(double d, double L) {
  return d > 0.5 * L ? d - L : (d < -0.5 * L ? d + L : d);
}

// M2L into each target cell's field tensor (at its CoM) from its sources:
// 16 lanes per target, each over every 16th source of the target's list in
// order, the lanes' tensors combined by shuffles (a target has ~0-300
// sources; a thread per target left the chip idle).
constexpr int kM2LLanes = 16;
template <typename T>
__global__ __launch_bounds__(256) void m2l_kernel(const swh_multipole* __restrict__ mp,
                                                  int ncells, const int* __restrict__ off,
                                                  const int2* __restrict__ src, int periodic,
                                                  double dimx, double dimy, double dimz,
                                                  T r_s_inv, double* __restrict__ F) {
  const int gid = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int c = gid / kM2LLanes, s = gid % kM2LLanes;
  const int q0 = c < ncells ? off[c] : 0, q1 = c < ncells ? off[c + 1] : 0;
  if (__ballot(q1 > q0) == 0ull) return;  // wave-uniform
  T Fl[SWH_MPOLE_TERMS];
#pragma unroll
  for (int t = 0; t < SWH_MPOLE_TERMS; t++) Fl[t] = (T)0;
  if (q1 > q0) {
    const double bx = mp[c].CoM[0], by = mp[c].CoM[1], bz = mp[c].CoM[2];
    const float bsoft = mp[c].max_softening;
    for (int q = q0 + s; q < q1; q += kM2LLanes) {
      const int2 e = src[q];
      const swh_multipole& A = mp[e.x];
      double dx = bx - A.CoM[0], dy = by - A.CoM[1], dz = bz - A.CoM[2];
      if (periodic) {
        dx = wrap_box(dx, dimx);
        dy = wrap_box(dy, dimy);
        dz = wrap_box(dz, dimz);
      }
      // gravity_M2L_symmetric: max of both softenings; _nonsym: the source's
      const T eps = (T)(e.y ? fmaxf(A.max_softening, bsoft) : A.max_softening);
      m2l<T>(A.M, (T)dx, (T)dy, (T)dz, eps, periodic != 0, r_s_inv, Fl);
    }
  }
#pragma unroll
  for (int t = 0; t < SWH_MPOLE_TERMS; t++)
    for (int o = kM2LLanes / 2; o > 0; o >>= 1) Fl[t] += __shfl_xor(Fl[t], o);
  if (s == 0 && q1 > q0) {
    double* out = F + (size_t)c * SWH_MPOLE_TERMS;
#pragma unroll
    for (int t = 0; t < SWH_MPOLE_TERMS; t++) out[t] += (double)Fl[t];
  }
}

// One depth of the down pass: F_cell += L2L(F_parent, CoM_cell - CoM_parent).
template <typename T>
__global__ __launch_bounds__(64) void l2l_kernel(const int2* __restrict__ list, int n,
                           const swh_multipole* __restrict__ mp, double* __restrict__ F) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int2 e = list[k];
  const double* Fp = F + (size_t)e.y * SWH_MPOLE_TERMS;
  T P[SWH_MPOLE_TERMS];
  bool any = false;
#pragma unroll
  for (int t = 0; t < SWH_MPOLE_TERMS; t++) {
    P[t] = (T)Fp[t];
    any |= Fp[t] != 0.;
  }
  if (!any) return;  // the parent's tensor received nothing (pot.interacted == 0)
  T X[SWH_MPOLE_TERMS];
  xpowers<T>((T)(mp[e.x].CoM[0] - mp[e.y].CoM[0]), (T)(mp[e.x].CoM[1] - mp[e.y].CoM[1]),
             (T)(mp[e.x].CoM[2] - mp[e.y].CoM[2]), X);
  T Fc[SWH_MPOLE_TERMS];
#pragma unroll
  for (int t = 0; t < SWH_MPOLE_TERMS; t++) Fc[t] = (T)0;
  l2l_k<T, 0>(X, P, Fc);
  double* out = F + (size_t)e.x * SWH_MPOLE_TERMS;
#pragma unroll
  for (int t = 0; t < SWH_MPOLE_TERMS; t++) out[t] += (double)Fc[t];
}

// L2P, one thread per gpart (leaves hold ~10-50 gparts: a wave per leaf
// left most lanes idle at two waves per SIMD): the gpart's leaf tensor and
// CoM come from L2 (every gpart of a leaf reads the same 35 doubles).
template <typename T>
__global__ __launch_bounds__(256) void l2p_part_kernel(int64_t n, const int* __restrict__ leaf_of,
                                                       const swh_multipole* __restrict__ mp,
                                                       const double* __restrict__ F, GSoA g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !g.active[i]) return;
  const int c = leaf_of[i];
  if (c < 0) return;
  const double* Fc = F + (size_t)c * SWH_MPOLE_TERMS;
  const double4 p = g.pos[i];
  T o[4];
  l2p<T>(Fc, (T)(p.x - mp[c].CoM[0]), (T)(p.y - mp[c].CoM[1]), (T)(p.z - mp[c].CoM[2]), o);
  double4 a = g.acc[i];
  a.x += (double)o[1];
  a.y += (double)o[2];
  a.z += (double)o[3];
  a.w += (double)o[0];
  g.acc[i] = a;
}

// The recursive walk (host).
struct TreeWalk {
  const swh_gcell* cells;
  const swh_multipole* mp;
  const int8_t* act;
  const uint8_t* own;  // null: every cell owned (swh_gspace_set_owned_cells)
  const swh_grav_params* G;
  MacParams mac;
  // the tasks' entries in walk order: {i-cell, P-P entry} and {target, {source,
  // symmetric}} (grouped per cell afterwards, stably, so the lists are the
  // serial walk's whatever the threads)
  std::vector<std::pair<int, swh_leaf_pair>> pp;
  std::vector<std::pair<int, int2>> mm;
  int64_t skipped = 0;

  double nearest(double d, int k) const {
    const double L = (double)G->dim[k];
    return d > 0.5 * L ? d - L : (d < -0.5 * L ? d + L : d);
  }
  bool emits(int c) const { return act[c] && (!own || own[c]); }
  // runner_doself_recursive_grav (2386-2431)
  void self(int c) {
    if (!emits(c)) return;
    const swh_gcell& C = cells[c];
    if (C.split) {
      for (int j = 0; j < 8; j++) {
        if (C.progeny[j] < 0) continue;
        self(C.progeny[j]);
        for (int k = j + 1; k < 8; k++)
          if (C.progeny[k] >= 0) pair(C.progeny[j], C.progeny[k]);
      }
    } else {
      // runner_doself_grav_pp (1788-1871): truncated iff periodic && 2 r_max > r_cut_min
      swh_leaf_pair e;
      e.j = c;
      e.truncated = G->periodic && (2. * mp[c].r_max > G->r_cut_min);
      e.allow_mpole = 0;
      pp.emplace_back(c, e);
    }
  }
  // runner_dopair_grav_pp_no_cache (1440-1483): ci's leaves <- all of cj
  void no_cache(int ci, int cj) {
    if (!emits(ci)) return;
    if (cells[ci].count == 0 || cells[cj].count == 0) return;
    if (cells[ci].split) {
      for (int k = 0; k < 8; k++)
        if (cells[ci].progeny[k] >= 0) no_cache(cells[ci].progeny[k], cj);
    } else {
      swh_leaf_pair e;
      e.j = cj;
      e.truncated = G->periodic ? 1 : 0;
      e.allow_mpole = 0;
      pp.emplace_back(ci, e);
    }
  }
  // runner_dopair_grav_mm (2050-2064): symmetric when both are active
  // (an entry only for an owned target; the symmetry from both activities)
  void mmpair(int ci, int cj) {
    const int sym = act[ci] && act[cj] ? 1 : 0;
    if (emits(ci)) mm.emplace_back(ci, make_int2(cj, sym));
    if (emits(cj)) mm.emplace_back(cj, make_int2(ci, sym));
  }
  // runner_dopair_grav_pp(ci, cj, symmetric = 1, allow_mpole = 1) (1202-1425):
  // truncated iff periodic && |CoM_i - CoM_j| + r_max_i + r_max_j > r_cut_min
  void pppair(int ci, int cj) {
    int trunc = 0;
    if (G->periodic) {
      double d2 = 0.;
      for (int k = 0; k < 3; k++) {
        float dxf = (float)mp[cj].CoM[k] - (float)mp[ci].CoM[k];
        const float L = G->dim[k];
        dxf = dxf > 0.5f * L ? dxf - L : (dxf < -0.5f * L ? dxf + L : dxf);
        d2 += (double)dxf * (double)dxf;
      }
      trunc = (std::sqrt(d2) + (double)(float)mp[ci].r_max + (double)(float)mp[cj].r_max) >
              G->r_cut_min;
    }
    if (emits(ci)) pp.emplace_back(ci, swh_leaf_pair{cj, trunc, 1});
    if (emits(cj)) pp.emplace_back(cj, swh_leaf_pair{ci, trunc, 1});
  }
  // runner_dopair_recursive_grav (2208-2374)
  void pair(int ci, int cj) {
    if (!(emits(ci) || emits(cj))) return;
    const swh_multipole& A = mp[ci];
    const swh_multipole& B = mp[cj];
    double dx = A.CoM[0] - B.CoM[0], dy = A.CoM[1] - B.CoM[1], dz = A.CoM[2] - B.CoM[2];
    if (G->periodic) {
      dx = nearest(dx, 0);
      dy = nearest(dy, 1);
      dz = nearest(dz, 2);
    }
    const double r2 = dx * dx + dy * dy + dz * dz;
    const double r_lr_check = std::sqrt(r2) - (A.r_max + B.r_max);
    if (G->periodic && r_lr_check > G->r_cut_max) {
      skipped++;
      return;
    }
    const swh_gcell& Ci = cells[ci];
    const swh_gcell& Cj = cells[cj];
    if (Ci.count <= 1 || Cj.count <= 1) {
      no_cache(ci, cj);
      no_cache(cj, ci);
    } else if (m2l_accept(mac, m2l_side(A), m2l_side(B), (float)r2) &&
               m2l_accept(mac, m2l_side(B), m2l_side(A), (float)r2)) {
      mmpair(ci, cj);
    } else if (!Ci.split && !Cj.split) {
      pppair(ci, cj);
    } else if (A.r_max > B.r_max) {
      if (Ci.split) {
        for (int k = 0; k < 8; k++)
          if (Ci.progeny[k] >= 0) pair(Ci.progeny[k], cj);
      } else {
        for (int k = 0; k < 8; k++)
          if (Cj.progeny[k] >= 0) pair(ci, Cj.progeny[k]);
      }
    } else {
      if (Cj.split) {
        for (int k = 0; k < 8; k++)
          if (Cj.progeny[k] >= 0) pair(ci, Cj.progeny[k]);
      } else {
        for (int k = 0; k < 8; k++)
          if (Ci.progeny[k] >= 0) pair(Ci.progeny[k], cj);
      }
    }
  }
};


// ---------------------------------------------------------------------------
// The recursive walk on the device (level-synchronous): every thread takes one
// task of the frontier -- self(c), pair(ci, cj) or no_cache(ci, cj), the
// decisions of TreeWalk above -- and either emits its P-P / M-M entries or
// pushes its sub-tasks into the next frontier. Entries are keyed
// (cell << 32 | other cell), unique per walk, and sorted by key afterwards, so
// the lists do not depend on the threads' order.
enum { GW_SELF = 0, GW_PAIR = 1, GW_NOCACHE = 2 };

// Per-wave output counts of one level (written by the count pass, scanned
// over the waves, read back by the write pass: no global atomics -- thousands
// of waves adding into one counter serialise on its L2 channel).
struct GWCnt {
  unsigned int next, pp, mm, skip, self, pad[3];
};
struct GWCntSum {
  __host__ __device__ GWCnt operator()(const GWCnt& a, const GWCnt& b) const {
    GWCnt c;
    c.next = a.next + b.next;
    c.pp = a.pp + b.pp;
    c.mm = a.mm + b.mm;
    c.skip = a.skip + b.skip;
    c.self = a.self + b.self;
    c.pad[0] = c.pad[1] = c.pad[2] = 0u;
    return c;
  }
};

struct GWalkOut {
  int4* next;
  GWCnt* wcnt;         // count pass: this level's per-wave counts
  const GWCnt* wbase;  // write pass: their exclusive scan plus the running totals
  unsigned long long* pp_key;
  int* pp_val;  // truncated | allow_mpole << 1
  unsigned long long* mm_key;
  int* mm_val;  // symmetric
  int bits;     // key = cell << bits | other cell
  int narrow;   // 2 bits <= 32: the keys are stored as 32-bit words (a lighter sort)
};

// The walk's view of a cell, one 64-byte line (a task reads two of them, not
// the 200-byte multipoles and 96-byte cells): the CoM and r_max in double,
// the acceptance test's float fields, the gpart count and split / active.
struct __align__(64) GWRec {
  double com[3];
  double r_max;
  float max_soft, min_a, power[3];
  int count;
  int flags;  // 1: split, 2: active, 4: owned
  int pad;
};
static_assert(sizeof(GWRec) == 64, "one cache line per cell");

__global__ void gw_rec_kernel(const swh_gcell* __restrict__ cells,
                              const swh_multipole* __restrict__ mp,
                              const int8_t* __restrict__ act, const uint8_t* __restrict__ own,
                              int n, GWRec* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  GWRec r;
  for (int k = 0; k < 3; k++) r.com[k] = mp[c].CoM[k];
  r.r_max = mp[c].r_max;
  r.max_soft = mp[c].max_softening;
  r.min_a = mp[c].min_old_a_grav_norm;
  for (int k = 0; k < 3; k++) r.power[k] = mp[c].power[k];
  r.count = cells[c].count;
  r.flags = (cells[c].split ? 1 : 0) | (act[c] ? 2 : 0) | ((!own || own[c]) ? 4 : 0);
  r.pad = 0;
  out[c] = r;
}

// m2l_side of a record (M_000 = power[0], gravity_multipole_compute_power)
__device__ __forceinline__ M2LSide rec_side(const GWRec& r) {
  M2LSide s;
  s.rho = (float)r.r_max;
  s.max_soft = r.max_soft;
  s.min_a = r.min_a;
  s.M000 = r.power[0];
  for (int k = 0; k < 3; k++) s.power[k] = r.power[k];
  return s;
}

// What one frontier task does (decided first, written after the wave has
// reserved its slots with one atomic per counter).
enum {
  GA_NONE = 0, GA_SELF_SPLIT, GA_SELF_LEAF, GA_NC_SPLIT, GA_NC_LEAF, GA_SKIP, GA_PAIR_NC,
  GA_MM, GA_PP, GA_SPLIT
};

// Exclusive prefix over the wave of four packed 16-bit counts; *tot gets the
// wave's totals (every lane).
__device__ __forceinline__ unsigned long long wave_excl_scan16x4(unsigned long long v,
                                                                 unsigned long long* tot) {
  const int lane = threadIdx.x & 63;
  unsigned long long s = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long u = __shfl_up(s, o);
    if (lane >= o) s += u;
  }
  *tot = __shfl(s, 63);
  return s - v;
}

template <bool WRITE>
__global__ __launch_bounds__(256) void gwalk_kernel(
    const int4* __restrict__ cur, int n, const swh_gcell* __restrict__ cells,
    const GWRec* __restrict__ rec, MacParams mac, int periodic,
    double dimx, double dimy, double dimz, double r_cut_min, double r_cut_max, GWalkOut o) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  if (__ballot(k < n) == 0ull) return;  // wave-uniform
  int ga = GA_NONE, ci = -1, cj = -1, nn = 0, npp = 0, nmm = 0, ns = 0;
  int trunc = 0, di = 0, dj = 0, ei = 0, ej = 0, split_i = 0;
  if (k < n) {
    const int4 it = cur[k];
    ci = it.x;
    cj = it.y;
    if (it.z == GW_SELF) {  // runner_doself_recursive_grav (2386-2431)
      const GWRec C = rec[ci];
      if ((C.flags & 6) == 6) {  // active and owned
        if (C.flags & 1) {
          int m = 0;
          for (int j = 0; j < 8; j++) m += cells[ci].progeny[j] >= 0 ? 1 : 0;
          ga = GA_SELF_SPLIT;
          nn = m + m * (m - 1) / 2;
          ns = m;
        } else {
          ga = GA_SELF_LEAF;
          trunc = periodic && (2. * C.r_max > r_cut_min);
          npp = 1;
        }
      }
    } else if (it.z == GW_NOCACHE) {  // runner_dopair_grav_pp_no_cache (1440-1483)
      const GWRec Ci = rec[ci];
      if ((Ci.flags & 6) == 6 && Ci.count > 0 && rec[cj].count > 0) {
        if (Ci.flags & 1) {
          for (int j = 0; j < 8; j++) nn += cells[ci].progeny[j] >= 0 ? 1 : 0;
          ga = GA_NC_SPLIT;
        } else {
          ga = GA_NC_LEAF;
          trunc = periodic ? 1 : 0;
          npp = 1;
        }
      }
    } else {  // runner_dopair_recursive_grav (2208-2374)
      const GWRec A = rec[ci];
      const GWRec B = rec[cj];
      di = (A.flags >> 1) & 1;
      dj = (B.flags >> 1) & 1;
      ei = (A.flags & 6) == 6;  // an entry for ci / cj: active and owned
      ej = (B.flags & 6) == 6;
      if (ei || ej) {
        double dx = A.com[0] - B.com[0], dy = A.com[1] - B.com[1], dz = A.com[2] - B.com[2];
        if (periodic) {
          dx = dx > 0.5 * dimx ? dx - dimx : (dx < -0.5 * dimx ? dx + dimx : dx);
          dy = dy > 0.5 * dimy ? dy - dimy : (dy < -0.5 * dimy ? dy + dimy : dy);
          dz = dz > 0.5 * dimz ? dz - dimz : (dz < -0.5 * dimz ? dz + dimz : dz);
        }
        const double r2 = dx * dx + dy * dy + dz * dz;
        const double r_lr_check = sqrt(r2) - (A.r_max + B.r_max);
        const bool si = A.flags & 1, sj = B.flags & 1;
        if (periodic && r_lr_check > r_cut_max) {
          ga = GA_SKIP;
        } else if (A.count <= 1 || B.count <= 1) {
          ga = GA_PAIR_NC;
          nn = 2;
        } else if (m2l_accept(mac, rec_side(A), rec_side(B), (float)r2) &&
                   m2l_accept(mac, rec_side(B), rec_side(A), (float)r2)) {
          // runner_dopair_grav_mm (2050-2064): symmetric when both are active
          ga = GA_MM;
          nmm = ei + ej;
        } else if (!si && !sj) {
          // runner_dopair_grav_pp(ci, cj, 1, 1): truncated iff periodic &&
          // |CoM_i - CoM_j| + r_max_i + r_max_j > r_cut_min (float separations)
          if (periodic) {
            const float L[3] = {(float)dimx, (float)dimy, (float)dimz};
            double d2 = 0.;
            for (int q = 0; q < 3; q++) {
              float dxf = (float)B.com[q] - (float)A.com[q];
              dxf = dxf > 0.5f * L[q] ? dxf - L[q] : (dxf < -0.5f * L[q] ? dxf + L[q] : dxf);
              d2 += (double)dxf * (double)dxf;
            }
            trunc = (sqrt(d2) + (double)(float)A.r_max + (double)(float)B.r_max) > r_cut_min;
          }
          ga = GA_PP;
          npp = ei + ej;
        } else {
          // split the larger cell (or the only split one)
          split_i = A.r_max > B.r_max ? si : !sj;
          const swh_gcell& S = split_i ? cells[ci] : cells[cj];
          for (int j = 0; j < 8; j++) nn += S.progeny[j] >= 0 ? 1 : 0;
          ga = GA_SPLIT;
        }
      }
    }
  }
  const unsigned long long mine = (unsigned long long)nn | ((unsigned long long)npp << 16) |
                                  ((unsigned long long)nmm << 32);
  unsigned long long tot;
  const unsigned long long ex = wave_excl_scan16x4(mine, &tot);
  const int wave = k >> 6;
  if (!WRITE) {
    int sk = ga == GA_SKIP ? 1 : 0, nself = ns;
    for (int d = 32; d > 0; d >>= 1) {
      sk += __shfl_xor(sk, d);
      nself += __shfl_xor(nself, d);
    }
    if (lane == 0) {
      GWCnt c;
      c.next = (unsigned int)(tot & 0xffffull);
      c.pp = (unsigned int)((tot >> 16) & 0xffffull);
      c.mm = (unsigned int)((tot >> 32) & 0xffffull);
      c.skip = (unsigned int)sk;
      c.self = (unsigned int)nself;
      c.pad[0] = c.pad[1] = c.pad[2] = 0u;
      o.wcnt[wave] = c;
    }
    return;
  }
  const GWCnt wb = o.wbase[wave];
  unsigned int q = wb.next + (unsigned int)(ex & 0xffffull);
  unsigned int p = wb.pp + (unsigned int)((ex >> 16) & 0xffffull);
  unsigned int w = wb.mm + (unsigned int)((ex >> 32) & 0xffffull);
  const int bits = o.bits;
  auto pp = [&](int a, int b, int tr, int mpole) {
    const unsigned long long key = ((unsigned long long)(unsigned int)a << bits) | (unsigned int)b;
    if (o.narrow) reinterpret_cast<unsigned int*>(o.pp_key)[p] = (unsigned int)key;
    else o.pp_key[p] = key;
    o.pp_val[p] = tr | (mpole << 1);
    p++;
  };
  auto mm = [&](int t, int s, int sym) {
    const unsigned long long key = ((unsigned long long)(unsigned int)t << bits) | (unsigned int)s;
    if (o.narrow) reinterpret_cast<unsigned int*>(o.mm_key)[w] = (unsigned int)key;
    else o.mm_key[w] = key;
    o.mm_val[w] = sym;
    w++;
  };
  switch (ga) {
    case GA_SELF_SPLIT: {
      const swh_gcell& C = cells[ci];
      int ch[8], m = 0;
      for (int j = 0; j < 8; j++)
        if (C.progeny[j] >= 0) ch[m++] = C.progeny[j];
      for (int j = 0; j < m; j++) {
        o.next[q++] = make_int4(ch[j], -1, GW_SELF, 0);
        for (int l = j + 1; l < m; l++) o.next[q++] = make_int4(ch[j], ch[l], GW_PAIR, 0);
      }
      break;
    }
    case GA_SELF_LEAF: pp(ci, ci, trunc, 0); break;
    case GA_NC_SPLIT: {
      const swh_gcell& Ci = cells[ci];
      for (int j = 0; j < 8; j++)
        if (Ci.progeny[j] >= 0) o.next[q++] = make_int4(Ci.progeny[j], cj, GW_NOCACHE, 0);
      break;
    }
    case GA_NC_LEAF: pp(ci, cj, trunc, 0); break;
    case GA_PAIR_NC:
      o.next[q] = make_int4(ci, cj, GW_NOCACHE, 0);
      o.next[q + 1] = make_int4(cj, ci, GW_NOCACHE, 0);
      break;
    case GA_MM:  // symmetric when both are active, an entry per owned target
      if (ei) mm(ci, cj, di & dj);
      if (ej) mm(cj, ci, di & dj);
      break;
    case GA_PP:
      if (ei) pp(ci, cj, trunc, 1);
      if (ej) pp(cj, ci, trunc, 1);
      break;
    case GA_SPLIT: {
      const swh_gcell& S = split_i ? cells[ci] : cells[cj];
      for (int j = 0; j < 8; j++) {
        if (S.progeny[j] < 0) continue;
        o.next[q++] = split_i ? make_int4(S.progeny[j], cj, GW_PAIR, 0)
                              : make_int4(ci, S.progeny[j], GW_PAIR, 0);
      }
      break;
    }
    default: break;
  }
}

// CSR offsets from keys sorted by (cell << bits | other): off[c] = the first
// entry of cell c (lower bound), c = 0..ncells.
template <typename K>
__global__ void gw_csr_kernel(const K* __restrict__ key, int n, int bits, int ncells,
                              int* __restrict__ off) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > ncells) return;
  // (c = ncells: all keys lie below it; 64-bit so that it cannot wrap)
  const unsigned long long v = (unsigned long long)(unsigned int)c << bits;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((unsigned long long)key[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  off[c] = lo;
}

template <typename K>
__global__ void gw_unpack_pp(const K* __restrict__ key, const int* __restrict__ val, int n,
                             unsigned long long mask, swh_leaf_pair* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  swh_leaf_pair e;
  e.j = (int)((unsigned long long)key[k] & mask);
  e.truncated = val[k] & 1;
  e.allow_mpole = (val[k] >> 1) & 1;
  out[k] = e;
}
template <typename K>
__global__ void gw_unpack_mm(const K* __restrict__ key, const int* __restrict__ val, int n,
                             unsigned long long mask, int2* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  out[k] = make_int2((int)((unsigned long long)key[k] & mask), val[k]);
}

// Grow a device buffer keeping its first `used` bytes.
static swh_status grow_keep(DevBuf& b, size_t need, size_t used, hipStream_t st) {
  if (need <= b.bytes) return SWH_OK;
  DevBuf nb;
  SWH_TRY(nb.reserve(std::max(need, 2 * b.bytes)));
  if (used > 0) SWH_HIP(hipMemcpyAsync(nb.ptr, b.ptr, used, hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipStreamSynchronize(st));
  b.release();
  b.ptr = nb.ptr;
  b.bytes = nb.bytes;
  nb.ptr = nullptr;
  nb.bytes = 0;
  return SWH_OK;
}

static bool walk_debug() {
  static const bool on = std::getenv("SWH_WALK_DEBUG") != nullptr;
  return on;
}

// Sort one entry list by key (only the bits keys use) and build its CSR.
template <typename K>
static swh_status gw_sort_csr(swh_gspace* g, DevBuf& key, DevBuf& val, DevBuf& key2, DevBuf& val2,
                              int n, int bits, int ncells, DevBuf& off, hipStream_t st) {
  SWH_TRY(off.reserve(((size_t)ncells + 1) * sizeof(int32_t)));
  if (n > 0) {
    SWH_TRY(key2.reserve((size_t)n * sizeof(K)));
    SWH_TRY(val2.reserve((size_t)n * 4));
    size_t tb = 0;
    SWH_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key.as<K>(), key2.as<K>(),
                                               val.as<int>(), val2.as<int>(), n, 0, 2 * bits,
                                               st));
    SWH_TRY(g->wsort_tmp.reserve(tb));
    tb = g->wsort_tmp.bytes;
    SWH_HIP(hipcub::DeviceRadixSort::SortPairs(g->wsort_tmp.ptr, tb, key.as<K>(), key2.as<K>(),
                                               val.as<int>(), val2.as<int>(), n, 0, 2 * bits,
                                               st));
  }
  hipLaunchKernelGGL(gw_csr_kernel<K>, dim3((ncells + 1 + 255) / 256), dim3(256), 0, st,
                     key2.as<const K>(), n, bits, ncells, off.as<int>());
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

// The walk on the device; fills g->pair_off / g->pairs (P-P CSR over i-cells)
// and g->m2l_off / g->m2l_src (M-M CSR over targets). Each level reserves the
// next frontier by task type: a split self task fans out to at most 8 + 28
// tasks, a pair or no-cache task to at most 8.
static swh_status device_walk(swh_gspace* g, const swh_grav_params* G, const int32_t* self_cells,
                              int32_t nself, const int32_t* pair_cells, int32_t npair,
                              int64_t* n_pp, int64_t* n_mm, int64_t* n_skip) {
  hipStream_t st = g->stream;
  const int ncells = (int)g->tree.size();
  int bits = 1;
  while ((1ll << bits) < (long long)ncells) bits++;  // <= 31: keys of 2 * bits <= 62 bits
  const unsigned long long mask = (1ull << bits) - 1ull;
  const bool narrow = 2 * bits <= 32;
  // the tasks that can reach an owned cell (all of them without ownership)
  const bool owns = !g->owned.empty();
  auto own = [&](int c) { return !owns || g->owned[c] != 0; };
  std::vector<int4> init;
  init.reserve((size_t)nself + npair + 1);
  int64_t nself_kept = 0;
  for (int k = 0; k < nself; k++)
    if (own(self_cells[k])) init.push_back(make_int4(self_cells[k], -1, GW_SELF, 0));
  nself_kept = (int64_t)init.size();
  for (int k = 0; k < npair; k++)
    if (own(pair_cells[2 * k]) || own(pair_cells[2 * k + 1]))
      init.push_back(make_int4(pair_cells[2 * k], pair_cells[2 * k + 1], GW_PAIR, 0));
  const int64_t ntask = (int64_t)init.size();
  if (init.empty()) init.push_back(make_int4(0, 0, GW_PAIR, 0));
  SWH_TRY(g->wf0.reserve((size_t)std::max<int64_t>(1, ntask) * sizeof(int4)));
  if (ntask > 0)
    SWH_HIP(hipMemcpyAsync(g->wf0.ptr, init.data(), (size_t)ntask * sizeof(int4),
                           hipMemcpyHostToDevice, st));
  const MacParams mac = mac_params(G);
  SWH_TRY(g->wrec.reserve((size_t)std::max(1, ncells) * sizeof(GWRec)));
  hipLaunchKernelGGL(gw_rec_kernel, dim3((ncells + 255) / 256), dim3(256), 0, st,
                     g->tree_d.as<const swh_gcell>(), g->mpoles.as<const swh_multipole>(),
                     g->cell_act.as<const int8_t>(),
                     owns ? g->owned_d.as<const uint8_t>() : nullptr, ncells, g->wrec.as<GWRec>());
  SWH_HIP(hipGetLastError());
  int64_t n_cur = ntask, n_self_cur = nself_kept;
  GWCnt h{};  // running totals: P-P and M-M entries, skipped pairs
  DevBuf* cur = &g->wf0;
  DevBuf* nxt = &g->wf1;
  while (n_cur > 0) {
    const size_t bound = (size_t)n_self_cur * 36 + (size_t)(n_cur - n_self_cur) * 8;
    SWH_TRY(nxt->reserve(std::max<size_t>(1, bound) * sizeof(int4)));
    const size_t pp_need = (size_t)h.pp + 2 * (size_t)n_cur, mm_need = (size_t)h.mm + 2 * (size_t)n_cur;
    SWH_TRY(grow_keep(g->pp_key, pp_need * 8, (size_t)h.pp * 8, st));
    SWH_TRY(grow_keep(g->pp_val, pp_need * 4, (size_t)h.pp * 4, st));
    SWH_TRY(grow_keep(g->mm_key, mm_need * 8, (size_t)h.mm * 8, st));
    SWH_TRY(grow_keep(g->mm_val, mm_need * 4, (size_t)h.mm * 4, st));
    // count pass -> per-wave counts; their exclusive scan from the running
    // totals (slot nw holds the new totals) -> write pass
    const int nw = (int)((n_cur + 63) / 64);
    SWH_TRY(g->wcnt.reserve(((size_t)nw + 1) * sizeof(GWCnt)));
    SWH_TRY(g->wbase.reserve(((size_t)nw + 1) * sizeof(GWCnt)));
    GWCnt* wcnt = g->wcnt.as<GWCnt>();
    GWalkOut o{nxt->as<int4>(), wcnt, g->wbase.as<const GWCnt>(),
               g->pp_key.as<unsigned long long>(), g->pp_val.as<int>(),
               g->mm_key.as<unsigned long long>(), g->mm_val.as<int>(), bits, narrow ? 1 : 0};
    const dim3 grid((unsigned)((n_cur + 255) / 256));
    hipLaunchKernelGGL(gwalk_kernel<false>, grid, dim3(256), 0, st, cur->as<const int4>(),
                       (int)n_cur, g->tree_d.as<const swh_gcell>(), g->wrec.as<const GWRec>(), mac,
                       G->periodic, (double)G->dim[0], (double)G->dim[1], (double)G->dim[2],
                       G->r_cut_min, G->r_cut_max, o);
    SWH_HIP(hipGetLastError());
    GWCnt init = h;
    init.next = 0u;
    init.self = 0u;
    SWH_HIP(hipMemsetAsync(wcnt + nw, 0, sizeof(GWCnt), st));
    size_t tb = 0;
    SWH_HIP(hipcub::DeviceScan::ExclusiveScan(nullptr, tb, wcnt, g->wbase.as<GWCnt>(), GWCntSum(),
                                              init, nw + 1, st));
    SWH_TRY(g->wsort_tmp.reserve(tb));
    tb = g->wsort_tmp.bytes;
    SWH_HIP(hipcub::DeviceScan::ExclusiveScan(g->wsort_tmp.ptr, tb, wcnt, g->wbase.as<GWCnt>(),
                                              GWCntSum(), init, nw + 1, st));
    hipLaunchKernelGGL(gwalk_kernel<true>, grid, dim3(256), 0, st, cur->as<const int4>(),
                       (int)n_cur, g->tree_d.as<const swh_gcell>(), g->wrec.as<const GWRec>(), mac,
                       G->periodic, (double)G->dim[0], (double)G->dim[1], (double)G->dim[2],
                       G->r_cut_min, G->r_cut_max, o);
    SWH_HIP(hipGetLastError());
    SWH_HIP(hipMemcpyAsync(&h, g->wbase.as<GWCnt>() + nw, sizeof(GWCnt), hipMemcpyDeviceToHost, st));
    SWH_HIP(hipStreamSynchronize(st));
    if (walk_debug())
      std::fprintf(stderr, "[swh walk] frontier %lld -> %u (self %u), pp %u, mm %u, skipped %u\n",
                   (long long)n_cur, h.next, h.self, h.pp, h.mm, h.skip);
    n_cur = h.next;
    n_self_cur = h.self;
    std::swap(cur, nxt);
  }
  const int npp = (int)h.pp, nmm = (int)h.mm;
  *n_pp = npp;
  *n_mm = nmm;
  *n_skip = h.skip;
  // 32-bit keys when they fit: half the radix sort's key traffic
  auto sort_csr = narrow ? gw_sort_csr<unsigned int> : gw_sort_csr<unsigned long long>;
  SWH_TRY(sort_csr(g, g->pp_key, g->pp_val, g->pp_key2, g->pp_val2, npp, bits, ncells,
                   g->pair_off, st));
  SWH_TRY(sort_csr(g, g->mm_key, g->mm_val, g->mm_key2, g->mm_val2, nmm, bits, ncells,
                   g->m2l_off, st));
  SWH_TRY(g->pairs.reserve((size_t)std::max(1, npp) * sizeof(swh_leaf_pair)));
  SWH_TRY(g->m2l_src.reserve((size_t)std::max(1, nmm) * sizeof(int2)));
  if (npp > 0) {
    if (narrow)
      hipLaunchKernelGGL(gw_unpack_pp<unsigned int>, dim3((npp + 255) / 256), dim3(256), 0, st,
                         g->pp_key2.as<const unsigned int>(), g->pp_val2.as<const int>(), npp,
                         mask, g->pairs.as<swh_leaf_pair>());
    else
      hipLaunchKernelGGL(gw_unpack_pp<unsigned long long>, dim3((npp + 255) / 256), dim3(256),
                         0, st, g->pp_key2.as<const unsigned long long>(),
                         g->pp_val2.as<const int>(), npp, mask, g->pairs.as<swh_leaf_pair>());
    SWH_HIP(hipGetLastError());
  }
  if (nmm > 0) {
    if (narrow)
      hipLaunchKernelGGL(gw_unpack_mm<unsigned int>, dim3((nmm + 255) / 256), dim3(256), 0, st,
                         g->mm_key2.as<const unsigned int>(), g->mm_val2.as<const int>(), nmm,
                         mask, g->m2l_src.as<int2>());
    else
      hipLaunchKernelGGL(gw_unpack_mm<unsigned long long>, dim3((nmm + 255) / 256), dim3(256),
                         0, st, g->mm_key2.as<const unsigned long long>(),
                         g->mm_val2.as<const int>(), nmm, mask, g->m2l_src.as<int2>());
    SWH_HIP(hipGetLastError());
  }
  g->npairs = npp;
  g->nleaves = ncells;
  g->max_leaf = g->tree_max_leaf;
  g->any_mpole = npp > 0;  // leaf-leaf entries allow M2P (allow_mpole = 1)
  return SWH_OK;
}

}  // namespace swh

extern "C" {

swh_status swh_gspace_set_tree(swh_gspace* g, const swh_gcell* cells, int32_t ncells) {
  if (!g || ncells < 0 || (ncells > 0 && !cells)) return SWH_ERR_ARG;
  g->mpoles_given = false;
  std::vector<int> parent(ncells, -1);
  for (int c = 0; c < ncells; c++) {
    const swh_gcell& C = cells[c];
    if (C.start < 0 || C.count <= 0 || C.start + C.count > g->n) {
      set_error("cell %d [%d,+%d) empty or outside the gpart set of %lld", c, C.start, C.count,
                (long long)g->n);
      return SWH_ERR_ARG;
    }
    if (C.split) {
      // m2m_kernel bounds r_max by the CoM's distance to the farthest
      // corner of [loc, loc + width] (space_split.c:419-433): a split cell
      // needs real geometry, and its progeny must lie inside it
      if (!(C.width[0] > 0. && C.width[1] > 0. && C.width[2] > 0.)) {
        set_error("cell %d is split but its width (%g, %g, %g) is not positive", c, C.width[0],
                  C.width[1], C.width[2]);
        return SWH_ERR_ARG;
      }
      int64_t sum = 0;
      for (int k = 0; k < 8; k++) {
        const int p = C.progeny[k];
        if (p < 0) continue;
        if (p >= ncells || p == c || parent[p] >= 0) {
          set_error("cell %d: bad progeny %d", c, p);
          return SWH_ERR_ARG;
        }
        const swh_gcell& P = cells[p];
        if (P.start < C.start || P.start + P.count > C.start + C.count) {
          set_error("cell %d: progeny %d outside its range", c, p);
          return SWH_ERR_ARG;
        }
        for (int a = 0; a < 3; a++) {
          const double tol = 1e-12 * C.width[a];
          if (P.loc[a] < C.loc[a] - tol || P.loc[a] + P.width[a] > C.loc[a] + C.width[a] + tol) {
            set_error("cell %d: progeny %d box outside the cell's box (axis %d)", c, p, a);
            return SWH_ERR_ARG;
          }
        }
        parent[p] = c;
        sum += P.count;
      }
      if (sum != C.count) {
        set_error("cell %d: progeny hold %lld of its %d gparts", c, (long long)sum, C.count);
        return SWH_ERR_ARG;
      }
    }
  }
  // depth of every cell (roots: no parent), L2L list grouped by depth
  std::vector<int> depth(ncells, -1);
  int maxd = 0;
  for (int c = 0; c < ncells; c++) {
    int d = 0, x = c;
    while (parent[x] >= 0) {
      x = parent[x];
      d++;
      if (d > ncells) {
        set_error("cell tree has a cycle");
        return SWH_ERR_ARG;
      }
    }
    depth[c] = d;
    maxd = std::max(maxd, d);
  }
  std::vector<int2> l2l;
  std::vector<int32_t> doff(1, 0);
  for (int d = 1; d <= maxd; d++) {
    for (int c = 0; c < ncells; c++)
      if (depth[c] == d) l2l.push_back(make_int2(c, parent[c]));
    doff.push_back((int32_t)l2l.size());
  }
  // the upward pass: split cells, deepest first (M2M reads finished progeny)
  std::vector<int> m2m;
  std::vector<int32_t> moff(1, 0);
  for (int d = maxd; d >= 0; d--) {
    for (int c = 0; c < ncells; c++)
      if (depth[c] == d && cells[c].split) m2m.push_back(c);
    moff.push_back((int32_t)m2m.size());
  }
  std::vector<int> leaves;
  std::vector<swh_leaf> ranges(ncells);
  std::vector<int> leaf_of((size_t)g->n, -1);  // gpart -> its leaf cell (L2P)
  for (int c = 0; c < ncells; c++) {
    if (!cells[c].split) {
      leaves.push_back(c);
      for (int k = cells[c].start; k < cells[c].start + cells[c].count; k++) leaf_of[k] = c;
    }
    ranges[c] = swh_leaf{cells[c].start, cells[c].count};
  }
  // the cell table doubles as the P2P kernels' leaf table (pairs set later)
  std::vector<int32_t> off(ncells + 1, 0);
  SWH_TRY(swh_gspace_set_leaves(g, ranges.data(), ncells, off.data(), nullptr, 0));
  SWH_HIP(hipSetDevice(g->ctx->device));
  g->tree.assign(cells, cells + ncells);
  g->tree_parent = parent;
  g->owned.clear();
  SWH_TRY(g->cell_act.reserve((size_t)std::max(1, ncells)));
  SWH_TRY(g->ftens.reserve((size_t)std::max(1, ncells) * SWH_MPOLE_TERMS * sizeof(double)));
  SWH_TRY(g->l2l_list.reserve(std::max<size_t>(1, l2l.size()) * sizeof(int2)));
  SWH_TRY(g->leaf_ids.reserve(std::max<size_t>(1, leaves.size()) * sizeof(int)));
  SWH_TRY(g->leaf_of.reserve(std::max<size_t>(1, leaf_of.size()) * sizeof(int)));
  SWH_TRY(g->m2m_list.reserve(std::max<size_t>(1, m2m.size()) * sizeof(int)));
  if (!m2m.empty())
    SWH_HIP(hipMemcpyAsync(g->m2m_list.ptr, m2m.data(), m2m.size() * sizeof(int),
                           hipMemcpyHostToDevice, g->stream));
  if (!leaf_of.empty())
    SWH_HIP(hipMemcpyAsync(g->leaf_of.ptr, leaf_of.data(), leaf_of.size() * sizeof(int),
                           hipMemcpyHostToDevice, g->stream));
  if (!l2l.empty())
    SWH_HIP(hipMemcpyAsync(g->l2l_list.ptr, l2l.data(), l2l.size() * sizeof(int2),
                           hipMemcpyHostToDevice, g->stream));
  if (!leaves.empty())
    SWH_HIP(hipMemcpyAsync(g->leaf_ids.ptr, leaves.data(), leaves.size() * sizeof(int),
                           hipMemcpyHostToDevice, g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  g->l2l_depth_off = doff;
  g->m2m_depth_off = moff;
  g->nleaf_cells = (int32_t)leaves.size();
  int32_t ml = 0;
  for (int c : leaves) ml = std::max(ml, cells[c].count);
  g->tree_max_leaf = ml;
  SWH_TRY(g->tree_d.reserve((size_t)std::max(1, ncells) * sizeof(swh_gcell)));
  if (ncells > 0) {
    SWH_HIP(hipMemcpyAsync(g->tree_d.ptr, cells, (size_t)ncells * sizeof(swh_gcell),
                           hipMemcpyHostToDevice, g->stream));
    SWH_HIP(hipStreamSynchronize(g->stream));
  }
  return SWH_OK;
}

swh_status swh_gspace_set_owned_cells(swh_gspace* g, const uint8_t* owned, int32_t ncells) {
  if (!g) return SWH_ERR_ARG;
  if (!owned) {
    g->owned.clear();
    return SWH_OK;
  }
  if (ncells != (int32_t)g->tree.size()) {
    set_error("set_owned_cells: %d cells, the tree has %zu (swh_gspace_set_tree first)", ncells,
              g->tree.size());
    return SWH_ERR_ARG;
  }
  for (int c = 0; c < ncells; c++) {
    const int p = g->tree_parent[c];
    if (p >= 0 && (owned[c] != 0) != (owned[p] != 0)) {
      set_error("set_owned_cells: cell %d and its parent %d differ (own whole subtrees)", c, p);
      return SWH_ERR_ARG;
    }
  }
  SWH_HIP(hipSetDevice(g->ctx->device));
  g->owned.assign(owned, owned + ncells);
  for (auto& o : g->owned) o = o ? 1 : 0;
  SWH_TRY(g->owned_d.reserve((size_t)std::max(1, ncells)));
  SWH_HIP(hipMemcpyAsync(g->owned_d.ptr, g->owned.data(), (size_t)ncells, hipMemcpyHostToDevice,
                         g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  return SWH_OK;
}

// The multipoles of the tree's cells: P2M at the leaves, M2M up the tree
// (space_split.c:340-440), unless the caller gave them.
static swh_status tree_multipoles(swh_gspace* g) {
  const int ncells = (int)g->tree.size();
  SWH_TRY(g->mpoles.reserve((size_t)ncells * sizeof(swh_multipole)));
  if (g->mpoles_given) return SWH_OK;
  if (g->nleaf_cells > 0)
    hipLaunchKernelGGL(p2m_kernel, dim3((g->nleaf_cells + kP2MWaves - 1) / kP2MWaves), dim3(64 * kP2MWaves), 0, g->stream,
                       g->layout, g->aos.as<const char>(), g->leaves.as<const swh_leaf>(),
                       g->leaf_ids.as<const int>(), g->nleaf_cells, g->mpoles.as<swh_multipole>());
  for (size_t d = 0; d + 1 < g->m2m_depth_off.size(); d++) {
    const int o0 = g->m2m_depth_off[d], o1 = g->m2m_depth_off[d + 1];
    if (o1 > o0)
      hipLaunchKernelGGL(m2m_kernel, dim3((o1 - o0 + 63) / 64), dim3(64), 0, g->stream,
                         g->m2m_list.as<const int>() + o0, o1 - o0,
                         g->tree_d.as<const swh_gcell>(), g->mpoles.as<swh_multipole>());
  }
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

// The down pass (runner_do_grav_down, runner_doiact_grav.c:65-164): L2L from
// every cell into its progeny, depth by depth, then L2P at the leaves. A cell
// whose tensor received nothing holds zeros, so pushing it changes nothing,
// as the reference's `interacted` test skips it.
static swh_status tree_down(swh_gspace* g) {
  const bool f64 = g->ctx->precision == SWH_PRECISION_F64;
  for (size_t d = 0; d + 1 < g->l2l_depth_off.size(); d++) {
    const int o0 = g->l2l_depth_off[d], o1 = g->l2l_depth_off[d + 1];
    if (o1 <= o0) continue;
    const int2* lst = g->l2l_list.as<const int2>() + o0;
    if (f64)
      hipLaunchKernelGGL((l2l_kernel<double>), dim3((o1 - o0 + 63) / 64), dim3(64), 0,
                         g->stream, lst, o1 - o0, g->mpoles.as<const swh_multipole>(),
                         g->ftens.as<double>());
    else
      hipLaunchKernelGGL((l2l_kernel<float>), dim3((o1 - o0 + 63) / 64), dim3(64), 0,
                         g->stream, lst, o1 - o0, g->mpoles.as<const swh_multipole>(),
                         g->ftens.as<double>());
    SWH_HIP(hipGetLastError());
  }
  if (g->nleaf_cells > 0) {
    const dim3 pg((unsigned)((g->n + 255) / 256));
    if (f64)
      hipLaunchKernelGGL((l2p_part_kernel<double>), pg, dim3(256), 0, g->stream, g->n,
                         g->leaf_of.as<const int>(), g->mpoles.as<const swh_multipole>(),
                         g->ftens.as<const double>(), gsoa_of(g));
    else
      hipLaunchKernelGGL((l2p_part_kernel<float>), pg, dim3(256), 0, g->stream, g->n,
                         g->leaf_of.as<const int>(), g->mpoles.as<const swh_multipole>(),
                         g->ftens.as<const double>(), gsoa_of(g));
    SWH_HIP(hipGetLastError());
  }
  return SWH_OK;
}

swh_status swh_grav_tree(swh_gspace* g, const swh_grav_params* G, const int32_t* self_cells,
                         int32_t nself, const int32_t* pair_cells, int32_t npair,
                         swh_grav_tree_stats* stats) {
  return swh_grav_tree_tasks(g, G, self_cells, nself, pair_cells, npair, 0, stats);
}

swh_status swh_grav_tree_tasks(swh_gspace* g, const swh_grav_params* G,
                               const int32_t* self_cells, int32_t nself,
                               const int32_t* pair_cells, int32_t npair, int32_t flags,
                               swh_grav_tree_stats* stats) {
  if (!g || !G || nself < 0 || npair < 0 || (nself > 0 && !self_cells) ||
      (npair > 0 && !pair_cells))
    return SWH_ERR_ARG;
  if (stats) *stats = swh_grav_tree_stats{0, 0, 0, 0, 0};
  const int ncells = (int)g->tree.size();
  if (g->n == 0 || ncells == 0) {
    set_error("swh_gspace_set_tree must precede swh_grav_tree");
    return ncells == 0 ? SWH_ERR_STATE : SWH_OK;
  }
  for (int k = 0; k < nself; k++)
    if (self_cells[k] < 0 || self_cells[k] >= ncells) return SWH_ERR_ARG;
  for (int k = 0; k < 2 * npair; k++)
    if (pair_cells[k] < 0 || pair_cells[k] >= ncells) return SWH_ERR_ARG;
  SWH_HIP(hipSetDevice(g->ctx->device));
  const int block = 256;
  // activity, accumulators
  hipLaunchKernelGGL(gunpack_kernel, dim3((int)((g->n + block - 1) / block)), dim3(block), 0,
                     g->stream, g->layout, g->aos.as<const char>(), g->n, gsoa_of(g),
                     G->max_active_bin);
  SWH_HIP(hipGetLastError());
  // multipoles: P2M at the leaves, M2M up the tree (space_split.c:340-440)
  // the phase events, destroyed on every exit path (SWH_TRY / SWH_HIP return early)
  struct Events {
    hipEvent_t e[6] = {};
    ~Events() {
      for (auto& x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } evs;
  hipEvent_t* ev = evs.e;
  if (stats) {
    for (int k = 0; k < 6; k++) SWH_HIP(hipEventCreate(&ev[k]));
    SWH_HIP(hipEventRecord(ev[0], g->stream));
  }
  SWH_TRY(tree_multipoles(g));
  if (stats) SWH_HIP(hipEventRecord(ev[1], g->stream));
  hipLaunchKernelGGL(cell_active_kernel, dim3(ncells), dim3(256), 0, g->stream,
                     g->leaves.as<const swh_leaf>(), g->active.as<const int8_t>(),
                     g->cell_act.as<int8_t>());
  SWH_HIP(hipGetLastError());
  int64_t npp = 0, nmm = 0, skipped = 0;
  if (!std::getenv("SWH_HOST_WALK")) {
    // the walk on the device (the default)
    SWH_TRY(device_walk(g, G, self_cells, nself, pair_cells, npair, &npp, &nmm, &skipped));
  } else {
    std::vector<swh_multipole> mp(ncells);
    std::vector<int8_t> act(ncells);
    SWH_HIP(hipMemcpyAsync(mp.data(), g->mpoles.ptr, ncells * sizeof(swh_multipole),
                           hipMemcpyDeviceToHost, g->stream));
    SWH_HIP(hipMemcpyAsync(act.data(), g->cell_act.ptr, ncells, hipMemcpyDeviceToHost, g->stream));
    SWH_HIP(hipStreamSynchronize(g->stream));
    // the walk: the self and pair tasks in chunks of consecutive tasks spread
    // over host threads (the recursive tasks are independent, as SWIFT's runners
    // execute them); each chunk keeps its entries, and the chunks are joined in
    // task order, so the lists equal a serial walk's
    const int64_t ntask = (int64_t)nself + npair;
    constexpr int64_t kChunk = 64;
    const int64_t nchunk = (ntask + kChunk - 1) / kChunk;
    std::vector<TreeWalk> part((size_t)nchunk);
    const MacParams mac = mac_params(G);
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
      for (int64_t ch = next++; ch < nchunk; ch = next++) {
        TreeWalk& w = part[(size_t)ch];
        w.cells = g->tree.data();
        w.mp = mp.data();
        w.act = act.data();
        w.own = g->owned.empty() ? nullptr : g->owned.data();
        w.G = G;
        w.mac = mac;
        const int64_t t1 = std::min(ntask, (ch + 1) * kChunk);
        for (int64_t t = ch * kChunk; t < t1; t++) {
          if (t < nself) w.self(self_cells[t]);
          else w.pair(pair_cells[2 * (t - nself)], pair_cells[2 * (t - nself) + 1]);
        }
      }
    };
    int nthr = (int)std::min<int64_t>(nchunk, 16);  // the host share of one GPU
    if (const char* e = std::getenv("SWH_HOST_THREADS")) nthr = std::max(1, std::atoi(e));
    nthr = (int)std::max<int64_t>(1, std::min<int64_t>(nthr, nchunk));
    {
      std::vector<std::thread> pool;
      for (int k = 1; k < nthr; k++) pool.emplace_back(worker);
      worker();
      for (auto& th : pool) th.join();
    }
    // P-P lists (CSR over i-cells) and M-M lists (CSR over targets): stable
    // counting sort of the chunks' entries by cell
    std::vector<int32_t> poff(ncells + 1, 0), moff(ncells + 1, 0);
    for (const TreeWalk& w : part) {
      for (const auto& e : w.pp) poff[e.first + 1]++;
      for (const auto& e : w.mm) moff[e.first + 1]++;
      skipped += w.skipped;
    }
    for (int c = 0; c < ncells; c++) {
      poff[c + 1] += poff[c];
      moff[c + 1] += moff[c];
    }
    std::vector<swh_leaf_pair> pairs((size_t)poff[ncells]);
    std::vector<int2> msrc((size_t)moff[ncells]);
    {
      std::vector<int32_t> pcur(poff.begin(), poff.end() - 1), mcur(moff.begin(), moff.end() - 1);
      for (const TreeWalk& w : part) {
        for (const auto& e : w.pp) pairs[(size_t)pcur[e.first]++] = e.second;
        for (const auto& e : w.mm) msrc[(size_t)mcur[e.first]++] = e.second;
      }
    }
    part.clear();
    std::vector<swh_leaf> ranges(ncells);
    for (int c = 0; c < ncells; c++) ranges[c] = swh_leaf{g->tree[c].start, g->tree[c].count};
    SWH_TRY(swh_gspace_set_leaves(g, ranges.data(), ncells, poff.data(), pairs.data(),
                                  (int32_t)pairs.size()));
    npp = (int64_t)pairs.size();
    nmm = (int64_t)msrc.size();
    if (!msrc.empty()) {
      SWH_TRY(g->m2l_off.reserve((size_t)(ncells + 1) * sizeof(int32_t)));
      SWH_TRY(g->m2l_src.reserve(msrc.size() * sizeof(int2)));
      SWH_HIP(hipMemcpyAsync(g->m2l_off.ptr, moff.data(), (ncells + 1) * sizeof(int32_t),
                             hipMemcpyHostToDevice, g->stream));
      SWH_HIP(hipMemcpyAsync(g->m2l_src.ptr, msrc.data(), msrc.size() * sizeof(int2),
                             hipMemcpyHostToDevice, g->stream));
      SWH_HIP(hipStreamSynchronize(g->stream));  // the host vectors go out of scope
    }
  }

  g->mpoles_valid = true;  // the same cell table: the multipoles stay
  if (stats) SWH_HIP(hipEventRecord(ev[2], g->stream));
  // P2P + M2P
  SWH_TRY(g->counter.reserve(3 * sizeof(unsigned long long)));
  unsigned long long* ctr = g->counter.as<unsigned long long>();
  SWH_HIP(hipMemsetAsync(ctr, 0, 3 * sizeof(unsigned long long), g->stream));
  if (npp > 0) SWH_TRY(launch_pp(g, G, mac_params(G), ctr, stats ? ev[3] : nullptr));
  if (stats) SWH_HIP(hipEventRecord(ev[4], g->stream));
  // M2L
  const bool f64 = g->ctx->precision == SWH_PRECISION_F64;
  SWH_HIP(hipMemsetAsync(g->ftens.ptr, 0, (size_t)ncells * SWH_MPOLE_TERMS * sizeof(double),
                         g->stream));
  if (nmm > 0) {
    const dim3 mg((unsigned)(((int64_t)ncells * kM2LLanes + 255) / 256));
    if (f64)
      hipLaunchKernelGGL((m2l_kernel<double>), mg, dim3(256), 0, g->stream,
                         g->mpoles.as<const swh_multipole>(), ncells, g->m2l_off.as<const int>(),
                         g->m2l_src.as<const int2>(), G->periodic, (double)G->dim[0],
                         (double)G->dim[1], (double)G->dim[2], (double)G->r_s_inv,
                         g->ftens.as<double>());
    else
      hipLaunchKernelGGL((m2l_kernel<float>), mg, dim3(256), 0, g->stream,
                         g->mpoles.as<const swh_multipole>(), ncells, g->m2l_off.as<const int>(),
                         g->m2l_src.as<const int2>(), G->periodic, (double)G->dim[0],
                         (double)G->dim[1], (double)G->dim[2], (float)G->r_s_inv,
                         g->ftens.as<double>());
    SWH_HIP(hipGetLastError());
    // down pass: L2L depth by depth, then L2P at the leaves (SWH_TREE_NO_DOWN:
    // the caller runs it later, swh_gspace_grav_down, as SWIFT's grav_down task)
    if (!(flags & SWH_TREE_NO_DOWN)) SWH_TRY(tree_down(g));
  }
  if (stats) SWH_HIP(hipEventRecord(ev[5], g->stream));
  // stats: the P2P pairs of truncated entries (a counting pass after the
  // step, outside its timed phases)
  if (stats && npp > 0) {
    SWH_HIP(hipMemsetAsync(ctr + 2, 0, sizeof(unsigned long long), g->stream));
    const bool small = f64 && g->max_leaf <= 64;  // (the batch kernel's mbits are valid)
    hipLaunchKernelGGL(pp_trunc_count_kernel, dim3(g->nleaves), dim3(64), 0, g->stream,
                       gsoa_of(g), g->leaves.as<const swh_leaf>(), g->pair_off.as<const int>(),
                       g->pairs.as<const swh_leaf_pair>(), mac_params(G), g->any_mpole ? 1 : 0,
                       small && g->any_mpole ? g->m2p_bits.as<const unsigned long long>() : nullptr,
                       ctr + 2);
    SWH_HIP(hipGetLastError());
  }
  unsigned long long h[3] = {0, 0, 0};
  SWH_HIP(hipMemcpyAsync(h, ctr, sizeof(h), hipMemcpyDeviceToHost, g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  if (stats) {
    stats->n_pp = (int64_t)h[0];
    stats->n_m2p = (int64_t)h[1];
    stats->n_pp_truncated = (int64_t)h[2];
    stats->n_m2l = nmm;
    stats->n_pp_tasks = npp;
    stats->n_skipped = skipped;
    float* ms[5] = {&stats->ms_multipoles, &stats->ms_walk, &stats->ms_p2p, &stats->ms_m2p,
                    &stats->ms_down};
    for (int k = 0; k < 5; k++) {
      *ms[k] = 0.f;
      if (k == 3 && npp == 0) continue;  // no M2P launch: ev[3] never recorded
      hipEvent_t a = ev[k], b = ev[k + 1];
      if (k == 2 && npp > 0) b = ev[3];  // P2P ends where M2P starts
      if (k == 2 && npp == 0) b = ev[4];
      (void)hipEventElapsedTime(ms[k], a, b);
    }
  }
  return SWH_OK;
}

swh_status swh_gspace_multipoles(swh_gspace* g, swh_multipole* out) {
  if (!g || !out) return SWH_ERR_ARG;
  const size_t n = g->tree.size();
  if (n == 0) return SWH_OK;
  if (!g->mpoles_valid && !g->mpoles_given) {
    set_error("swh_gspace_multipoles: no tree multipoles yet (run swh_grav_tree)");
    return SWH_ERR_STATE;
  }
  SWH_HIP(hipSetDevice(g->ctx->device));
  SWH_HIP(hipMemcpyAsync(out, g->mpoles.ptr, n * sizeof(swh_multipole), hipMemcpyDeviceToHost,
                         g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  return SWH_OK;
}

swh_status swh_gspace_set_multipoles(swh_gspace* g, const swh_multipole* in) {
  if (!g || !in) return SWH_ERR_ARG;
  const size_t n = g->tree.size();
  if (n == 0) {
    set_error("swh_gspace_set_tree must precede swh_gspace_set_multipoles");
    return SWH_ERR_STATE;
  }
  SWH_HIP(hipSetDevice(g->ctx->device));
  SWH_TRY(g->mpoles.reserve(n * sizeof(swh_multipole)));
  SWH_HIP(hipMemcpyAsync(g->mpoles.ptr, in, n * sizeof(swh_multipole), hipMemcpyHostToDevice,
                         g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  g->mpoles_given = true;
  return SWH_OK;
}

swh_status swh_gspace_grav_down(swh_gspace* g, const swh_grav_params* G, const float* fields) {
  if (!g || !G || !fields) return SWH_ERR_ARG;
  const int ncells = (int)g->tree.size();
  if (g->n == 0 || ncells == 0) {
    set_error("swh_gspace_set_tree must precede swh_gspace_grav_down");
    return ncells == 0 ? SWH_ERR_STATE : SWH_OK;
  }
  SWH_HIP(hipSetDevice(g->ctx->device));
  // activity and the accumulators (swh_gspace_download adds them)
  hipLaunchKernelGGL(gunpack_kernel, dim3((int)((g->n + 255) / 256)), dim3(256), 0, g->stream,
                     g->layout, g->aos.as<const char>(), g->n, gsoa_of(g), G->max_active_bin);
  SWH_HIP(hipGetLastError());
  SWH_TRY(tree_multipoles(g));
  const size_t nt = (size_t)ncells * SWH_MPOLE_TERMS;
  std::vector<double> f(nt);
  for (size_t k = 0; k < nt; k++) f[k] = (double)fields[k];
  SWH_TRY(g->ftens.reserve(nt * sizeof(double)));
  SWH_HIP(hipMemcpyAsync(g->ftens.ptr, f.data(), nt * sizeof(double), hipMemcpyHostToDevice,
                         g->stream));
  SWH_TRY(tree_down(g));
  SWH_HIP(hipStreamSynchronize(g->stream));  // f goes out of scope
  return SWH_OK;
}

// M-M interactions of explicit (target <- source) pairs of the caller's
// multipoles: SWIFT's M-M tasks outside the recursive walk,
// runner_dopair_grav_mm_progenies (runner_doiact_grav.c:2067-2093, the
// well-separated progeny pairs flagged at the rebuild) and
// runner_do_grav_long_range (2441-2530, a cell against every far top-level
// cell). pairs[3k..3k+2] = {target, source, symmetric}: symmetric selects
// gravity_M2L_symmetric's softening (the larger of the two), else
// gravity_M2L_nonsym's (the source's); a symmetric M-M pair is two entries.
// The tree's m2l_kernel over a CSR by target (targets sum their sources in
// the given order); fields[35 t ..] = target t's sums, zero for the others.
swh_status swh_grav_m2l_pairs(swh_context* ctx, const swh_grav_params* G, const swh_multipole* mp,
                              int32_t nmp, const int32_t* pairs, int32_t npairs, float* fields) {
  if (!ctx || !G || (nmp > 0 && (!mp || !fields)) || (npairs > 0 && !pairs) || nmp < 0 ||
      npairs < 0)
    return SWH_ERR_ARG;
  if (nmp == 0) return SWH_OK;
  std::vector<int> off((size_t)nmp + 1, 0);
  for (int32_t k = 0; k < npairs; k++) {
    const int t = pairs[3 * k], so = pairs[3 * k + 1];
    if (t < 0 || t >= nmp || so < 0 || so >= nmp || t == so) {
      set_error("swh_grav_m2l_pairs: pair %d = (%d, %d) out of range or self", (int)k, t, so);
      return SWH_ERR_ARG;
    }
    off[(size_t)t + 1]++;
  }
  for (int32_t c = 0; c < nmp; c++) off[(size_t)c + 1] += off[(size_t)c];
  std::vector<int2> src((size_t)std::max(1, npairs));
  {
    std::vector<int> fill(off.begin(), off.end() - 1);
    for (int32_t k = 0; k < npairs; k++)
      src[(size_t)fill[(size_t)pairs[3 * k]]++] =
          make_int2(pairs[3 * k + 1], pairs[3 * k + 2] ? 1 : 0);
  }
  TaskWorker* w = ctx->lease();
  if (!w) return SWH_ERR_HIP;
  struct Unlease {
    swh_context* c;
    TaskWorker* w;
    ~Unlease() { c->unlease(w); }
  } unl{ctx, w};
  SWH_HIP(hipSetDevice(ctx->device));
  const size_t bm = (size_t)nmp * sizeof(swh_multipole);
  const size_t bo = off.size() * sizeof(int), bs = src.size() * sizeof(int2);
  const size_t bf = (size_t)nmp * SWH_MPOLE_TERMS * sizeof(double);
  SWH_TRY(w->dparts.reserve(bm));
  SWH_TRY(w->dind.reserve(bo));
  SWH_TRY(w->dself.reserve(bs));
  SWH_TRY(w->dparts2.reserve(bf));
  SWH_TRY(w->hstage.reserve(bf));
  SWH_HIP(hipMemcpyAsync(w->dparts.ptr, mp, bm, hipMemcpyHostToDevice, w->stream));
  SWH_HIP(hipMemcpyAsync(w->dind.ptr, off.data(), bo, hipMemcpyHostToDevice, w->stream));
  SWH_HIP(hipMemcpyAsync(w->dself.ptr, src.data(), bs, hipMemcpyHostToDevice, w->stream));
  SWH_HIP(hipMemsetAsync(w->dparts2.ptr, 0, bf, w->stream));
  if (npairs > 0) {
    const dim3 mg((unsigned)(((int64_t)nmp * kM2LLanes + 255) / 256));
    if (ctx->precision == SWH_PRECISION_F64)
      hipLaunchKernelGGL((m2l_kernel<double>), mg, dim3(256), 0, w->stream,
                         w->dparts.as<const swh_multipole>(), (int)nmp, w->dind.as<const int>(),
                         w->dself.as<const int2>(), G->periodic, (double)G->dim[0],
                         (double)G->dim[1], (double)G->dim[2], (double)G->r_s_inv,
                         w->dparts2.as<double>());
    else
      hipLaunchKernelGGL((m2l_kernel<float>), mg, dim3(256), 0, w->stream,
                         w->dparts.as<const swh_multipole>(), (int)nmp, w->dind.as<const int>(),
                         w->dself.as<const int2>(), G->periodic, (double)G->dim[0],
                         (double)G->dim[1], (double)G->dim[2], (float)G->r_s_inv,
                         w->dparts2.as<double>());
    SWH_HIP(hipGetLastError());
  }
  SWH_HIP(hipMemcpyAsync(w->hstage.ptr, w->dparts2.ptr, bf, hipMemcpyDeviceToHost, w->stream));
  SWH_HIP(hipStreamSynchronize(w->stream));
  const double* h = static_cast<const double*>(w->hstage.ptr);
  for (size_t k = 0; k < (size_t)nmp * SWH_MPOLE_TERMS; k++) fields[k] = (float)h[k];
  return SWH_OK;
}

// gravity_M2L_accept_symmetric (multipole_accept.h:78-176, 190-205) on the
// caller's multipoles at squared CoM distance r2: the tree walk's own MAC
// (m2l_accept, in the reference's float arithmetic). For the rebuild-time
// decisions of cell_can_use_pair_mm (cell.c:1420-1460, use_rebuild_data)
// the caller passes CoM_rebuild / r_max_rebuild.
int swh_grav_m2l_accept(const swh_grav_params* G, const swh_multipole* A, const swh_multipole* B,
                        double r2) {
  if (!G || !A || !B) return 0;
  const MacParams mac = mac_params(G);
  return (m2l_accept(mac, m2l_side(*A), m2l_side(*B), (float)r2) &&
          m2l_accept(mac, m2l_side(*B), m2l_side(*A), (float)r2))
             ? 1
             : 0;
}

swh_status swh_gspace_field_tensors(swh_gspace* g, float* out) {
  if (!g || !out) return SWH_ERR_ARG;
  const size_t n = g->tree.size() * SWH_MPOLE_TERMS;
  if (n == 0) return SWH_OK;
  std::vector<double> h(n);
  SWH_HIP(hipSetDevice(g->ctx->device));
  SWH_HIP(hipMemcpyAsync(h.data(), g->ftens.ptr, n * sizeof(double), hipMemcpyDeviceToHost,
                         g->stream));
  SWH_HIP(hipStreamSynchronize(g->stream));
  for (size_t k = 0; k < n; k++) out[k] = (float)h[k];
  return SWH_OK;
}

}  // extern "C"
