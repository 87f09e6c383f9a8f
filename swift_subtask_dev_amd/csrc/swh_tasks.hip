// swh_tasks.hip — per-task (drop-in) entry points of libswifthip.
//
// One call = one SWIFT task on the caller's host struct part / gpart records.
// The cell records are staged into a per-thread device buffer (AoS, as laid
// out by the caller), one kernel evaluates every interaction of the task in
// gather form (each active i sums over its in-range j; identical per-pair
// arithmetic to the symmetric iacts, src/hydro/SPHENIX/hydro_iact.h and
// tests/testSymmetry.c), and the updated records are copied back before
// return (the task contract: results visible to the next task).
//
//   swh_doself_density / swh_dopair_density   DOSELF1 / DOPAIR1 (density)
//   swh_doself_gradient / swh_dopair_gradient DOSELF1 / DOPAIR1 (gradient)
//   swh_doself_force / swh_dopair_force       DOSELF2 / DOPAIR2 (+ timebin)
//   swh_do{self,pair}_subset_density          DOSELF_SUBSET / DOPAIR_SUBSET
//   swh_grav_self_pp / swh_grav_pair_pp       runner_doself/dopair_grav_pp (P2P)
#include "swh_internal.h"
#include "swh_mpole.h"
#include "swh_physics.h"

namespace swh {

enum { LOOP_DENSITY = 0, LOOP_GRADIENT = 1, LOOP_FORCE = 2 };

__device__ __forceinline__ float ldf(const char* r, int off) {
  return *reinterpret_cast<const float*>(r + off);
}
__device__ __forceinline__ void stf(char* r, int off, float v) {
  *reinterpret_cast<float*>(r + off) = v;
}
__device__ __forceinline__ double ldd(const char* r, int off) {
  return *reinterpret_cast<const double*>(r + off);
}
__device__ __forceinline__ int ldb(const char* r, int off) {
  return (int)*reinterpret_cast<const int8_t*>(r + off);
}

template <typename T>
__device__ __forceinline__ void load_force_in(const char* r, const Layout& L, ForceIn<T>& F) {
  F.m = ldf(r, L.mass);
  F.h = ldf(r, L.h);
  F.rho = ldf(r, L.rho);
  F.P = ldf(r, L.pressure);
  F.c = ldf(r, L.soundspeed);
  F.f = ldf(r, L.f);
  F.balsara = ldf(r, L.balsara);
  F.alpha_visc = ldf(r, L.visc_alpha);
  F.alpha_diff = ldf(r, L.diff_alpha);
  F.u = ldf(r, L.u);
  F.vx = ldf(r, L.v);
  F.vy = ldf(r, L.v + 4);
  F.vz = ldf(r, L.v + 8);
}

// Gather of one i-record over a j-set (records jrec[0..nj) displaced by jsh).
// skip = index in the j-set that is i itself (-1: none).
template <int LOOP, typename T>
__device__ void gather_task(const Layout L, char* irec, const char* jrec, int nj,
                            double shx, double shy, double shz, int skip,
                            T a2_Hubble) {
  const double xi = ldd(irec, L.x), yi = ldd(irec, L.x + 8), zi = ldd(irec, L.x + 16);
  const T hi = ldf(irec, L.h);
  const T hig2 = hi * hi * (T)kGamma2;
  const T hi_inv = (T)1 / hi;
  const T vix = ldf(irec, L.v), viy = ldf(irec, L.v + 4), viz = ldf(irec, L.v + 8);
  DensityAcc<T> D;
  D.zero();
  GradientAcc<T> G;
  ForceIn<T> I;
  ForceAcc<T> F;
  if (LOOP == LOOP_GRADIENT) {
    G.v_sig = ldf(irec, L.v_sig);
    G.laplace_u = 0;
    G.alpha_visc_max_ngb = ldf(irec, L.avmn);
  }
  if (LOOP == LOOP_FORCE) {
    load_force_in(irec, L, I);
    force_prep_i(I);
    F.ax = F.ay = F.az = F.u_dt = F.h_dt = (T)0;
    F.min_ngb_time_bin = ldb(irec, L.min_tb);
  }
  const T ci_ = (LOOP == LOOP_GRADIENT) ? (T)ldf(irec, L.soundspeed) : (T)0;
  const T ui_ = (LOOP == LOOP_GRADIENT) ? (T)ldf(irec, L.u) : (T)0;
  const T hi_inv2 = hi_inv * hi_inv;
  const T hid_inv = hi_inv2 * hi_inv2;
  for (int j = 0; j < nj; j++) {
    if (j == skip) continue;
    const char* jr = jrec + (size_t)j * L.stride;
    const int tbj = ldb(jr, L.time_bin);
    if (tbj == kTimeBinInhibited) continue;
    const T dx = (T)(xi - (ldd(jr, L.x) + shx));
    const T dy = (T)(yi - (ldd(jr, L.x + 8) + shy));
    const T dz = (T)(zi - (ldd(jr, L.x + 16) + shz));
    const T r2 = dx * dx + dy * dy + dz * dz;
    if (LOOP == LOOP_FORCE) {
      const T hj = ldf(jr, L.h);
      const T hjg2 = hj * hj * (T)kGamma2;
      if (r2 < hig2 || r2 < hjg2) {
        ForceIn<T> J;
        load_force_in(jr, L, J);
        iact_nonsym_force<T>(r2, dx, dy, dz, I, hid_inv, hi_inv, J, a2_Hubble, F);
        if (tbj > 0 && tbj < F.min_ngb_time_bin) F.min_ngb_time_bin = tbj;
      }
    } else if (r2 < hig2) {
      const T mj = ldf(jr, L.mass);
      const T vjx = ldf(jr, L.v), vjy = ldf(jr, L.v + 4), vjz = ldf(jr, L.v + 8);
      if (LOOP == LOOP_DENSITY) {
        iact_nonsym_density<T>(r2, dx, dy, dz, hi_inv, vix, viy, viz, mj, vjx, vjy, vjz, D);
      } else {
        iact_nonsym_gradient<T>(r2, dx, dy, dz, hi, vix, viy, viz, ui_, ci_, mj, vjx, vjy,
                                vjz, (T)ldf(jr, L.u), (T)ldf(jr, L.rho),
                                (T)ldf(jr, L.soundspeed), (T)ldf(jr, L.visc_alpha),
                                a2_Hubble, G);
      }
    }
  }
  if (LOOP == LOOP_DENSITY) {
    stf(irec, L.rho, (float)((T)ldf(irec, L.rho) + D.rho));
    stf(irec, L.rho_dh, (float)((T)ldf(irec, L.rho_dh) + D.rho_dh));
    stf(irec, L.wcount, (float)((T)ldf(irec, L.wcount) + D.wcount));
    stf(irec, L.wcount_dh, (float)((T)ldf(irec, L.wcount_dh) + D.wcount_dh));
    stf(irec, L.div_v, (float)((T)ldf(irec, L.div_v) + D.div_v));
    stf(irec, L.rot_v, (float)((T)ldf(irec, L.rot_v) + D.rot_x));
    stf(irec, L.rot_v + 4, (float)((T)ldf(irec, L.rot_v + 4) + D.rot_y));
    stf(irec, L.rot_v + 8, (float)((T)ldf(irec, L.rot_v + 8) + D.rot_z));
  } else if (LOOP == LOOP_GRADIENT) {
    stf(irec, L.v_sig, (float)G.v_sig);
    stf(irec, L.laplace_u, (float)((T)ldf(irec, L.laplace_u) + G.laplace_u));
    stf(irec, L.avmn, (float)G.alpha_visc_max_ngb);
  } else {
    stf(irec, L.a_hydro, (float)((T)ldf(irec, L.a_hydro) + F.ax));
    stf(irec, L.a_hydro + 4, (float)((T)ldf(irec, L.a_hydro + 4) + F.ay));
    stf(irec, L.a_hydro + 8, (float)((T)ldf(irec, L.a_hydro + 8) + F.az));
    stf(irec, L.u_dt, (float)((T)ldf(irec, L.u_dt) + F.u_dt));
    stf(irec, L.h_dt, (float)((T)ldf(irec, L.h_dt) + F.h_dt));
    *reinterpret_cast<int8_t*>(irec + L.min_tb) = (int8_t)F.min_ngb_time_bin;
  }
}

// Records [0, nA) = cell A, [nA, nA+nB) = cell B (pair) in one device buffer.
// Thread t < nA: i in A against B displaced by +shift (pair) or against A
// (self); t >= nA: i in B against A displaced by -shift.
template <int LOOP, typename T>
__global__ void task_kernel(Layout L, char* rec, int nA, int nB, int self, double sx,
                            double sy, double sz, int activeA, int activeB,
                            int max_active_bin, T a2_Hubble) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nA + nB) return;
  const bool inA = t < nA;
  if (inA ? !activeA : !activeB) return;
  char* irec = rec + (size_t)t * L.stride;
  const int tbi = ldb(irec, L.time_bin);
  if (tbi > max_active_bin) return;  // part_is_active (src/active.h:357)
  if (self) {
    gather_task<LOOP, T>(L, irec, rec, nA, 0., 0., 0., t, a2_Hubble);
  } else if (inA) {
    gather_task<LOOP, T>(L, irec, rec + (size_t)nA * L.stride, nB, sx, sy, sz, -1,
                         a2_Hubble);
  } else {
    gather_task<LOOP, T>(L, irec, rec, nA, -sx, -sy, -sz, -1, a2_Hubble);
  }
}

// Subset density: records srec[0..ns) (gathered i-particles) against the
// j-set jrec[0..nj) displaced by +shift; skip[k] = alias of i in the j-set.
template <typename T>
__global__ void subset_kernel(Layout L, char* srec, int ns, const char* jrec, int nj,
                              const int* skip, double sx, double sy, double sz) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ns) return;
  gather_task<LOOP_DENSITY, T>(L, srec + (size_t)t * L.stride, jrec, nj, sx, sy, sz,
                               skip[t], (T)0);
}

// ---------------------------------------------------------------------------
template <int LOOP>
static swh_status run_task(swh_context* ctx, const swh_cell_view* ci,
                           const swh_cell_view* cj, const double* shift,
                           const swh_part_layout* PL, const swh_hydro_params* P) {
  if (!ctx || !ci || !PL || !P) return SWH_ERR_ARG;
  const bool self = (cj == nullptr);
  const int nA = ci->count, nB = self ? 0 : cj->count;
  if (nA < 0 || nB < 0) return SWH_ERR_ARG;
  if (nA == 0 || (!self && nB == 0)) return SWH_OK;
  if (!ci->active && (self || !cj->active)) return SWH_OK;
  Layout L;
  SWH_TRY(make_layout(PL, &L));
  TaskWorker* w = ctx->lease();
  if (!w) {
    set_error("could not create a task stream");
    return SWH_ERR_HIP;
  }
  struct Unlease {
    swh_context* c;
    TaskWorker* w;
    ~Unlease() { c->unlease(w); }
  } unl{ctx, w};
  SWH_HIP(hipSetDevice(ctx->device));
  const size_t bA = (size_t)nA * L.stride, bB = (size_t)nB * L.stride;
  SWH_TRY(w->dparts.reserve(bA + bB));
  SWH_TRY(w->hstage.reserve(bA + bB));
  char* hs = static_cast<char*>(w->hstage.ptr);
  std::memcpy(hs, ci->parts, bA);
  if (!self) std::memcpy(hs + bA, cj->parts, bB);
  SWH_HIP(hipMemcpyAsync(w->dparts.ptr, hs, bA + bB, hipMemcpyHostToDevice, w->stream));
  const double sx = self ? 0. : shift[0], sy = self ? 0. : shift[1],
               sz = self ? 0. : shift[2];
  const int nt = nA + nB;
  const int block = 64;
  const int grid = (nt + block - 1) / block;
  const double a2H = P->a * P->a * P->H;
  if (ctx->precision == SWH_PRECISION_F64)
    hipLaunchKernelGGL((task_kernel<LOOP, double>), dim3(grid), dim3(block), 0, w->stream,
                       L, w->dparts.as<char>(), nA, nB, self ? 1 : 0, sx, sy, sz,
                       ci->active, self ? 0 : cj->active, P->max_active_bin, a2H);
  else
    hipLaunchKernelGGL((task_kernel<LOOP, float>), dim3(grid), dim3(block), 0, w->stream,
                       L, w->dparts.as<char>(), nA, nB, self ? 1 : 0, sx, sy, sz,
                       ci->active, self ? 0 : cj->active, P->max_active_bin, (float)a2H);
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemcpyAsync(hs, w->dparts.ptr, bA + bB, hipMemcpyDeviceToHost, w->stream));
  SWH_HIP(hipStreamSynchronize(w->stream));
  std::memcpy(ci->parts, hs, bA);
  if (!self) std::memcpy(cj->parts, hs + bA, bB);
  return SWH_OK;
}

static swh_status run_subset(swh_context* ctx, const swh_cell_view* ci, void* parts_i,
                             const int32_t* ind, int32_t count, const swh_cell_view* cj,
                             const double* shift, const swh_part_layout* PL,
                             const swh_hydro_params* P) {
  if (!ctx || !ci || !parts_i || (count > 0 && !ind) || !PL || !P) return SWH_ERR_ARG;
  const swh_cell_view* jc = cj ? cj : ci;
  if (count <= 0 || jc->count <= 0) return SWH_OK;
  Layout L;
  SWH_TRY(make_layout(PL, &L));
  TaskWorker* w = ctx->lease();
  if (!w) return SWH_ERR_HIP;
  struct Unlease {
    swh_context* c;
    TaskWorker* w;
    ~Unlease() { c->unlease(w); }
  } unl{ctx, w};
  SWH_HIP(hipSetDevice(ctx->device));
  const size_t st = (size_t)L.stride;
  const size_t bJ = (size_t)jc->count * st, bS = (size_t)count * st;
  SWH_TRY(w->dparts.reserve(bJ));
  SWH_TRY(w->dparts2.reserve(bS));
  SWH_TRY(w->dself.reserve((size_t)count * sizeof(int)));
  SWH_TRY(w->hstage.reserve(bJ));
  SWH_TRY(w->hstage2.reserve(bS + (size_t)count * sizeof(int)));
  std::memcpy(w->hstage.ptr, jc->parts, bJ);
  char* hs = static_cast<char*>(w->hstage2.ptr);
  int* hskip = reinterpret_cast<int*>(hs + bS);
  const char* jbase = static_cast<const char*>(jc->parts);
  char* ibase = static_cast<char*>(parts_i);
  for (int k = 0; k < count; k++) {
    const char* rec = ibase + (size_t)ind[k] * st;
    std::memcpy(hs + (size_t)k * st, rec, st);
    // DOSELF_SUBSET skips pi == pj; only a self-subset can alias the j-set.
    hskip[k] = -1;
    if (!cj && rec >= jbase && rec < jbase + bJ) hskip[k] = (int)((rec - jbase) / st);
  }
  SWH_HIP(hipMemcpyAsync(w->dparts.ptr, w->hstage.ptr, bJ, hipMemcpyHostToDevice, w->stream));
  SWH_HIP(hipMemcpyAsync(w->dparts2.ptr, hs, bS, hipMemcpyHostToDevice, w->stream));
  SWH_HIP(hipMemcpyAsync(w->dself.ptr, hskip, (size_t)count * sizeof(int),
                         hipMemcpyHostToDevice, w->stream));
  const double sx = cj ? shift[0] : 0., sy = cj ? shift[1] : 0., sz = cj ? shift[2] : 0.;
  const int block = 64, grid = (count + block - 1) / block;
  // subset i's interact as x_i - shift  <=>  j displaced by +shift
  if (ctx->precision == SWH_PRECISION_F64)
    hipLaunchKernelGGL((subset_kernel<double>), dim3(grid), dim3(block), 0, w->stream, L,
                       w->dparts2.as<char>(), count, w->dparts.as<char>(), jc->count,
                       w->dself.as<int>(), sx, sy, sz);
  else
    hipLaunchKernelGGL((subset_kernel<float>), dim3(grid), dim3(block), 0, w->stream, L,
                       w->dparts2.as<char>(), count, w->dparts.as<char>(), jc->count,
                       w->dself.as<int>(), sx, sy, sz);
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemcpyAsync(hs, w->dparts2.ptr, bS, hipMemcpyDeviceToHost, w->stream));
  SWH_HIP(hipStreamSynchronize(w->stream));
  for (int k = 0; k < count; k++)
    std::memcpy(ibase + (size_t)ind[k] * st, hs + (size_t)k * st, st);
  return SWH_OK;
}

// ---------------------------------------------------------------------------
// P2P gravity per task
// ---------------------------------------------------------------------------
template <typename T, bool TRUNC>
__global__ void grav_task_kernel(GLayout L, char* gi, int ni, const char* gj, int nj,
                                 int self, double fx, double fy, double fz, int periodic,
                                 T dimx, T dimy, T dimz, T r_s_inv, int max_active_bin,
                                 const swh_multipole* __restrict__ mpj, MacParams mac) {
  const int pid = blockIdx.x * blockDim.x + threadIdx.x;
  if (pid >= ni) return;
  char* ri = gi + (size_t)pid * L.stride;
  const int tbi = ldb(ri, L.time_bin);
  if (tbi == kTimeBinInhibited || tbi > max_active_bin) return;
  // gravity_cache frame: positions relative to (fx,fy,fz), evaluated in T
  const T x_i = (T)(ldd(ri, L.x) - fx), y_i = (T)(ldd(ri, L.x + 8) - fy),
          z_i = (T)(ldd(ri, L.x + 16) - fz);
  const T h_i = ldf(ri, L.epsilon);
  T ax = 0, ay = 0, az = 0, pot = 0;
  if (mpj) {
    // gravity_cache_populate's use_mpole (float, frame = the pair's zero
    // shift), then runner_dopair_grav_pm_full / _truncated in T
    const double xd = ldd(ri, L.x), yd = ldd(ri, L.x + 8), zd = ldd(ri, L.x + 16);
    const float oag = L.old_a_grav_norm >= 0 ? ldf(ri, L.old_a_grav_norm) : 0.f;
    const float eps_i = ldf(ri, L.epsilon);
    if (m2p_accept(mac, mac_source(*mpj), (float)xd, (float)yd, (float)zd, eps_i, oag)) {
      T dx = (T)(mpj->CoM[0] - xd), dy = (T)(mpj->CoM[1] - yd), dz = (T)(mpj->CoM[2] - zd);
      if (periodic) {
        dx = dx > (T)0.5 * dimx ? dx - dimx : (dx < (T)-0.5 * dimx ? dx + dimx : dx);
        dy = dy > (T)0.5 * dimy ? dy - dimy : (dy < (T)-0.5 * dimy ? dy + dimy : dy);
        dz = dz > (T)0.5 * dimz ? dz - dimz : (dz < (T)-0.5 * dimz ? dz + dimz : dz);
      }
      T F[4];
      m2p<T>(mpj->M, dx, dy, dz, (T)fmaxf(eps_i, mpj->max_softening), TRUNC, r_s_inv, F);
      stf(ri, L.a_grav, ldf(ri, L.a_grav) + (float)F[1]);
      stf(ri, L.a_grav + 4, ldf(ri, L.a_grav + 4) + (float)F[2]);
      stf(ri, L.a_grav + 8, ldf(ri, L.a_grav + 8) + (float)F[3]);
      stf(ri, L.potential, ldf(ri, L.potential) + (float)F[0]);
      return;
    }
  }
  for (int pjd = 0; pjd < nj; pjd++) {
    if (self && pjd == pid) continue;
    const char* rj = gj + (size_t)pjd * L.stride;
    const T mass_j = (ldb(rj, L.time_bin) == kTimeBinInhibited) ? (T)0 : (T)ldf(rj, L.mass);
    T dx = (T)(ldd(rj, L.x) - fx) - x_i;
    T dy = (T)(ldd(rj, L.x + 8) - fy) - y_i;
    T dz = (T)(ldd(rj, L.x + 16) - fz) - z_i;
    if (periodic) {
      dx = dx > (T)0.5 * dimx ? dx - dimx : (dx < (T)-0.5 * dimx ? dx + dimx : dx);
      dy = dy > (T)0.5 * dimy ? dy - dimy : (dy < (T)-0.5 * dimy ? dy + dimy : dy);
      dz = dz > (T)0.5 * dimz ? dz - dimz : (dz < (T)-0.5 * dimz ? dz + dimz : dz);
    }
    const T r2 = dx * dx + dy * dy + dz * dz;
    const T h = tmax(h_i, (T)ldf(rj, L.epsilon));
    const T h2 = h * h;
    const T h_inv = (T)1 / h;
    const T h_inv3 = h_inv * h_inv * h_inv;
    T f_ij, pot_ij;
    iact_grav_pp<T, TRUNC>(r2, h2, h_inv, h_inv3, mass_j, r_s_inv, f_ij, pot_ij);
    ax += f_ij * dx;
    ay += f_ij * dy;
    az += f_ij * dz;
    pot += pot_ij;
  }
  stf(ri, L.a_grav, ldf(ri, L.a_grav) + (float)ax);
  stf(ri, L.a_grav + 4, ldf(ri, L.a_grav + 4) + (float)ay);
  stf(ri, L.a_grav + 8, ldf(ri, L.a_grav + 8) + (float)az);
  stf(ri, L.potential, ldf(ri, L.potential) + (float)pot);
}

template <typename T>
static void launch_grav_task(hipStream_t s, const GLayout& L, char* gi, int ni,
                             const char* gj, int nj, int self, const double f[3],
                             int periodic, const swh_grav_params* G, bool trunc,
                             const swh_multipole* mpj = nullptr) {
  const int block = 64, grid = (ni + block - 1) / block;
  const MacParams mac = mac_params(G);
  if (trunc)
    hipLaunchKernelGGL((grav_task_kernel<T, true>), dim3(grid), dim3(block), 0, s, L, gi,
                       ni, gj, nj, self, f[0], f[1], f[2], periodic, (T)G->dim[0],
                       (T)G->dim[1], (T)G->dim[2], (T)G->r_s_inv, G->max_active_bin, mpj, mac);
  else
    hipLaunchKernelGGL((grav_task_kernel<T, false>), dim3(grid), dim3(block), 0, s, L, gi,
                       ni, gj, nj, self, f[0], f[1], f[2], periodic, (T)G->dim[0],
                       (T)G->dim[1], (T)G->dim[2], (T)G->r_s_inv, G->max_active_bin, mpj, mac);
}

}  // namespace swh

using namespace swh;

extern "C" {

swh_status swh_doself_density(swh_context* c, const swh_cell_view* ci,
                              const swh_part_layout* L, const swh_hydro_params* P) {
  return run_task<LOOP_DENSITY>(c, ci, nullptr, nullptr, L, P);
}
swh_status swh_dopair_density(swh_context* c, const swh_cell_view* ci,
                              const swh_cell_view* cj, const double shift[3],
                              const swh_part_layout* L, const swh_hydro_params* P) {
  if (!cj || !shift) return SWH_ERR_ARG;
  return run_task<LOOP_DENSITY>(c, ci, cj, shift, L, P);
}
swh_status swh_doself_gradient(swh_context* c, const swh_cell_view* ci,
                               const swh_part_layout* L, const swh_hydro_params* P) {
  return run_task<LOOP_GRADIENT>(c, ci, nullptr, nullptr, L, P);
}
swh_status swh_dopair_gradient(swh_context* c, const swh_cell_view* ci,
                               const swh_cell_view* cj, const double shift[3],
                               const swh_part_layout* L, const swh_hydro_params* P) {
  if (!cj || !shift) return SWH_ERR_ARG;
  return run_task<LOOP_GRADIENT>(c, ci, cj, shift, L, P);
}
swh_status swh_doself_force(swh_context* c, const swh_cell_view* ci,
                            const swh_part_layout* L, const swh_hydro_params* P) {
  return run_task<LOOP_FORCE>(c, ci, nullptr, nullptr, L, P);
}
swh_status swh_dopair_force(swh_context* c, const swh_cell_view* ci,
                            const swh_cell_view* cj, const double shift[3],
                            const swh_part_layout* L, const swh_hydro_params* P) {
  if (!cj || !shift) return SWH_ERR_ARG;
  return run_task<LOOP_FORCE>(c, ci, cj, shift, L, P);
}
swh_status swh_doself_subset_density(swh_context* c, const swh_cell_view* ci,
                                     void* parts_i, const int32_t* ind, int32_t count,
                                     const swh_part_layout* L, const swh_hydro_params* P) {
  return run_subset(c, ci, parts_i, ind, count, nullptr, nullptr, L, P);
}
swh_status swh_dopair_subset_density(swh_context* c, const swh_cell_view* ci,
                                     void* parts_i, const int32_t* ind, int32_t count,
                                     const swh_cell_view* cj, const double shift[3],
                                     const swh_part_layout* L, const swh_hydro_params* P) {
  if (!cj || !shift) return SWH_ERR_ARG;
  return run_subset(c, ci, parts_i, ind, count, cj, shift, L, P);
}

// runner_doself_grav_pp (src/runner_doiact_grav.c:1788-1871)
swh_status swh_grav_self_pp(swh_context* ctx, const swh_gcell_view* c,
                            const swh_gpart_layout* GL, const swh_grav_params* G) {
  if (!ctx || !c || !GL || !G) return SWH_ERR_ARG;
  if (c->count <= 0 || !c->active) return SWH_OK;
  GLayout L;
  SWH_TRY(make_glayout(GL, &L));
  TaskWorker* w = ctx->lease();
  if (!w) return SWH_ERR_HIP;
  struct Unlease {
    swh_context* c;
    TaskWorker* w;
    ~Unlease() { c->unlease(w); }
  } unl{ctx, w};
  SWH_HIP(hipSetDevice(ctx->device));
  const size_t b = (size_t)c->count * L.stride;
  SWH_TRY(w->dparts.reserve(b));
  SWH_TRY(w->hstage.reserve(b));
  std::memcpy(w->hstage.ptr, c->gparts, b);
  SWH_HIP(hipMemcpyAsync(w->dparts.ptr, w->hstage.ptr, b, hipMemcpyHostToDevice, w->stream));
  const double frame[3] = {c->loc[0] + 0.5 * c->width[0], c->loc[1] + 0.5 * c->width[1],
                           c->loc[2] + 0.5 * c->width[2]};
  const bool trunc = G->periodic && (2. * c->r_max > G->r_cut_min);
  if (ctx->precision == SWH_PRECISION_F64)
    launch_grav_task<double>(w->stream, L, w->dparts.as<char>(), c->count,
                             w->dparts.as<char>(), c->count, 1, frame, 0, G, trunc);
  else
    launch_grav_task<float>(w->stream, L, w->dparts.as<char>(), c->count,
                            w->dparts.as<char>(), c->count, 1, frame, 0, G, trunc);
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemcpyAsync(w->hstage.ptr, w->dparts.ptr, b, hipMemcpyDeviceToHost, w->stream));
  SWH_HIP(hipStreamSynchronize(w->stream));
  std::memcpy(c->gparts, w->hstage.ptr, b);
  return SWH_OK;
}

// runner_dopair_grav_pp (src/runner_doiact_grav.c:1202-1425): P2P, and with
// allow_mpole the M2P route for the particles passing the MAC against the
// other cell's multipole (allow_multipole_i/j need more than one particle,
// runner_doiact_grav.c:1273-1274).
swh_status swh_grav_pair_pp(swh_context* ctx, const swh_gcell_view* ci,
                            const swh_gcell_view* cj, int symmetric, int allow_mpole,
                            const swh_gpart_layout* GL, const swh_grav_params* G) {
  if (!ctx || !ci || !cj || !GL || !G) return SWH_ERR_ARG;
  const bool do_i = ci->active, do_j = cj->active && symmetric;
  if (!do_i && !do_j) return SWH_OK;
  if (ci->count <= 0 || cj->count <= 0) return SWH_OK;
  const bool mp_j = allow_mpole && cj->count > 1;  // multipole of cj used by ci's particles
  const bool mp_i = allow_mpole && ci->count > 1;
  if ((mp_j && do_i && !cj->multipole) || (mp_i && do_j && !ci->multipole)) {
    set_error("allow_mpole needs the cells' multipoles (swh_gcell_view.multipole)");
    return SWH_ERR_ARG;
  }
  GLayout L;
  SWH_TRY(make_glayout(GL, &L));
  TaskWorker* w = ctx->lease();
  if (!w) return SWH_ERR_HIP;
  struct Unlease {
    swh_context* c;
    TaskWorker* w;
    ~Unlease() { c->unlease(w); }
  } unl{ctx, w};
  SWH_HIP(hipSetDevice(ctx->device));
  const size_t bi = (size_t)ci->count * L.stride, bj = (size_t)cj->count * L.stride;
  const size_t bm = 2 * sizeof(swh_multipole);  // multipoles of ci, cj after the records
  SWH_TRY(w->dparts.reserve(bi + bj + bm));
  SWH_TRY(w->dparts2.reserve(bi + bj + bm));
  SWH_TRY(w->hstage.reserve(bi + bj + bm));
  char* hs = static_cast<char*>(w->hstage.ptr);
  std::memcpy(hs, ci->gparts, bi);
  std::memcpy(hs + bi, cj->gparts, bj);
  swh_multipole* hm = reinterpret_cast<swh_multipole*>(hs + bi + bj);
  if (ci->multipole) hm[0] = *ci->multipole;
  if (cj->multipole) hm[1] = *cj->multipole;
  SWH_HIP(hipMemcpyAsync(w->dparts.ptr, hs, bi + bj + bm, hipMemcpyHostToDevice, w->stream));
  // read-only source copy so both directions see the pre-task accelerations
  SWH_HIP(hipMemcpyAsync(w->dparts2.ptr, w->dparts.ptr, bi + bj + bm, hipMemcpyDeviceToDevice,
                         w->stream));
  const swh_multipole* dm = reinterpret_cast<const swh_multipole*>(w->dparts2.as<char>() + bi + bj);
  bool trunc = false;
  if (G->periodic) {
    double d2 = 0;
    for (int k = 0; k < 3; k++) {
      float dx = (float)cj->CoM[k] - (float)ci->CoM[k];
      dx = dx > 0.5f * G->dim[k] ? dx - G->dim[k] : (dx < -0.5f * G->dim[k] ? dx + G->dim[k] : dx);
      d2 += (double)dx * dx;
    }
    trunc = (sqrt(d2) + ci->r_max + cj->r_max) > G->r_cut_min;
  }
  const double zero[3] = {0., 0., 0.};
  char* di = w->dparts.as<char>();
  char* dj = di + bi;
  const char* si = w->dparts2.as<char>();
  const char* sj = si + bi;
  const bool f64 = ctx->precision == SWH_PRECISION_F64;
  const swh_multipole* use_j = mp_j ? dm + 1 : nullptr;
  const swh_multipole* use_i = mp_i ? dm : nullptr;
  if (do_i) {
    if (f64) launch_grav_task<double>(w->stream, L, di, ci->count, sj, cj->count, 0, zero, G->periodic, G, trunc, use_j);
    else launch_grav_task<float>(w->stream, L, di, ci->count, sj, cj->count, 0, zero, G->periodic, G, trunc, use_j);
  }
  if (do_j) {
    if (f64) launch_grav_task<double>(w->stream, L, dj, cj->count, si, ci->count, 0, zero, G->periodic, G, trunc, use_i);
    else launch_grav_task<float>(w->stream, L, dj, cj->count, si, ci->count, 0, zero, G->periodic, G, trunc, use_i);
  }
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemcpyAsync(hs, w->dparts.ptr, bi + bj, hipMemcpyDeviceToHost, w->stream));
  SWH_HIP(hipStreamSynchronize(w->stream));
  std::memcpy(ci->gparts, hs, bi);
  std::memcpy(cj->gparts, hs + bi, bj);
  return SWH_OK;
}

}  // extern "C"
