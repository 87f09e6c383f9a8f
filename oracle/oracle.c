/*
 * oracle/oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of SWIFT's SPH density/gradient/force neighbour loops
 * and leaf-leaf P2P gravity (reference: /root/reference @ SWIFT 0.9.0), used
 * as the parity CHECKER for the HIP path and as the CPU baseline timer
 * (bench.py cpu_baseline, kind "port"). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product
 * (swift_subtask_dev_amd) never links or calls it.
 *
 * Compiled twice per SPH kernel (oracle/Makefile; cubic spline, and Wendland C2
 * with -DORACLE_WENDLAND_C2 into liboracle_wc2_{f32,f64}.so):
 *   ORACLE_F32 -> liboracle_f32.so, symbols orf_*: float arithmetic with the
 *      reference's exact operation order, operating in place on the 160-byte
 *      struct part (include/swift_compat.h). This is the faithful restatement.
 *   ORACLE_F64 -> liboracle_f64.so, symbols ord_*: the same formulas with every
 *      float temporary and accumulator promoted to double (constants keep the
 *      reference's float values). This is the fp64 reference the GPU's fp64
 *      path is compared with at ~float-ulp tolerance.
 *
 * Pinning (see DESIGN.md "Oracle"): the reference C build needs a generated
 * config.h and an hdf5.h stand-in, so per the task rules it is treated as
 * unbuildable here. The restatement is pinned by the reference's own tests:
 *   - test27cells/test125cells/testActivePair/testPeriodicBC structure: sorted
 *     DOSELF/DOPAIR loops vs brute force under tests/tolerance_*.dat;
 *   - testPotentialSelf/testPotentialPair analytic KATs (rel 1e-6 / 2e-6);
 *   - testSymmetry identity (symmetric iact == two non-symmetric iacts);
 *   - test125cells analytic fields (get_solution: rho, div_v, a_hydro);
 *   - reference-run values recorded in SURVEY.md (kernel_root 0.418429,
 *     kernel_norm 25.492, sizeof(struct part)=160, 47.82 directed density
 *     interactions per particle on the perturbed-lattice recipe).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "swift_compat.h"

#if defined(ORACLE_F64)
typedef double real;
#define PFX(name) ord_##name
#define SQRT sqrt
#define FABS fabs
#define EXP exp
#else
#define ORACLE_F32 1
typedef float real;
#define PFX(name) orf_##name
#define SQRT sqrtf
#define FABS fabsf
#define EXP expf
#endif

#define API __attribute__((visibility("default")))

static inline real rmax(real a, real b) { return a > b ? a : b; }
static inline real rmin(real a, real b) { return a < b ? a : b; }

/* ======================================================================== */
/* Constants — restated from src/kernel_hydro.h:45-64,121-147,195-241 (3D),
 * src/dimension.h:40-43, src/adiabatic_index.h:43-44,
 * src/hydro/SPHENIX/hydro_parameters.h:53. Same C expressions, so the float
 * values are bit-identical to the reference macros. The kernel is a
 * compile-time choice as in SWIFT (configure --with-kernel): cubic spline by
 * default, Wendland C2 with -DORACLE_WENDLAND_C2 (liboracle_wc2_*.so).       */
/* ======================================================================== */
#if defined(ORACLE_WENDLAND_C2)
#define kernel_degree 5
#define kernel_ivals 1
#define kernel_gamma ((float)(1.936492))
#define kernel_constant ((float)(21. * M_1_PI / 2.))
#else
#define kernel_degree 3
#define kernel_ivals 2
#define kernel_gamma ((float)(1.825742))
#define kernel_constant ((float)(16. * M_1_PI))
#endif
#define kernel_gamma_inv ((float)(1. / kernel_gamma))
#define kernel_gamma2 ((float)(kernel_gamma * kernel_gamma))
#define kernel_gamma_dim ((float)(kernel_gamma * kernel_gamma * kernel_gamma))
#define kernel_gamma_inv_dim \
  ((float)(1. / (kernel_gamma * kernel_gamma * kernel_gamma)))
#define kernel_gamma_inv_dim_plus_one \
  ((float)(1. / (kernel_gamma * kernel_gamma * kernel_gamma * kernel_gamma)))
#define kernel_ivals_f ((float)(kernel_ivals))
#if defined(ORACLE_WENDLAND_C2)
static const float kernel_coeffs[(kernel_degree + 1) * (kernel_ivals + 1)] = {
    4.f, -15.f, 20.f, -10.f, 0.f, 1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#else
static const float kernel_coeffs[(kernel_degree + 1) * (kernel_ivals + 1)] = {
    3.f, -3.f, 0.f, 0.5f, -1.f, 3.f, -3.f, 1.f, 0.f, 0.f, 0.f, 0.f};
#endif
#define kernel_root \
  ((float)(kernel_coeffs[kernel_degree]) * kernel_constant * kernel_gamma_inv_dim)
#define hydro_dimension 3.f
#define hydro_dimension_inv 0.3333333333f
#define hydro_dimension_unit_sphere ((float)(4. * M_PI / 3.))
#define kernel_norm ((float)(hydro_dimension_unit_sphere * kernel_gamma_dim))
#define hydro_gamma 1.66666666666666667f
#define hydro_gamma_minus_one 0.66666666666666667f
#define const_viscosity_beta 3.0f

API float PFX(kernel_root)(void) { return kernel_root; }
API float PFX(kernel_norm)(void) { return kernel_norm; }
API float PFX(kernel_gamma)(void) { return kernel_gamma; }

static inline real pow_dimension(real x) { return x * x * x; }
static inline real pow_dimension_plus_one(real x) {
  const real x2 = x * x;
  return x2 * x2;
}
static inline real pow_dimension_minus_one(real x) { return x * x; }

/* src/kernel_hydro.h:257-284 */
static inline void kernel_deval(real u, real *W, real *dW_dx) {
  const real x = u * (real)kernel_gamma_inv;
  const int temp = (int)(x * (real)kernel_ivals_f);
  const int ind = temp > kernel_ivals ? kernel_ivals : temp;
  const float *const coeffs = &kernel_coeffs[ind * (kernel_degree + 1)];
  real w = (real)coeffs[0] * x + (real)coeffs[1];
  real dw_dx = (real)coeffs[0];
  for (int k = 2; k <= kernel_degree; k++) {
    dw_dx = dw_dx * x + w;
    w = x * w + (real)coeffs[k];
  }
  w = rmax(w, (real)0);
  dw_dx = rmin(dw_dx, (real)0);
  *W = w * (real)kernel_constant * (real)kernel_gamma_inv_dim;
  *dW_dx = dw_dx * (real)kernel_constant * (real)kernel_gamma_inv_dim_plus_one;
}

API void PFX(kernel_deval)(real u, real *W, real *dW) { kernel_deval(u, W, dW); }

/* ======================================================================== */
/* Oracle particle record. In the f32 build it IS the ABI struct part; in   */
/* the f64 build every float field is promoted to double (x is double in    */
/* both, as in the reference).                                              */
/* ======================================================================== */
#ifdef ORACLE_F32
typedef struct part opart;
#else
typedef struct opart {
  long long id;
  double x[3];
  real v[3];
  real a_hydro[3];
  real mass, h, u, u_dt, rho;
  struct {
    real div_v, div_v_dt, div_v_previous_step, alpha, v_sig;
  } viscosity;
  struct {
    real laplace_u, alpha;
  } diffusion;
  union {
    struct {
      real wcount, wcount_dh, rho_dh, rot_v[3];
    } density;
    struct {
      real f, pressure, soundspeed, h_dt, balsara, alpha_visc_max_ngb;
    } force;
  };
  timebin_t time_bin;
  struct {
    timebin_t min_ngb_time_bin;
  } limiter_data;
} opart;
#endif

/* Which union member is live when converting f64 records <-> ABI parts. */
enum { PHASE_DENSITY = 0, PHASE_FORCE = 1 };

__attribute__((unused)) static void part_to_opart(const struct part *p, opart *o, int phase) {
#ifdef ORACLE_F32
  (void)phase;
  *o = *p;
#else
  o->id = p->id;
  for (int k = 0; k < 3; k++) {
    o->x[k] = p->x[k];
    o->v[k] = p->v[k];
    o->a_hydro[k] = p->a_hydro[k];
  }
  o->mass = p->mass; o->h = p->h; o->u = p->u; o->u_dt = p->u_dt; o->rho = p->rho;
  o->viscosity.div_v = p->viscosity.div_v;
  o->viscosity.div_v_dt = p->viscosity.div_v_dt;
  o->viscosity.div_v_previous_step = p->viscosity.div_v_previous_step;
  o->viscosity.alpha = p->viscosity.alpha;
  o->viscosity.v_sig = p->viscosity.v_sig;
  o->diffusion.laplace_u = p->diffusion.laplace_u;
  o->diffusion.alpha = p->diffusion.alpha;
  if (phase == PHASE_DENSITY) {
    o->density.wcount = p->density.wcount;
    o->density.wcount_dh = p->density.wcount_dh;
    o->density.rho_dh = p->density.rho_dh;
    for (int k = 0; k < 3; k++) o->density.rot_v[k] = p->density.rot_v[k];
  } else {
    o->force.f = p->force.f;
    o->force.pressure = p->force.pressure;
    o->force.soundspeed = p->force.soundspeed;
    o->force.h_dt = p->force.h_dt;
    o->force.balsara = p->force.balsara;
    o->force.alpha_visc_max_ngb = p->force.alpha_visc_max_ngb;
  }
  o->time_bin = p->time_bin;
  o->limiter_data.min_ngb_time_bin = p->limiter_data.min_ngb_time_bin;
#endif
}

__attribute__((unused)) static void opart_to_part(const opart *o, struct part *p, int phase) {
#ifdef ORACLE_F32
  (void)phase;
  *p = *o;
#else
  for (int k = 0; k < 3; k++) {
    p->v[k] = (float)o->v[k];
    p->a_hydro[k] = (float)o->a_hydro[k];
  }
  p->h = (float)o->h; p->u = (float)o->u; p->u_dt = (float)o->u_dt;
  p->rho = (float)o->rho;
  p->viscosity.div_v = (float)o->viscosity.div_v;
  p->viscosity.div_v_dt = (float)o->viscosity.div_v_dt;
  p->viscosity.div_v_previous_step = (float)o->viscosity.div_v_previous_step;
  p->viscosity.alpha = (float)o->viscosity.alpha;
  p->viscosity.v_sig = (float)o->viscosity.v_sig;
  p->diffusion.laplace_u = (float)o->diffusion.laplace_u;
  p->diffusion.alpha = (float)o->diffusion.alpha;
  if (phase == PHASE_DENSITY) {
    p->density.wcount = (float)o->density.wcount;
    p->density.wcount_dh = (float)o->density.wcount_dh;
    p->density.rho_dh = (float)o->density.rho_dh;
    for (int k = 0; k < 3; k++) p->density.rot_v[k] = (float)o->density.rot_v[k];
  } else {
    p->force.f = (float)o->force.f;
    p->force.pressure = (float)o->force.pressure;
    p->force.soundspeed = (float)o->force.soundspeed;
    p->force.h_dt = (float)o->force.h_dt;
    p->force.balsara = (float)o->force.balsara;
    p->force.alpha_visc_max_ngb = (float)o->force.alpha_visc_max_ngb;
  }
  p->limiter_data.min_ngb_time_bin = o->limiter_data.min_ngb_time_bin;
#endif
}

static inline int part_is_active(const opart *p, timebin_t max_active_bin) {
  return p->time_bin <= max_active_bin; /* src/active.h:357-373 */
}
static inline int part_is_inhibited(const opart *p) {
  return p->time_bin == time_bin_inhibited; /* src/active.h */
}

/* ======================================================================== */
/* SPHENIX interaction functions — src/hydro/SPHENIX/hydro_iact.h.          */
/* a=1,H=0-independent except where the reference uses them.                */
/* ======================================================================== */

/* hydro_iact.h:46-116 */
static inline void iact_density(real r2, const real dx[3], real hi, real hj,
                                opart *pi, opart *pj, real a, real H) {
  (void)a; (void)H;
  real wi, wj, wi_dx, wj_dx, dv[3], curlvr[3];
  const real r = SQRT(r2);
  const real mi = pi->mass, mj = pj->mass;
  const real hi_inv = (real)1 / hi;
  const real ui = r * hi_inv;
  kernel_deval(ui, &wi, &wi_dx);
  pi->rho += mj * wi;
  pi->density.rho_dh -= mj * ((real)hydro_dimension * wi + ui * wi_dx);
  pi->density.wcount += wi;
  pi->density.wcount_dh -= ((real)hydro_dimension * wi + ui * wi_dx);
  const real hj_inv = (real)1 / hj;
  const real uj = r * hj_inv;
  kernel_deval(uj, &wj, &wj_dx);
  pj->rho += mi * wj;
  pj->density.rho_dh -= mi * ((real)hydro_dimension * wj + uj * wj_dx);
  pj->density.wcount += wj;
  pj->density.wcount_dh -= ((real)hydro_dimension * wj + uj * wj_dx);
  const real r_inv = r ? (real)1 / r : (real)0;
  const real faci = mj * wi_dx * r_inv;
  const real facj = mi * wj_dx * r_inv;
  dv[0] = pi->v[0] - pj->v[0];
  dv[1] = pi->v[1] - pj->v[1];
  dv[2] = pi->v[2] - pj->v[2];
  const real dvdr = dv[0] * dx[0] + dv[1] * dx[1] + dv[2] * dx[2];
  pi->viscosity.div_v -= faci * dvdr;
  pj->viscosity.div_v -= facj * dvdr;
  curlvr[0] = dv[1] * dx[2] - dv[2] * dx[1];
  curlvr[1] = dv[2] * dx[0] - dv[0] * dx[2];
  curlvr[2] = dv[0] * dx[1] - dv[1] * dx[0];
  pi->density.rot_v[0] += faci * curlvr[0];
  pi->density.rot_v[1] += faci * curlvr[1];
  pi->density.rot_v[2] += faci * curlvr[2];
  pj->density.rot_v[0] += facj * curlvr[0];
  pj->density.rot_v[1] += facj * curlvr[1];
  pj->density.rot_v[2] += facj * curlvr[2];
}

/* hydro_iact.h:130-178 */
static inline void iact_nonsym_density(real r2, const real dx[3], real hi,
                                       real hj, opart *pi, const opart *pj,
                                       real a, real H) {
  (void)hj; (void)a; (void)H;
  real wi, wi_dx, dv[3], curlvr[3];
  const real mj = pj->mass;
  const real r = SQRT(r2);
  const real h_inv = (real)1 / hi;
  const real ui = r * h_inv;
  kernel_deval(ui, &wi, &wi_dx);
  pi->rho += mj * wi;
  pi->density.rho_dh -= mj * ((real)hydro_dimension * wi + ui * wi_dx);
  pi->density.wcount += wi;
  pi->density.wcount_dh -= ((real)hydro_dimension * wi + ui * wi_dx);
  const real r_inv = r ? (real)1 / r : (real)0;
  const real faci = mj * wi_dx * r_inv;
  dv[0] = pi->v[0] - pj->v[0];
  dv[1] = pi->v[1] - pj->v[1];
  dv[2] = pi->v[2] - pj->v[2];
  const real dvdr = dv[0] * dx[0] + dv[1] * dx[1] + dv[2] * dx[2];
  pi->viscosity.div_v -= faci * dvdr;
  curlvr[0] = dv[1] * dx[2] - dv[2] * dx[1];
  curlvr[1] = dv[2] * dx[0] - dv[0] * dx[2];
  curlvr[2] = dv[0] * dx[1] - dv[1] * dx[0];
  pi->density.rot_v[0] += faci * curlvr[0];
  pi->density.rot_v[1] += faci * curlvr[1];
  pi->density.rot_v[2] += faci * curlvr[2];
}

/* src/hydro/SPHENIX/hydro.h:490-498 (via src/signal_velocity.h) */
static inline real signal_velocity(const opart *pi, const opart *pj, real mu_ij,
                                   real beta) {
  return pi->force.soundspeed + pj->force.soundspeed - beta * mu_ij;
}

/* hydro_iact.h:196-257 */
static inline void iact_gradient(real r2, const real dx[3], real hi, real hj,
                                 opart *pi, opart *pj, real a, real H) {
  const real r = SQRT(r2);
  const real r_inv = r ? (real)1 / r : (real)0;
  const real fac_mu = (real)1; /* pow_three_gamma_minus_five_over_two, gamma=5/3 */
  const real a2_Hubble = a * a * H;
  const real dvdr = (pi->v[0] - pj->v[0]) * dx[0] + (pi->v[1] - pj->v[1]) * dx[1] +
                    (pi->v[2] - pj->v[2]) * dx[2];
  const real dvdr_Hubble = dvdr + a2_Hubble * r2;
  const real omega_ij = rmin(dvdr_Hubble, (real)0);
  const real mu_ij = fac_mu * r_inv * omega_ij;
  const real new_v_sig = signal_velocity(pi, pj, mu_ij, (real)const_viscosity_beta);
  pi->viscosity.v_sig = rmax(pi->viscosity.v_sig, new_v_sig);
  pj->viscosity.v_sig = rmax(pj->viscosity.v_sig, new_v_sig);
  real wi, wi_dx, wj, wj_dx;
  const real ui = r / hi;
  const real uj = r / hj;
  kernel_deval(ui, &wi, &wi_dx);
  kernel_deval(uj, &wj, &wj_dx);
  const real delta_u_factor = (pi->u - pj->u) * r_inv;
  pi->diffusion.laplace_u += pj->mass * delta_u_factor * wi_dx / pj->rho;
  pj->diffusion.laplace_u -= pi->mass * delta_u_factor * wj_dx / pi->rho;
  const real alpha_i = pi->viscosity.alpha;
  const real alpha_j = pj->viscosity.alpha;
  pi->force.alpha_visc_max_ngb = rmax(pi->force.alpha_visc_max_ngb, alpha_j);
  pj->force.alpha_visc_max_ngb = rmax(pj->force.alpha_visc_max_ngb, alpha_i);
}

/* hydro_iact.h:276-329 */
static inline void iact_nonsym_gradient(real r2, const real dx[3], real hi,
                                        real hj, opart *pi, const opart *pj,
                                        real a, real H) {
  (void)hj;
  const real r = SQRT(r2);
  const real r_inv = r ? (real)1 / r : (real)0;
  const real fac_mu = (real)1;
  const real a2_Hubble = a * a * H;
  const real dvdr = (pi->v[0] - pj->v[0]) * dx[0] + (pi->v[1] - pj->v[1]) * dx[1] +
                    (pi->v[2] - pj->v[2]) * dx[2];
  const real dvdr_Hubble = dvdr + a2_Hubble * r2;
  const real omega_ij = rmin(dvdr_Hubble, (real)0);
  const real mu_ij = fac_mu * r_inv * omega_ij;
  const real new_v_sig = signal_velocity(pi, pj, mu_ij, (real)const_viscosity_beta);
  pi->viscosity.v_sig = rmax(pi->viscosity.v_sig, new_v_sig);
  real wi, wi_dx;
  const real ui = r / hi;
  kernel_deval(ui, &wi, &wi_dx);
  const real delta_u_factor = (pi->u - pj->u) * r_inv;
  pi->diffusion.laplace_u += pj->mass * delta_u_factor * wi_dx / pj->rho;
  const real alpha_j = pj->viscosity.alpha;
  pi->force.alpha_visc_max_ngb = rmax(pi->force.alpha_visc_max_ngb, alpha_j);
}

/* hydro_iact.h:343-474 */
static inline void iact_force(real r2, const real dx[3], real hi, real hj,
                              opart *pi, opart *pj, real a, real H) {
  const real fac_mu = (real)1;
  const real a2_Hubble = a * a * H;
  const real r = SQRT(r2);
  const real r_inv = r ? (real)1 / r : (real)0;
  const real mj = pj->mass, mi = pi->mass;
  const real rhoi = pi->rho, rhoj = pj->rho;
  const real pressurei = pi->force.pressure, pressurej = pj->force.pressure;
  const real hi_inv = (real)1 / hi;
  const real hid_inv = pow_dimension_plus_one(hi_inv);
  const real xi = r * hi_inv;
  real wi, wi_dx;
  kernel_deval(xi, &wi, &wi_dx);
  const real wi_dr = hid_inv * wi_dx;
  const real hj_inv = (real)1 / hj;
  const real hjd_inv = pow_dimension_plus_one(hj_inv);
  const real xj = r * hj_inv;
  real wj, wj_dx;
  kernel_deval(xj, &wj, &wj_dx);
  const real wj_dr = hjd_inv * wj_dx;
  const real dvdr = (pi->v[0] - pj->v[0]) * dx[0] + (pi->v[1] - pj->v[1]) * dx[1] +
                    (pi->v[2] - pj->v[2]) * dx[2];
  const real dvdr_Hubble = dvdr + a2_Hubble * r2;
  const real omega_ij = rmin(dvdr_Hubble, (real)0);
  const real mu_ij = fac_mu * r_inv * omega_ij;
  const real v_sig = signal_velocity(pi, pj, mu_ij, (real)const_viscosity_beta);
  const real f_ij = (real)1 - pi->force.f / mj;
  const real f_ji = (real)1 - pj->force.f / mi;
  const real balsara_i = pi->force.balsara, balsara_j = pj->force.balsara;
  const real rho_ij = rhoi + rhoj;
  const real alpha = pi->viscosity.alpha + pj->viscosity.alpha;
  const real visc =
      (real)-0.25f * alpha * v_sig * mu_ij * (balsara_i + balsara_j) / rho_ij;
  const real visc_acc_term = (real)0.5f * visc * (wi_dr * f_ij + wj_dr * f_ji) * r_inv;
  const real P_over_rho2_i = pressurei / (rhoi * rhoi) * f_ij;
  const real P_over_rho2_j = pressurej / (rhoj * rhoj) * f_ji;
  const real sph_acc_term = (P_over_rho2_i * wi_dr + P_over_rho2_j * wj_dr) * r_inv;
  const real acc = sph_acc_term + visc_acc_term;
  pi->a_hydro[0] -= mj * acc * dx[0];
  pi->a_hydro[1] -= mj * acc * dx[1];
  pi->a_hydro[2] -= mj * acc * dx[2];
  pj->a_hydro[0] += mi * acc * dx[0];
  pj->a_hydro[1] += mi * acc * dx[1];
  pj->a_hydro[2] += mi * acc * dx[2];
  const real sph_du_term_i = P_over_rho2_i * dvdr * r_inv * wi_dr;
  const real sph_du_term_j = P_over_rho2_j * dvdr * r_inv * wj_dr;
  const real visc_du_term = (real)0.5f * visc_acc_term * dvdr_Hubble;
  const real alpha_diff =
      (pressurei * pi->diffusion.alpha + pressurej * pj->diffusion.alpha) /
      (pressurei + pressurej);
  const real v_diff = alpha_diff * (real)0.5f *
                      (SQRT((real)2.f * FABS(pressurei - pressurej) / rho_ij) +
                       FABS(fac_mu * r_inv * dvdr_Hubble));
  const real diff_du_term =
      v_diff * (pi->u - pj->u) * (f_ij * wi_dr / rhoi + f_ji * wj_dr / rhoj);
  const real du_dt_i = sph_du_term_i + visc_du_term + diff_du_term;
  const real du_dt_j = sph_du_term_j + visc_du_term - diff_du_term;
  pi->u_dt += du_dt_i * mj;
  pj->u_dt += du_dt_j * mi;
  pi->force.h_dt -= mj * dvdr * r_inv / rhoj * wi_dr;
  pj->force.h_dt -= mi * dvdr * r_inv / rhoi * wj_dr;
}

/* hydro_iact.h:488-609 */
static inline void iact_nonsym_force(real r2, const real dx[3], real hi, real hj,
                                     opart *pi, const opart *pj, real a, real H) {
  const real fac_mu = (real)1;
  const real a2_Hubble = a * a * H;
  const real r = SQRT(r2);
  const real r_inv = r ? (real)1 / r : (real)0;
  const real mi = pi->mass, mj = pj->mass;
  const real rhoi = pi->rho, rhoj = pj->rho;
  const real pressurei = pi->force.pressure, pressurej = pj->force.pressure;
  const real hi_inv = (real)1 / hi;
  const real hid_inv = pow_dimension_plus_one(hi_inv);
  const real xi = r * hi_inv;
  real wi, wi_dx;
  kernel_deval(xi, &wi, &wi_dx);
  const real wi_dr = hid_inv * wi_dx;
  const real hj_inv = (real)1 / hj;
  const real hjd_inv = pow_dimension_plus_one(hj_inv);
  const real xj = r * hj_inv;
  real wj, wj_dx;
  kernel_deval(xj, &wj, &wj_dx);
  const real wj_dr = hjd_inv * wj_dx;
  const real dvdr = (pi->v[0] - pj->v[0]) * dx[0] + (pi->v[1] - pj->v[1]) * dx[1] +
                    (pi->v[2] - pj->v[2]) * dx[2];
  const real dvdr_Hubble = dvdr + a2_Hubble * r2;
  const real omega_ij = rmin(dvdr_Hubble, (real)0);
  const real mu_ij = fac_mu * r_inv * omega_ij;
  const real v_sig = signal_velocity(pi, pj, mu_ij, (real)const_viscosity_beta);
  const real f_ij = (real)1 - pi->force.f / mj;
  const real f_ji = (real)1 - pj->force.f / mi;
  const real balsara_i = pi->force.balsara, balsara_j = pj->force.balsara;
  const real rho_ij = rhoi + rhoj;
  const real alpha = pi->viscosity.alpha + pj->viscosity.alpha;
  const real visc =
      (real)-0.25f * alpha * v_sig * mu_ij * (balsara_i + balsara_j) / rho_ij;
  const real visc_acc_term = (real)0.5f * visc * (wi_dr * f_ij + wj_dr * f_ji) * r_inv;
  const real P_over_rho2_i = pressurei / (rhoi * rhoi) * f_ij;
  const real P_over_rho2_j = pressurej / (rhoj * rhoj) * f_ji;
  const real sph_acc_term = (P_over_rho2_i * wi_dr + P_over_rho2_j * wj_dr) * r_inv;
  const real acc = sph_acc_term + visc_acc_term;
  pi->a_hydro[0] -= mj * acc * dx[0];
  pi->a_hydro[1] -= mj * acc * dx[1];
  pi->a_hydro[2] -= mj * acc * dx[2];
  const real sph_du_term_i = P_over_rho2_i * dvdr * r_inv * wi_dr;
  const real visc_du_term = (real)0.5f * visc_acc_term * dvdr_Hubble;
  const real alpha_diff =
      (pressurei * pi->diffusion.alpha + pressurej * pj->diffusion.alpha) /
      (pressurei + pressurej);
  const real v_diff = alpha_diff * (real)0.5f *
                      (SQRT((real)2.f * FABS(pressurei - pressurej) / rho_ij) +
                       FABS(fac_mu * r_inv * dvdr_Hubble));
  const real diff_du_term =
      v_diff * (pi->u - pj->u) * (f_ij * wi_dr / rhoi + f_ji * wj_dr / rhoj);
  const real du_dt_i = sph_du_term_i + visc_du_term + diff_du_term;
  pi->u_dt += du_dt_i * mj;
  pi->force.h_dt -= mj * dvdr * r_inv / rhoj * wi_dr;
}

/* src/timestep_limiter_iact.h:34-66 */
static inline void iact_timebin(opart *pi, opart *pj) {
  if (pj->time_bin > 0 && pj->time_bin < pi->limiter_data.min_ngb_time_bin)
    pi->limiter_data.min_ngb_time_bin = pj->time_bin;
  if (pi->time_bin > 0 && pi->time_bin < pj->limiter_data.min_ngb_time_bin)
    pj->limiter_data.min_ngb_time_bin = pi->time_bin;
}
static inline void iact_nonsym_timebin(opart *pi, const opart *pj) {
  if (pj->time_bin > 0 && pj->time_bin < pi->limiter_data.min_ngb_time_bin)
    pi->limiter_data.min_ngb_time_bin = pj->time_bin;
}

/* Exported single-interaction entry points (testSymmetry-style checks). */
API void PFX(iact_density)(real r2, const real *dx, real hi, real hj, opart *pi,
                           opart *pj, real a, real H) {
  iact_density(r2, dx, hi, hj, pi, pj, a, H);
}
API void PFX(iact_nonsym_density)(real r2, const real *dx, real hi, real hj,
                                  opart *pi, const opart *pj, real a, real H) {
  iact_nonsym_density(r2, dx, hi, hj, pi, pj, a, H);
}
API void PFX(iact_force)(real r2, const real *dx, real hi, real hj, opart *pi,
                         opart *pj, real a, real H) {
  iact_force(r2, dx, hi, hj, pi, pj, a, H);
}
API void PFX(iact_nonsym_force)(real r2, const real *dx, real hi, real hj,
                                opart *pi, const opart *pj, real a, real H) {
  iact_nonsym_force(r2, dx, hi, hj, pi, pj, a, H);
}
API void PFX(iact_gradient)(real r2, const real *dx, real hi, real hj, opart *pi,
                            opart *pj, real a, real H) {
  iact_gradient(r2, dx, hi, hj, pi, pj, a, H);
}
API void PFX(iact_nonsym_gradient)(real r2, const real *dx, real hi, real hj,
                                   opart *pi, const opart *pj, real a, real H) {
  iact_nonsym_gradient(r2, dx, hi, hj, pi, pj, a, H);
}

/* ======================================================================== */
/* Per-particle operations — src/hydro/SPHENIX/hydro.h                      */
/* ======================================================================== */

/* The engine-side scalars the particle ops read (plain POD for ctypes). */
struct oracle_params {
  double a, H, a2_inv, a_factor_sound_speed, a_factor_Balsara_eps;
  double time_base;
  float eta_neighbours, h_tolerance, h_max, h_min;
  int max_smoothing_iterations;
  int use_mass_weighted_num_ngb;
  float visc_alpha, visc_alpha_max, visc_alpha_min, visc_length;
  float diff_alpha, diff_beta, diff_alpha_max, diff_alpha_min;
  int max_active_bin;
  int periodic;
  double dim[3];
  const double *dt_alpha_bins; /* nullable: cosmological dt_alpha per time bin */
};

/* hydro.h:553-566 */
static inline void hydro_init_part(opart *p) {
  p->density.wcount = 0;
  p->density.wcount_dh = 0;
  p->rho = 0;
  p->density.rho_dh = 0;
  p->density.rot_v[0] = 0;
  p->density.rot_v[1] = 0;
  p->density.rot_v[2] = 0;
  p->viscosity.div_v = 0;
  p->diffusion.laplace_u = 0;
}

/* hydro.h:599-630 */
static inline void hydro_end_density(opart *p, const struct oracle_params *P) {
  const real h = p->h;
  const real h_inv = (real)1 / h;
  const real h_inv_dim = pow_dimension(h_inv);
  const real h_inv_dim_plus_one = h_inv_dim * h_inv;
  p->rho += p->mass * (real)kernel_root;
  p->density.rho_dh -= (real)hydro_dimension * p->mass * (real)kernel_root;
  p->density.wcount += (real)kernel_root;
  p->density.wcount_dh -= (real)hydro_dimension * (real)kernel_root;
  p->rho *= h_inv_dim;
  p->density.rho_dh *= h_inv_dim_plus_one;
  p->density.wcount *= h_inv_dim;
  p->density.wcount_dh *= h_inv_dim_plus_one;
  const real rho_inv = (real)1 / p->rho;
  const real a_inv2 = (real)P->a2_inv;
  p->density.rot_v[0] *= h_inv_dim_plus_one * a_inv2 * rho_inv;
  p->density.rot_v[1] *= h_inv_dim_plus_one * a_inv2 * rho_inv;
  p->density.rot_v[2] *= h_inv_dim_plus_one * a_inv2 * rho_inv;
  p->viscosity.div_v *= h_inv_dim_plus_one * rho_inv * a_inv2;
  p->viscosity.div_v += (real)P->H * (real)hydro_dimension;
}

/* src/equation_of_state/ideal_gas/equation_of_state.h:121,164 */
static inline real gas_pressure_from_internal_energy(real density, real u) {
  return (real)hydro_gamma_minus_one * u * density;
}
static inline real gas_soundspeed_from_pressure(real density, real Pr) {
  return SQRT((real)hydro_gamma * Pr / density);
}

/* hydro.h:654-717 */
static inline void hydro_prepare_gradient(opart *p, const struct oracle_params *P) {
  const real fac_B = (real)P->a_factor_Balsara_eps;
  const real curl_v = SQRT(p->density.rot_v[0] * p->density.rot_v[0] +
                           p->density.rot_v[1] * p->density.rot_v[1] +
                           p->density.rot_v[2] * p->density.rot_v[2]);
  const real abs_div_v = FABS(p->viscosity.div_v);
  const real pressure = gas_pressure_from_internal_energy(p->rho, p->u);
  const real soundspeed = gas_soundspeed_from_pressure(p->rho, pressure);
  const real balsara =
      abs_div_v / (abs_div_v + curl_v + (real)0.0001f * soundspeed * fac_B / p->h);
  const real common_factor = p->h * (real)hydro_dimension_inv / p->density.wcount;
  real grad_h_term;
  if (p->h > (real)0.9999f * (real)P->h_max) {
    grad_h_term = 0;
  } else {
    const real grad_W_term = common_factor * p->density.wcount_dh;
    if (grad_W_term < (real)-0.9999f)
      grad_h_term = 0;
    else
      grad_h_term = common_factor * p->density.rho_dh / ((real)1 + grad_W_term);
  }
  p->force.f = grad_h_term;
  p->force.pressure = pressure;
  p->force.soundspeed = soundspeed;
  p->force.balsara = balsara;
}

/* hydro.h:728-733 */
static inline void hydro_reset_gradient(opart *p) {
  p->viscosity.v_sig = (real)2 * p->force.soundspeed;
  p->force.alpha_visc_max_ngb = p->viscosity.alpha;
}

/* hydro.h:745-757 */
static inline void hydro_end_gradient(opart *p) {
  const real h = p->h;
  const real h_inv = (real)1 / h;
  const real h_inv_dim = pow_dimension(h_inv);
  const real h_inv_dim_plus_one = h_inv_dim * h_inv;
  p->diffusion.laplace_u *= (real)2 * h_inv_dim_plus_one;
}

/* hydro.h:774-802 */
static inline void hydro_part_has_no_neighbours(opart *p) {
  const real h = p->h;
  const real h_inv = (real)1 / h;
  const real h_inv_dim = pow_dimension(h_inv);
  p->rho = p->mass * (real)kernel_root * h_inv_dim;
  p->viscosity.v_sig = 0;
  p->density.wcount = (real)kernel_root * h_inv_dim;
  p->density.rho_dh = 0;
  p->density.wcount_dh = 0;
  p->density.rot_v[0] = 0;
  p->density.rot_v[1] = 0;
  p->density.rot_v[2] = 0;
  p->viscosity.div_v = 0;
  p->diffusion.laplace_u = 0;
}

/* hydro.h:823-934 */
static inline void hydro_prepare_force(opart *p, const struct oracle_params *P,
                                       real dt_alpha) {
  const real kernel_support_physical = p->h * (real)P->a * (real)kernel_gamma;
  const real kernel_support_physical_inv = (real)1 / kernel_support_physical;
  const real v_sig_physical = p->viscosity.v_sig * (real)P->a_factor_sound_speed;
  const real pressure = gas_pressure_from_internal_energy(p->rho, p->u);
  const real soundspeed_physical =
      gas_soundspeed_from_pressure(p->rho, pressure) * (real)P->a_factor_sound_speed;
  const real sound_crossing_time_inverse =
      soundspeed_physical * kernel_support_physical_inv;
  const real div_v_dt =
      dt_alpha == (real)0
          ? (real)0
          : (p->viscosity.div_v - p->viscosity.div_v_previous_step) / dt_alpha;
  const real S = p->viscosity.div_v < (real)0
                     ? kernel_support_physical * kernel_support_physical *
                           rmax((real)0, (real)-1 * div_v_dt)
                     : (real)0;
  const real soundspeed_square = soundspeed_physical * soundspeed_physical;
  const real alpha_loc = (real)P->visc_alpha_max * S / (soundspeed_square + S);
  if (alpha_loc > p->viscosity.alpha) {
    p->viscosity.alpha = alpha_loc;
  } else {
    const real timescale_ratio =
        dt_alpha * sound_crossing_time_inverse * (real)P->visc_length;
    p->viscosity.alpha += alpha_loc * timescale_ratio;
    p->viscosity.alpha /= ((real)1 + timescale_ratio);
  }
  p->viscosity.alpha = rmax(p->viscosity.alpha, (real)P->visc_alpha_min);
  p->viscosity.div_v_previous_step = p->viscosity.div_v;
  p->viscosity.div_v_dt = div_v_dt;
  const real diffusion_timescale_physical_inverse =
      v_sig_physical * kernel_support_physical_inv;
  const real sqrt_u_inv = (real)1 / SQRT(p->u);
  real alpha_diff_dt = (real)P->diff_beta * kernel_support_physical *
                       p->diffusion.laplace_u * (real)P->a_factor_sound_speed *
                       sqrt_u_inv * (real)P->a2_inv;
  alpha_diff_dt -= (p->diffusion.alpha - (real)P->diff_alpha_min) *
                   diffusion_timescale_physical_inverse;
  real new_diffusion_alpha = p->diffusion.alpha;
  new_diffusion_alpha += alpha_diff_dt * dt_alpha;
  new_diffusion_alpha = rmax(new_diffusion_alpha, (real)P->diff_alpha_min);
  const real viscous_diffusion_limit =
      (real)P->diff_alpha_max *
      ((real)1 - p->force.alpha_visc_max_ngb / (real)P->visc_alpha_max);
  new_diffusion_alpha = rmin(new_diffusion_alpha, viscous_diffusion_limit);
  p->diffusion.alpha = new_diffusion_alpha;
}

/* hydro.h:944-955 + src/timestep_limiter.h:35-39 */
static inline void hydro_reset_acceleration(opart *p) {
  p->a_hydro[0] = 0;
  p->a_hydro[1] = 0;
  p->a_hydro[2] = 0;
  p->u_dt = 0;
  p->force.h_dt = 0;
}
static inline void timestep_limiter_prepare_force(opart *p) {
  p->limiter_data.min_ngb_time_bin = num_time_bins + 1;
}

/* hydro.h:1080-1084 */
static inline void hydro_end_force(opart *p) {
  p->force.h_dt *= p->h * (real)hydro_dimension_inv;
}

/* src/timeline.h:56-61,91-95: non-cosmological dt of a time-bin */
static inline double get_timestep(timebin_t bin, double time_base) {
  if (bin <= 0) return 0.;
  return (double)(1LL << (bin + 1)) * time_base;
}

/* runner_ghost.c:1038-1046: with cosmology, dt_alpha is the physical time of
 * the bin's step (cosmology_get_delta_time over [ti_begin, ti_begin +
 * ti_step]); the caller tabulates it per bin in P->dt_alpha_bins. */
static inline double dt_alpha_of(timebin_t bin, const struct oracle_params *P) {
  if (P->dt_alpha_bins) return (bin >= 0 && bin <= num_time_bins) ? P->dt_alpha_bins[bin] : 0.;
  return get_timestep(bin, P->time_base);
}

/* ======================================================================== */
/* Grid-gather box loops: for each active i, visit the grid cells that      */
/* overlap [x_i - R, x_i + R] and apply the non-symmetric interaction with  */
/* every in-range j (nearest periodic image, as tools.c pairs_all_* do).    */
/* This is exactly the interaction set of all SWIFT density/force tasks of  */
/* a step (each active i meets every j within H_i, resp. max(H_i, H_j)).    */
/* ======================================================================== */
struct ogrid {
  int cdim[3];
  double w[3];
  int ncell;
  int *start; /* ncell+1 */
  int *index; /* particle indices sorted by cell */
};

/* Non-periodic: positions outside [0, dim) (drifted since the last rebuild)
 * are clamped into the boundary cells, whose extent is then open-ended; the
 * gathers clamp both ends of their cell range the same way. */
static void ogrid_build(struct ogrid *g, const opart *parts, long long N,
                        const double dim[3], double min_width, int periodic) {
  for (int k = 0; k < 3; k++) {
    int c = (int)floor(dim[k] / min_width);
    if (c < 1) c = 1;
    if (c > 256) c = 256;
    g->cdim[k] = c;
    g->w[k] = dim[k] / c;
  }
  g->ncell = g->cdim[0] * g->cdim[1] * g->cdim[2];
  g->start = (int *)calloc((size_t)g->ncell + 1, sizeof(int));
  g->index = (int *)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
  int *cellof = (int *)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
  for (long long i = 0; i < N; i++) {
    int c[3];
    for (int k = 0; k < 3; k++) {
      double xx = parts[i].x[k];
      if (periodic) xx -= floor(xx / dim[k]) * dim[k];
      c[k] = (int)floor(xx / g->w[k]);
      if (c[k] >= g->cdim[k]) c[k] = g->cdim[k] - 1;
      if (c[k] < 0) c[k] = 0;
    }
    cellof[i] = (c[2] * g->cdim[1] + c[1]) * g->cdim[0] + c[0];
    g->start[cellof[i] + 1]++;
  }
  for (int c = 0; c < g->ncell; c++) g->start[c + 1] += g->start[c];
  int *fill = (int *)malloc(sizeof(int) * (size_t)g->ncell);
  memcpy(fill, g->start, sizeof(int) * (size_t)g->ncell);
  for (long long i = 0; i < N; i++) g->index[fill[cellof[i]]++] = (int)i;
  free(fill);
  free(cellof);
}

static void ogrid_free(struct ogrid *g) {
  free(g->start);
  free(g->index);
}

/* Multi-level search structure: the particles are binned by their kernel
 * reach H = gamma h into levels (level L holds H in (H_max 2^-(L+1),
 * H_max 2^-L], the last level everything smaller), each with its own grid of
 * cells about as wide as its largest H (at most 256 per dimension). A gather
 * visits, per level, the cells within its own reach (r < H_i) or within
 * max(H_i, H_max of the level) (force: r < max(H_i, H_j)). The visited set
 * always contains every in-range j, so the interaction set is the one of
 * the single uniform grid; clustered boxes, whose H span decades, then cost
 * O(N n_ngb) instead of O(N n_clump). */
#define OLEV_MAX 8
struct olevels {
  int nlev;
  double hmax[OLEV_MAX]; /* largest H of each level */
  struct ogrid g[OLEV_MAX];
};

static void ogrid_build_sub(struct ogrid *g, const opart *parts, const int *ids, long long n,
                            const double dim[3], double min_width, int periodic) {
  for (int k = 0; k < 3; k++) {
    int c = (int)floor(dim[k] / min_width);
    if (c < 1) c = 1;
    if (c > 256) c = 256;
    g->cdim[k] = c;
    g->w[k] = dim[k] / c;
  }
  g->ncell = g->cdim[0] * g->cdim[1] * g->cdim[2];
  g->start = (int *)calloc((size_t)g->ncell + 1, sizeof(int));
  g->index = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  int *cellof = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  for (long long t = 0; t < n; t++) {
    const opart *p = &parts[ids[t]];
    int c[3];
    for (int k = 0; k < 3; k++) {
      double xx = p->x[k];
      if (periodic) xx -= floor(xx / dim[k]) * dim[k];
      c[k] = (int)floor(xx / g->w[k]);
      if (c[k] >= g->cdim[k]) c[k] = g->cdim[k] - 1;
      if (c[k] < 0) c[k] = 0;
    }
    cellof[t] = (c[2] * g->cdim[1] + c[1]) * g->cdim[0] + c[0];
    g->start[cellof[t] + 1]++;
  }
  for (int c = 0; c < g->ncell; c++) g->start[c + 1] += g->start[c];
  int *fill = (int *)malloc(sizeof(int) * (size_t)g->ncell);
  memcpy(fill, g->start, sizeof(int) * (size_t)g->ncell);
  for (long long t = 0; t < n; t++) g->index[fill[cellof[t]]++] = ids[t];
  free(fill);
  free(cellof);
}

static void olevels_build(struct olevels *L, const opart *parts, long long N,
                          const double dim[3], int periodic) {
  double hmax = 0;
  for (long long i = 0; i < N; i++)
    if (!part_is_inhibited(&parts[i]) && parts[i].h > hmax) hmax = parts[i].h;
  hmax *= kernel_gamma;
  const double dmax = fmax(dim[0], fmax(dim[1], dim[2]));
  if (!(hmax > 0)) hmax = dmax;
  /* levels down to the 256-cell resolution of the box (finer buys nothing) */
  int nlev = 1;
  while (nlev < OLEV_MAX && hmax / (double)(1 << nlev) > dmax / 256.) nlev++;
  L->nlev = nlev;
  long long *cnt = (long long *)calloc(OLEV_MAX, sizeof(long long));
  int *lev = (int *)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
  for (long long i = 0; i < N; i++) {
    lev[i] = -1;
    if (part_is_inhibited(&parts[i])) continue;
    const double H = (double)parts[i].h * kernel_gamma;
    int l = 0;
    while (l < nlev - 1 && H <= hmax / (double)(2 << l)) l++;
    lev[i] = l;
    cnt[l]++;
  }
  int *ids = (int *)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
  for (int l = 0; l < nlev; l++) {
    long long n = 0;
    double hl = 0;
    for (long long i = 0; i < N; i++)
      if (lev[i] == l) {
        ids[n++] = (int)i;
        if (parts[i].h > hl) hl = parts[i].h;
      }
    L->hmax[l] = hl * kernel_gamma;
    ogrid_build_sub(&L->g[l], parts, ids, n, dim, hl > 0 ? hl * kernel_gamma : dmax, periodic);
  }
  free(ids);
  free(lev);
  free(cnt);
}

static void olevels_free(struct olevels *L) {
  for (int l = 0; l < L->nlev; l++) ogrid_free(&L->g[l]);
}

/* src/periodic.h:66-72 */
static inline double nearest(double dx, double box) {
  return ((dx > 0.5 * box) ? (dx - box) : ((dx < -0.5 * box) ? (dx + box) : dx));
}

enum { LOOP_DENSITY = 0, LOOP_GRADIENT = 1, LOOP_FORCE = 2 };

/* Gather for one i over the grid; returns the number of interactions. */
static long long gather_one(opart *parts, const struct ogrid *g, long long i,
                            int loop, double reach, const struct oracle_params *P) {
  opart *pi = &parts[i];
  const real hi = pi->h;
  const real hig2 = hi * hi * (real)kernel_gamma2;
  const real a = (real)P->a, Hc = (real)P->H;
  long long n = 0;
  int lo[3], hi_c[3];
  for (int k = 0; k < 3; k++) {
    double xx = pi->x[k];
    if (P->periodic) xx -= floor(xx / P->dim[k]) * P->dim[k];
    lo[k] = (int)floor((xx - reach) / g->w[k]);
    hi_c[k] = (int)floor((xx + reach) / g->w[k]);
    if (!P->periodic) {
      lo[k] = lo[k] < 0 ? 0 : (lo[k] > g->cdim[k] - 1 ? g->cdim[k] - 1 : lo[k]);
      hi_c[k] = hi_c[k] < 0 ? 0 : (hi_c[k] > g->cdim[k] - 1 ? g->cdim[k] - 1 : hi_c[k]);
    } else if (hi_c[k] - lo[k] + 1 > g->cdim[k]) {
      lo[k] = 0;
      hi_c[k] = g->cdim[k] - 1;
    }
  }
  for (int cz = lo[2]; cz <= hi_c[2]; cz++) {
    const int wz = ((cz % g->cdim[2]) + g->cdim[2]) % g->cdim[2];
    for (int cy = lo[1]; cy <= hi_c[1]; cy++) {
      const int wy = ((cy % g->cdim[1]) + g->cdim[1]) % g->cdim[1];
      for (int cx = lo[0]; cx <= hi_c[0]; cx++) {
        const int wx = ((cx % g->cdim[0]) + g->cdim[0]) % g->cdim[0];
        const int c = (wz * g->cdim[1] + wy) * g->cdim[0] + wx;
        for (int q = g->start[c]; q < g->start[c + 1]; q++) {
          const int j = g->index[q];
          if (j == i) continue;
          opart *pj = &parts[j];
          if (part_is_inhibited(pj)) continue;
          real dx[3];
          real r2 = 0;
          for (int k = 0; k < 3; k++) {
            double d = pi->x[k] - pj->x[k];
            if (P->periodic) d = nearest(d, P->dim[k]);
            dx[k] = (real)d;
            r2 += dx[k] * dx[k];
          }
          const real hj = pj->h;
          if (loop == LOOP_FORCE) {
            const real hjg2 = hj * hj * (real)kernel_gamma2;
            if (r2 < hig2 || r2 < hjg2) {
              iact_nonsym_force(r2, dx, hi, hj, pi, pj, a, Hc);
              iact_nonsym_timebin(pi, pj);
              n++;
            }
          } else if (r2 < hig2) {
            if (loop == LOOP_DENSITY)
              iact_nonsym_density(r2, dx, hi, hj, pi, pj, a, Hc);
            else
              iact_nonsym_gradient(r2, dx, hi, hj, pi, pj, a, Hc);
            n++;
          }
        }
      }
    }
  }
  return n;
}

/* Convert the ABI array to oracle records (no-op view in the f32 build). */
static opart *to_oparts(struct part *parts, long long N, int phase) {
#ifdef ORACLE_F32
  (void)N; (void)phase;
  return parts;
#else
  opart *o = (opart *)malloc(sizeof(opart) * (size_t)(N > 0 ? N : 1));
  for (long long i = 0; i < N; i++) part_to_opart(&parts[i], &o[i], phase);
  return o;
#endif
}
static void from_oparts(opart *o, struct part *parts, long long N, int phase) {
#ifdef ORACLE_F32
  (void)o; (void)parts; (void)N; (void)phase;
#else
  for (long long i = 0; i < N; i++) opart_to_part(&o[i], &parts[i], phase);
  free(o);
#endif
}

static double max_h(const opart *o, long long N) {
  double m = 0;
  for (long long i = 0; i < N; i++)
    if (!part_is_inhibited(&o[i]) && o[i].h > m) m = o[i].h;
  return m;
}

/* Runs one loop over every active particle (subset = NULL) or over the
 * index list `subset`. Per-particle interaction counts go to `counts`
 * (optional). Returns the total number of directed interactions. */
static long long box_loop(opart *o, long long N, const struct oracle_params *P,
                          int loop, const int *subset, long long nsub,
                          int *counts) {
  struct olevels L;
  olevels_build(&L, o, N, P->dim, P->periodic);
  const long long nit = subset ? nsub : N;
  long long total = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : total)
  for (long long t = 0; t < nit; t++) {
    const long long i = subset ? subset[t] : t;
    if (!part_is_active(&o[i], (timebin_t)P->max_active_bin)) continue;
    if (part_is_inhibited(&o[i])) continue;
    const double Hi = (double)o[i].h * kernel_gamma;
    long long n = 0;
    for (int l = 0; l < L.nlev; l++) {
      const double reach = (loop == LOOP_FORCE) ? fmax(Hi, L.hmax[l]) : Hi;
      n += gather_one(o, &L.g[l], i, loop, reach, P);
    }
    if (counts) counts[i] = (int)n;
    total += n;
  }
  olevels_free(&L);
  return total;
}

/* Density loop over a periodic/non-periodic box (hydro_init_part is the
 * caller's job, as in SWIFT where the drift/init precedes the loop). */
API long long PFX(box_density)(struct part *parts, long long N,
                               const struct oracle_params *P, int *counts) {
  opart *o = to_oparts(parts, N, PHASE_DENSITY);
  const long long n = box_loop(o, N, P, LOOP_DENSITY, NULL, 0, counts);
  from_oparts(o, parts, N, PHASE_DENSITY);
  return n;
}

API long long PFX(box_density_subset)(struct part *parts, long long N,
                                      const struct oracle_params *P,
                                      const int *subset, long long nsub) {
  opart *o = to_oparts(parts, N, PHASE_DENSITY);
  const long long n = box_loop(o, N, P, LOOP_DENSITY, subset, nsub, NULL);
  from_oparts(o, parts, N, PHASE_DENSITY);
  return n;
}

API long long PFX(box_gradient)(struct part *parts, long long N,
                                const struct oracle_params *P, int *counts) {
  opart *o = to_oparts(parts, N, PHASE_FORCE);
  const long long n = box_loop(o, N, P, LOOP_GRADIENT, NULL, 0, counts);
  from_oparts(o, parts, N, PHASE_FORCE);
  return n;
}

API long long PFX(box_force)(struct part *parts, long long N,
                             const struct oracle_params *P, int *counts) {
  opart *o = to_oparts(parts, N, PHASE_FORCE);
  const long long n = box_loop(o, N, P, LOOP_FORCE, NULL, 0, counts);
  from_oparts(o, parts, N, PHASE_FORCE);
  return n;
}

API void PFX(init_parts)(struct part *parts, long long N,
                         const struct oracle_params *P) {
  for (long long i = 0; i < N; i++) {
    struct part *p = &parts[i];
    if (p->time_bin > P->max_active_bin) continue;
    p->density.wcount = 0.f;
    p->density.wcount_dh = 0.f;
    p->rho = 0.f;
    p->density.rho_dh = 0.f;
    p->density.rot_v[0] = p->density.rot_v[1] = p->density.rot_v[2] = 0.f;
    p->viscosity.div_v = 0.f;
    p->diffusion.laplace_u = 0.f;
  }
}

/* ------------------------------------------------------------------------ */
/* Ghost: src/runner_ghost.c:1085-1596, SPHENIX branch (EXTRA_HYDRO_LOOP),   */
/* non-cosmological, no mass-weighted neighbour number by default. The      */
/* "subset reruns" of runner_ghost.c:1503-1546 become box_loop(subset).     */
/* Returns the number of iterations; *n_failed = particles not converged.   */
/* ------------------------------------------------------------------------ */
/* The reference keeps struct part in float: between the ghost's passes the
 * density sums and h live in float fields (runner_ghost.c reads p->rho,
 * p->density.wcount, ... and writes p->h). The f64 build keeps its arithmetic
 * in double but rounds those stored values to float at the same points, so a
 * particle whose Newton step lands within float rounding of h_tolerance
 * takes the reference's storage path (identities in the f32 build). */
static inline real fstore(real x) { return (real)(float)x; }
static void store_density_sums(opart *p) {
  p->rho = fstore(p->rho);
  p->density.wcount = fstore(p->density.wcount);
  p->density.wcount_dh = fstore(p->density.wcount_dh);
  p->density.rho_dh = fstore(p->density.rho_dh);
  p->viscosity.div_v = fstore(p->viscosity.div_v);
  for (int k = 0; k < 3; k++) p->density.rot_v[k] = fstore(p->density.rot_v[k]);
}

API int PFX(box_ghost)(struct part *parts, long long N,
                       const struct oracle_params *P, long long *n_failed) {
  opart *o = to_oparts(parts, N, PHASE_DENSITY);
  const real eps = (real)P->h_tolerance;
  const real hydro_h_max = (real)P->h_max, hydro_h_min = (real)P->h_min;
  /* runner_ghost.c:1103-1105: eps and hydro_eta_dim are floats (the f64
   * build keeps the reference's float constants, like the kernel's) */
  const float eta_f = P->eta_neighbours;
  const real hydro_eta_dim = (real)(eta_f * eta_f * eta_f);
  int *pid = (int *)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
  real *left = (real *)malloc(sizeof(real) * (size_t)(N > 0 ? N : 1));
  real *right = (real *)malloc(sizeof(real) * (size_t)(N > 0 ? N : 1));
  long long count = 0;
  for (long long k = 0; k < N; k++)
    if (part_is_active(&o[k], (timebin_t)P->max_active_bin) &&
        !part_is_inhibited(&o[k])) {
      pid[count] = (int)k;
      left[count] = 0;
      right[count] = hydro_h_max;
      count++;
    }
  int num_reruns;
  for (num_reruns = 0; count > 0 && num_reruns < P->max_smoothing_iterations;
       num_reruns++) {
    long long redo = 0;
    for (long long i = 0; i < count; i++) {
      opart *p = &o[pid[i]];
      const real h_old = p->h;
      const real h_old_dim = pow_dimension(h_old);
      const real h_old_dim_minus_one = pow_dimension_minus_one(h_old);
      real h_new;
      int has_no_neighbours = 0;
      int done = 0;
      if (p->density.wcount < (real)(1.e-5 * kernel_root)) {
        has_no_neighbours = 1;
        h_new = (real)2 * h_old;
      } else {
        hydro_end_density(p, P);
        if (P->use_mass_weighted_num_ngb) {
          const real inv_mass = (real)1 / p->mass;
          p->density.wcount = p->rho * inv_mass;
          p->density.wcount_dh = p->density.rho_dh * inv_mass;
        }
        const real n_sum = p->density.wcount * h_old_dim;
        const real n_target = hydro_eta_dim;
        const real f = n_sum - n_target;
        const real f_prime = p->density.wcount_dh * h_old_dim +
                             (real)hydro_dimension * p->density.wcount * h_old_dim_minus_one;
        if (n_sum < n_target)
          left[i] = rmax(left[i], h_old);
        else if (n_sum > n_target)
          right[i] = rmin(right[i], h_old);
        if (((p->h >= hydro_h_max) && (f < (real)0)) ||
            ((p->h <= hydro_h_min) && (f > (real)0))) {
          done = 1; /* converged "by force": tidy up below */
          h_new = h_old;
        } else {
          h_new = h_old - f / (f_prime + (real)FLT_MIN);
          h_new = rmin(h_new, (real)2 * h_old);
          h_new = rmax(h_new, (real)0.5f * h_old);
          h_new = rmax(h_new, left[i]);
          h_new = rmin(h_new, right[i]);
        }
      }
      if (!done && FABS(h_new - h_old) > eps * h_old) {
        if ((h_new == left[i] && h_old == right[i]) ||
            (h_old == left[i] && h_new == right[i])) {
#ifdef ORACLE_F32
          p->h = cbrtf(0.5f * (pow_dimension(left[i]) + pow_dimension(right[i])));
#else
          p->h = fstore(cbrt(0.5 * (pow_dimension(left[i]) + pow_dimension(right[i]))));
#endif
        } else {
          p->h = fstore(h_new);
        }
        if (p->h < hydro_h_max && p->h > hydro_h_min) {
          pid[redo] = pid[i];
          left[redo] = left[i];
          right[redo] = right[i];
          redo++;
          hydro_init_part(p);
          continue;
        } else if (p->h <= hydro_h_min) {
          p->h = hydro_h_min;
        } else if (p->h >= hydro_h_max) {
          p->h = hydro_h_max;
          if (has_no_neighbours) hydro_part_has_no_neighbours(p);
        }
      }
      /* converged: prepare for the gradient loop (EXTRA_HYDRO_LOOP) */
      hydro_prepare_gradient(p, P);
      hydro_reset_gradient(p);
    }
    count = redo;
    if (count > 0) {
      box_loop(o, N, P, LOOP_DENSITY, pid, count, NULL);
      for (long long i = 0; i < count; i++) store_density_sums(&o[pid[i]]);
    }
  }
  if (n_failed) *n_failed = count;
  free(pid);
  free(left);
  free(right);
  /* After the ghost the force-side union members are live. */
  from_oparts(o, parts, N, PHASE_FORCE);
  return num_reruns;
}

/* runner_ghost.c:992-1083 (extra ghost) for every active particle */
API void PFX(box_extra_ghost)(struct part *parts, long long N,
                              const struct oracle_params *P) {
  opart *o = to_oparts(parts, N, PHASE_FORCE);
  for (long long i = 0; i < N; i++) {
    opart *p = &o[i];
    if (!part_is_active(p, (timebin_t)P->max_active_bin)) continue;
    hydro_end_gradient(p);
    const real dt_alpha = (real)dt_alpha_of(p->time_bin, P);
    hydro_prepare_force(p, P, dt_alpha);
    timestep_limiter_prepare_force(p);
    hydro_reset_acceleration(p);
  }
  from_oparts(o, parts, N, PHASE_FORCE);
}

/* Drift of every non-inhibited particle: drift_part (src/drift.h:143-232)
 * with SPHENIX hydro_predict_extra (src/hydro/SPHENIX/hydro.h:1012-1066),
 * entropy and pressure floors NONE, EOS_IDEAL_GAS. Float fields in float, as
 * the reference (both builds: the drift has no reduction). has_gpart[i]:
 * the part has a gpart (gravity kick). */
struct oracle_drift_params {
  double dt_drift, dt_kick_hydro, dt_kick_grav, dt_therm;
  float min_u;
};

static float approx_expf_o(float x) {  /* src/approx_math.h:35 */
  return 1.f + x * (1.f + x * (0.5f + x * (1.f / 6.f + 1.f / 24.f * x)));
}

API void PFX(box_drift)(struct part *parts, struct xpart *xparts, const char *has_gpart,
                        long long N, const struct oracle_drift_params *D) {
  for (long long i = 0; i < N; i++) {
    struct part *p = &parts[i];
    struct xpart *xp = &xparts[i];
    if (p->time_bin == time_bin_inhibited) continue;
    p->x[0] += xp->v_full[0] * D->dt_drift;
    p->x[1] += xp->v_full[1] * D->dt_drift;
    p->x[2] += xp->v_full[2] * D->dt_drift;
    p->v[0] += p->a_hydro[0] * D->dt_kick_hydro;
    p->v[1] += p->a_hydro[1] * D->dt_kick_hydro;
    p->v[2] += p->a_hydro[2] * D->dt_kick_hydro;
    if (has_gpart && has_gpart[i]) {
      p->v[0] += xp->a_grav[0] * D->dt_kick_grav;
      p->v[1] += xp->a_grav[1] * D->dt_kick_grav;
      p->v[2] += xp->a_grav[2] * D->dt_kick_grav;
    }
    /* hydro_predict_extra(p, xp, (float)dt_drift, (float)dt_therm, ...) */
    const float dt_drift = (float)D->dt_drift, dt_therm = (float)D->dt_therm;
    p->u += p->u_dt * dt_therm;
    const float h_inv = 1.f / p->h;
    const float w1 = p->force.h_dt * h_inv * dt_drift;
    if (fabsf(w1) < 0.2f)
      p->h *= approx_expf_o(w1);
    else
      p->h *= expf(w1);
    const float w2 = -3.f * w1;
    if (fabsf(w2) < 0.2f)
      p->rho *= approx_expf_o(w2);
    else
      p->rho *= expf(w2);
    const float floor_u = 0.f; /* entropy_floor NONE */
    p->u = p->u > floor_u ? p->u : floor_u;
    p->u = p->u > D->min_u ? p->u : D->min_u;
    const float pressure = hydro_gamma_minus_one * p->u * p->rho;
    const float soundspeed = sqrtf(hydro_gamma * pressure / p->rho);
    p->force.pressure = pressure;
    p->force.soundspeed = soundspeed;
    p->viscosity.v_sig = p->viscosity.v_sig > 2.f * soundspeed ? p->viscosity.v_sig
                                                               : 2.f * soundspeed;
    for (int k = 0; k < 3; k++) {
      const float dx = xp->v_full[k] * D->dt_drift;
      xp->x_diff[k] -= dx;
      xp->x_diff_sort[k] -= dx;
    }
  }
}

/* src/runner_others.c:618 -> hydro_end_force */
API void PFX(box_end_force)(struct part *parts, long long N,
                            const struct oracle_params *P) {
  opart *o = to_oparts(parts, N, PHASE_FORCE);
  for (long long i = 0; i < N; i++)
    if (part_is_active(&o[i], (timebin_t)P->max_active_bin)) hydro_end_force(&o[i]);
  from_oparts(o, parts, N, PHASE_FORCE);
}

/* Exact count of directed in-range pairs (density: r < H_i; force:
 * r < max(H_i, H_j)), active i only. Used as the metric's denominator. */
API long long PFX(box_count_pairs)(struct part *parts, long long N,
                                   const struct oracle_params *P, int force) {
  opart *o = to_oparts(parts, N, PHASE_DENSITY);
  const double hmax = max_h(o, N) * kernel_gamma;
  struct ogrid g;
  ogrid_build(&g, o, N, P->dim, hmax > 0 ? hmax : P->dim[0], P->periodic);
  long long total = 0;
#pragma omp parallel for schedule(dynamic, 1024) reduction(+ : total)
  for (long long i = 0; i < N; i++) {
    const opart *pi = &o[i];
    if (!part_is_active(pi, (timebin_t)P->max_active_bin)) continue;
    const real hig2 = pi->h * pi->h * (real)kernel_gamma2;
    const double reach = force ? hmax : (double)pi->h * kernel_gamma;
    int lo[3], hc[3];
    for (int k = 0; k < 3; k++) {
      double xx = pi->x[k];
      if (P->periodic) xx -= floor(xx / P->dim[k]) * P->dim[k];
      lo[k] = (int)floor((xx - reach) / g.w[k]);
      hc[k] = (int)floor((xx + reach) / g.w[k]);
      if (!P->periodic) {
        lo[k] = lo[k] < 0 ? 0 : (lo[k] > g.cdim[k] - 1 ? g.cdim[k] - 1 : lo[k]);
        hc[k] = hc[k] < 0 ? 0 : (hc[k] > g.cdim[k] - 1 ? g.cdim[k] - 1 : hc[k]);
      } else if (hc[k] - lo[k] + 1 > g.cdim[k]) {
        lo[k] = 0;
        hc[k] = g.cdim[k] - 1;
      }
    }
    for (int cz = lo[2]; cz <= hc[2]; cz++)
      for (int cy = lo[1]; cy <= hc[1]; cy++)
        for (int cx = lo[0]; cx <= hc[0]; cx++) {
          const int c = ((((cz % g.cdim[2]) + g.cdim[2]) % g.cdim[2]) * g.cdim[1] +
                         (((cy % g.cdim[1]) + g.cdim[1]) % g.cdim[1])) * g.cdim[0] +
                        (((cx % g.cdim[0]) + g.cdim[0]) % g.cdim[0]);
          for (int q = g.start[c]; q < g.start[c + 1]; q++) {
            const int j = g.index[q];
            if (j == i) continue;
            const opart *pj = &o[j];
            real r2 = 0;
            for (int k = 0; k < 3; k++) {
              double d = pi->x[k] - pj->x[k];
              if (P->periodic) d = nearest(d, P->dim[k]);
              const real dd = (real)d;
              r2 += dd * dd;
            }
            const real hjg2 = pj->h * pj->h * (real)kernel_gamma2;
            if (r2 < hig2 || (force && r2 < hjg2)) total++;
          }
        }
  }
  ogrid_free(&g);
#ifndef ORACLE_F32
  free(o);
#endif
  return total;
}

#ifdef ORACLE_F32
/* ======================================================================== */
/* Cell-task loops (faithful float restatement of                          */
/* src/runner_doiact_functions_hydro.h). These operate on SWIFT-style cells */
/* (include/swift_compat.h) exactly as the runner does, including sorted    */
/* pseudo-Verlet windows, activity masks and the ci/cj swap of              */
/* space_getsid.                                                            */
/* ======================================================================== */

/* src/sort_part.h:42-92 */
static const double runner_shift[13][3] = {
    {5.773502691896258e-01, 5.773502691896258e-01, 5.773502691896258e-01},
    {7.071067811865475e-01, 7.071067811865475e-01, 0.0},
    {5.773502691896258e-01, 5.773502691896258e-01, -5.773502691896258e-01},
    {7.071067811865475e-01, 0.0, 7.071067811865475e-01},
    {1.0, 0.0, 0.0},
    {7.071067811865475e-01, 0.0, -7.071067811865475e-01},
    {5.773502691896258e-01, -5.773502691896258e-01, 5.773502691896258e-01},
    {7.071067811865475e-01, -7.071067811865475e-01, 0.0},
    {5.773502691896258e-01, -5.773502691896258e-01, -5.773502691896258e-01},
    {0.0, 7.071067811865475e-01, 7.071067811865475e-01},
    {0.0, 1.0, 0.0},
    {0.0, 7.071067811865475e-01, -7.071067811865475e-01},
    {0.0, 0.0, 1.0},
};
static const int runner_flip[27] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static const int sortlistID[27] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 0,
                                   12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};
#define space_maxreldx 0.1f /* src/space.h:66 */

static int cmp_sort_entry(const void *a, const void *b) {
  const struct sort_entry *x = (const struct sort_entry *)a;
  const struct sort_entry *y = (const struct sort_entry *)b;
  if (x->d < y->d) return -1;
  if (x->d > y->d) return 1;
  return (x->i < y->i) ? -1 : (x->i > y->i);
}

/* src/runner_sort.c:352-391 (leaf branch): project on the 13 axes, add the
 * FLT_MAX sentinel, sort ascending. Storage: caller-owned per-cell lists. */
API void orf_cell_sort(struct cell *c, int flags) {
  const int count = c->hydro.count;
  for (int j = 0; j < 13; j++) {
    if (!(flags & (1 << j))) continue;
    if (c->hydro.sort[j] == NULL)
      c->hydro.sort[j] =
          (struct sort_entry *)malloc(sizeof(struct sort_entry) * (size_t)(count + 1));
    struct sort_entry *e = c->hydro.sort[j];
    for (int k = 0; k < count; k++) {
      const double *px = c->hydro.parts[k].x;
      e[k].i = k;
      e[k].d = px[0] * runner_shift[j][0] + px[1] * runner_shift[j][1] +
               px[2] * runner_shift[j][2];
    }
    e[count].d = FLT_MAX;
    e[count].i = 0;
    qsort(e, (size_t)count, sizeof(struct sort_entry), cmp_sort_entry);
    c->hydro.sorted |= (uint16_t)(1 << j);
  }
  c->hydro.dx_max_sort = 0.f;
  c->hydro.dx_max_sort_old = 0.f;
}

API void orf_cell_free_sorts(struct cell *c) {
  for (int j = 0; j < 13; j++) {
    free(c->hydro.sort[j]);
    c->hydro.sort[j] = NULL;
  }
  c->hydro.sorted = 0;
}

/* src/space_getsid.h:46-82 */
static int space_getsid(const struct space *s, struct cell **ci, struct cell **cj,
                        double shift[3]) {
  const int periodic = s->periodic;
  double dx[3];
  for (int k = 0; k < 3; k++) {
    dx[k] = (*cj)->loc[k] - (*ci)->loc[k];
    if (periodic && dx[k] < -s->dim[k] / 2)
      shift[k] = s->dim[k];
    else if (periodic && dx[k] > s->dim[k] / 2)
      shift[k] = -s->dim[k];
    else
      shift[k] = 0.0;
    dx[k] += shift[k];
  }
  int sid = 0;
  for (int k = 0; k < 3; k++)
    sid = 3 * sid + ((dx[k] < 0.0) ? 0 : ((dx[k] > 0.0) ? 2 : 1));
  if (runner_flip[sid]) {
    struct cell *temp = *ci;
    *ci = *cj;
    *cj = temp;
    for (int k = 0; k < 3; k++) shift[k] = -shift[k];
  }
  return sortlistID[sid];
}

static inline int cell_is_active_hydro(const struct cell *c, const struct engine *e) {
  return c->hydro.ti_end_min == e->ti_current; /* src/active.h:176-190 */
}

#define PA(p) part_is_active((p), e->max_active_bin)

/* DOPAIR1, runner_doiact_functions_hydro.h:1068-1320; loop = density or
 * gradient (both use the r < H_i criterion). */
static void dopair1(const struct engine *e, struct cell *ci, struct cell *cj,
                    const int sid, const double *shift, int loop) {
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  double rshift = 0.0;
  for (int k = 0; k < 3; k++) rshift += shift[k] * runner_shift[sid][k];
  const struct sort_entry *sort_i = cell_get_hydro_sorts(ci, sid);
  const struct sort_entry *sort_j = cell_get_hydro_sorts(cj, sid);
  const double hi_max = ci->hydro.h_max * kernel_gamma - rshift;
  const double hj_max = cj->hydro.h_max * kernel_gamma;
  const int count_i = ci->hydro.count, count_j = cj->hydro.count;
  struct part *parts_i = ci->hydro.parts, *parts_j = cj->hydro.parts;
  const double di_max = sort_i[count_i - 1].d - rshift;
  const double dj_min = sort_j[0].d;
  const float dx_max = (ci->hydro.dx_max_sort + cj->hydro.dx_max_sort);

  if (cell_is_active_hydro(ci, e)) {
    for (int pid = count_i - 1;
         pid >= 0 && sort_i[pid].d + hi_max + dx_max > dj_min; pid--) {
      struct part *pi = &parts_i[sort_i[pid].i];
      const float hi = pi->h;
      if (!PA(pi)) continue;
      const double di = sort_i[pid].d + hi * kernel_gamma + dx_max - rshift;
      if (di < dj_min) continue;
      const float hig2 = hi * hi * kernel_gamma2;
      const float pix = pi->x[0] - (cj->loc[0] + shift[0]);
      const float piy = pi->x[1] - (cj->loc[1] + shift[1]);
      const float piz = pi->x[2] - (cj->loc[2] + shift[2]);
      for (int pjd = 0; pjd < count_j && sort_j[pjd].d < di; pjd++) {
        struct part *pj = &parts_j[sort_j[pjd].i];
        if (part_is_inhibited(pj)) continue;
        const float hj = pj->h;
        const float pjx = pj->x[0] - cj->loc[0];
        const float pjy = pj->x[1] - cj->loc[1];
        const float pjz = pj->x[2] - cj->loc[2];
        float dx[3] = {pix - pjx, piy - pjy, piz - pjz};
        const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        if (r2 < hig2) {
          if (loop == LOOP_DENSITY)
            iact_nonsym_density(r2, dx, hi, hj, pi, pj, a, H);
          else
            iact_nonsym_gradient(r2, dx, hi, hj, pi, pj, a, H);
        }
      }
    }
  }
  if (cell_is_active_hydro(cj, e)) {
    for (int pjd = 0; pjd < count_j && sort_j[pjd].d - hj_max - dx_max < di_max;
         pjd++) {
      struct part *pj = &parts_j[sort_j[pjd].i];
      const float hj = pj->h;
      if (!PA(pj)) continue;
      const double dj = sort_j[pjd].d - hj * kernel_gamma - dx_max + rshift;
      if (dj - rshift > di_max) continue;
      const float hjg2 = hj * hj * kernel_gamma2;
      const float pjx = pj->x[0] - cj->loc[0];
      const float pjy = pj->x[1] - cj->loc[1];
      const float pjz = pj->x[2] - cj->loc[2];
      for (int pid = count_i - 1; pid >= 0 && sort_i[pid].d > dj; pid--) {
        struct part *pi = &parts_i[sort_i[pid].i];
        if (part_is_inhibited(pi)) continue;
        const float hi = pi->h;
        const float pix = pi->x[0] - (cj->loc[0] + shift[0]);
        const float piy = pi->x[1] - (cj->loc[1] + shift[1]);
        const float piz = pi->x[2] - (cj->loc[2] + shift[2]);
        float dx[3] = {pjx - pix, pjy - piy, pjz - piz};
        const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        if (r2 < hjg2) {
          if (loop == LOOP_DENSITY)
            iact_nonsym_density(r2, dx, hj, hi, pj, pi, a, H);
          else
            iact_nonsym_gradient(r2, dx, hj, hi, pj, pi, a, H);
        }
      }
    }
  }
}

/* DOSELF1, runner_doiact_functions_hydro.h:2062-2261 */
static void doself1(const struct engine *e, struct cell *c, int loop) {
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  struct part *parts = c->hydro.parts;
  const int count = c->hydro.count;
  int *indt = (int *)malloc(sizeof(int) * (size_t)(count > 0 ? count : 1));
  int countdt = 0, firstdt = 0;
  for (int k = 0; k < count; k++)
    if (PA(&parts[k])) indt[countdt++] = k;
  for (int pid = 0; pid < count; pid++) {
    struct part *pi = &parts[pid];
    if (part_is_inhibited(pi)) continue;
    double pix[3];
    for (int k = 0; k < 3; k++) pix[k] = pi->x[k];
    const float hi = pi->h;
    const float hig2 = hi * hi * kernel_gamma2;
    if (!PA(pi)) {
      for (int pjd = firstdt; pjd < countdt; pjd++) {
        struct part *pj = &parts[indt[pjd]];
        const float hj = pj->h;
        float r2 = 0.0f;
        float dx[3];
        for (int k = 0; k < 3; k++) {
          dx[k] = pj->x[k] - pix[k];
          r2 += dx[k] * dx[k];
        }
        if (r2 < hj * hj * kernel_gamma2) {
          if (loop == LOOP_DENSITY)
            iact_nonsym_density(r2, dx, hj, hi, pj, pi, a, H);
          else
            iact_nonsym_gradient(r2, dx, hj, hi, pj, pi, a, H);
        }
      }
    } else {
      firstdt += 1;
      for (int pjd = pid + 1; pjd < count; pjd++) {
        struct part *pj = &parts[pjd];
        if (part_is_inhibited(pj)) continue;
        const float hj = pj->h;
        float r2 = 0.0f;
        float dx[3];
        for (int k = 0; k < 3; k++) {
          dx[k] = pix[k] - pj->x[k];
          r2 += dx[k] * dx[k];
        }
        const int doj = (PA(pj)) && (r2 < hj * hj * kernel_gamma2);
        const int doi = (r2 < hig2);
        if (doi || doj) {
          if (doi && doj) {
            if (loop == LOOP_DENSITY)
              iact_density(r2, dx, hi, hj, pi, pj, a, H);
            else
              iact_gradient(r2, dx, hi, hj, pi, pj, a, H);
          } else if (doi) {
            if (loop == LOOP_DENSITY)
              iact_nonsym_density(r2, dx, hi, hj, pi, pj, a, H);
            else
              iact_nonsym_gradient(r2, dx, hi, hj, pi, pj, a, H);
          } else if (doj) {
            dx[0] = -dx[0];
            dx[1] = -dx[1];
            dx[2] = -dx[2];
            if (loop == LOOP_DENSITY)
              iact_nonsym_density(r2, dx, hj, hi, pj, pi, a, H);
            else
              iact_nonsym_gradient(r2, dx, hj, hi, pj, pi, a, H);
          }
        }
      }
    }
  }
  free(indt);
}

/* DOPAIR2, runner_doiact_functions_hydro.h:1424-1961 (force) */
static void dopair2(const struct engine *e, struct cell *ci, struct cell *cj,
                    const int sid, const double *shift) {
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  double rshift = 0.0;
  for (int k = 0; k < 3; k++) rshift += shift[k] * runner_shift[sid][k];
  struct sort_entry *sort_i = cell_get_hydro_sorts(ci, sid);
  struct sort_entry *sort_j = cell_get_hydro_sorts(cj, sid);
  const double hi_max = ci->hydro.h_max, hj_max = cj->hydro.h_max;
  const int count_i = ci->hydro.count, count_j = cj->hydro.count;
  struct part *parts_i = ci->hydro.parts, *parts_j = cj->hydro.parts;
  const double dx_max = (ci->hydro.dx_max_sort + cj->hydro.dx_max_sort);
  const double di_max = sort_i[count_i - 1].d;
  const double dj_min = sort_j[0].d;
  const double shift_i[3] = {cj->loc[0] + shift[0], cj->loc[1] + shift[1],
                             cj->loc[2] + shift[2]};
  const double shift_j[3] = {cj->loc[0], cj->loc[1], cj->loc[2]};
  int count_active_i = 0, count_active_j = 0;
  struct sort_entry *sort_active_i = NULL, *sort_active_j = NULL;
  if (cell_is_active_hydro(ci, e)) {
    sort_active_i = (struct sort_entry *)malloc(sizeof(struct sort_entry) * (size_t)count_i);
    for (int k = 0; k < count_i; k++)
      if (PA(&parts_i[sort_i[k].i])) sort_active_i[count_active_i++] = sort_i[k];
  }
  if (cell_is_active_hydro(cj, e)) {
    sort_active_j = (struct sort_entry *)malloc(sizeof(struct sort_entry) * (size_t)count_j);
    for (int k = 0; k < count_j; k++)
      if (PA(&parts_j[sort_j[k].i])) sort_active_j[count_active_j++] = sort_j[k];
  }
  for (int pid = count_i - 1;
       pid >= 0 && sort_i[pid].d + hi_max * kernel_gamma + dx_max - rshift > dj_min;
       pid--) {
    struct part *pi = &parts_i[sort_i[pid].i];
    if (part_is_inhibited(pi)) continue;
    const float hi = pi->h;
    const double di = sort_i[pid].d + hi * kernel_gamma + dx_max - rshift;
    if (di < dj_min) continue;
    const float hig2 = hi * hi * kernel_gamma2;
    const float pix = pi->x[0] - shift_i[0];
    const float piy = pi->x[1] - shift_i[1];
    const float piz = pi->x[2] - shift_i[2];
    if (!PA(pi)) {
      for (int pjd = 0; pjd < count_active_j && sort_active_j[pjd].d < di; pjd++) {
        struct part *pj = &parts_j[sort_active_j[pjd].i];
        if (part_is_inhibited(pj)) continue;
        const float hj = pj->h;
        const float pjx = pj->x[0] - shift_j[0];
        const float pjy = pj->x[1] - shift_j[1];
        const float pjz = pj->x[2] - shift_j[2];
        const float dx[3] = {pjx - pix, pjy - piy, pjz - piz};
        const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        if (r2 < hig2) {
          iact_nonsym_force(r2, dx, hj, hi, pj, pi, a, H);
          iact_nonsym_timebin(pj, pi);
        }
      }
    } else {
      for (int pjd = 0; pjd < count_j && sort_j[pjd].d < di; pjd++) {
        struct part *pj = &parts_j[sort_j[pjd].i];
        if (part_is_inhibited(pj)) continue;
        const float hj = pj->h;
        const float pjx = pj->x[0] - shift_j[0];
        const float pjy = pj->x[1] - shift_j[1];
        const float pjz = pj->x[2] - shift_j[2];
        const float dx[3] = {pix - pjx, piy - pjy, piz - pjz};
        const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        if (r2 < hig2) {
          if (PA(pj)) {
            iact_force(r2, dx, hi, hj, pi, pj, a, H);
            iact_timebin(pi, pj);
          } else {
            iact_nonsym_force(r2, dx, hi, hj, pi, pj, a, H);
            iact_nonsym_timebin(pi, pj);
          }
        }
      }
    }
  }
  for (int pjd = 0;
       pjd < count_j && sort_j[pjd].d - hj_max * kernel_gamma - dx_max < di_max - rshift;
       pjd++) {
    struct part *pj = &parts_j[sort_j[pjd].i];
    if (part_is_inhibited(pj)) continue;
    const float hj = pj->h;
    const double dj = sort_j[pjd].d - hj * kernel_gamma - dx_max;
    if (dj > di_max - rshift) continue;
    const float hjg2 = hj * hj * kernel_gamma2;
    const float pjx = pj->x[0] - shift_j[0];
    const float pjy = pj->x[1] - shift_j[1];
    const float pjz = pj->x[2] - shift_j[2];
    if (!PA(pj)) {
      for (int pid = count_active_i - 1;
           pid >= 0 && sort_active_i[pid].d - rshift > dj; pid--) {
        struct part *pi = &parts_i[sort_active_i[pid].i];
        if (part_is_inhibited(pi)) continue;
        const float hi = pi->h;
        const float hig2 = hi * hi * kernel_gamma2;
        const float pix = pi->x[0] - shift_i[0];
        const float piy = pi->x[1] - shift_i[1];
        const float piz = pi->x[2] - shift_i[2];
        const float dx[3] = {pix - pjx, piy - pjy, piz - pjz};
        const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        if (r2 < hjg2 && r2 >= hig2) {
          iact_nonsym_force(r2, dx, hi, hj, pi, pj, a, H);
          iact_nonsym_timebin(pi, pj);
        }
      }
    } else {
      for (int pid = count_i - 1; pid >= 0 && sort_i[pid].d - rshift > dj; pid--) {
        struct part *pi = &parts_i[sort_i[pid].i];
        if (part_is_inhibited(pi)) continue;
        const float hi = pi->h;
        const float hig2 = hi * hi * kernel_gamma2;
        const float pix = pi->x[0] - shift_i[0];
        const float piy = pi->x[1] - shift_i[1];
        const float piz = pi->x[2] - shift_i[2];
        const float dx[3] = {pjx - pix, pjy - piy, pjz - piz};
        const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        if (r2 < hjg2 && r2 >= hig2) {
          if (PA(pi)) {
            iact_force(r2, dx, hj, hi, pj, pi, a, H);
            iact_timebin(pj, pi);
          } else {
            iact_nonsym_force(r2, dx, hj, hi, pj, pi, a, H);
            iact_nonsym_timebin(pj, pi);
          }
        }
      }
    }
  }
  free(sort_active_i);
  free(sort_active_j);
}

/* DOSELF2, runner_doiact_functions_hydro.h:2304-2476 (force) */
static void doself2(const struct engine *e, struct cell *c) {
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  struct part *parts = c->hydro.parts;
  const int count = c->hydro.count;
  int *indt = (int *)malloc(sizeof(int) * (size_t)(count > 0 ? count : 1));
  int countdt = 0, firstdt = 0;
  for (int k = 0; k < count; k++)
    if (PA(&parts[k])) indt[countdt++] = k;
  for (int pid = 0; pid < count; pid++) {
    struct part *pi = &parts[pid];
    if (part_is_inhibited(pi)) continue;
    double pix[3];
    for (int k = 0; k < 3; k++) pix[k] = pi->x[k];
    const float hi = pi->h;
    const float hig2 = hi * hi * kernel_gamma2;
    if (!PA(pi)) {
      for (int pjd = firstdt; pjd < countdt; pjd++) {
        struct part *pj = &parts[indt[pjd]];
        const float hj = pj->h;
        float r2 = 0.0f;
        float dx[3];
        for (int k = 0; k < 3; k++) {
          dx[k] = pj->x[k] - pix[k];
          r2 += dx[k] * dx[k];
        }
        if (r2 < hig2 || r2 < hj * hj * kernel_gamma2) {
          iact_nonsym_force(r2, dx, hj, hi, pj, pi, a, H);
          iact_nonsym_timebin(pj, pi);
        }
      }
    } else {
      firstdt += 1;
      for (int pjd = pid + 1; pjd < count; pjd++) {
        struct part *pj = &parts[pjd];
        if (part_is_inhibited(pj)) continue;
        const float hj = pj->h;
        float r2 = 0.0f;
        float dx[3];
        for (int k = 0; k < 3; k++) {
          dx[k] = pix[k] - pj->x[k];
          r2 += dx[k] * dx[k];
        }
        if (r2 < hig2 || r2 < hj * hj * kernel_gamma2) {
          if (PA(pj)) {
            iact_force(r2, dx, hi, hj, pi, pj, a, H);
            iact_timebin(pi, pj);
          } else {
            iact_nonsym_force(r2, dx, hi, hj, pi, pj, a, H);
            iact_nonsym_timebin(pi, pj);
          }
        }
      }
    }
  }
  free(indt);
}

static int check_pair(const struct engine *e, struct cell **ci, struct cell **cj,
                      double shift[3], int *sid) {
  if ((*ci)->hydro.count == 0 || (*cj)->hydro.count == 0) return 0;
  if (!cell_is_active_hydro(*ci, e) && !cell_is_active_hydro(*cj, e)) return 0;
  *sid = space_getsid(e->s, ci, cj, shift);
  if (!((*ci)->hydro.sorted & (1 << *sid)) ||
      (*ci)->hydro.dx_max_sort_old > space_maxreldx * (*ci)->dmin)
    return -1;
  if (!((*cj)->hydro.sorted & (1 << *sid)) ||
      (*cj)->hydro.dx_max_sort_old > space_maxreldx * (*cj)->dmin)
    return -1;
  return 1;
}

/* DOPAIR1_BRANCH, runner_doiact_functions_hydro.h:1331-1413. Returns 0 on
 * success, -1 for "Interacting unsorted cells". */
API int orf_dopair1_branch(struct runner *r, struct cell *ci, struct cell *cj,
                           int loop) {
  double shift[3] = {0.0, 0.0, 0.0};
  int sid;
  const int ok = check_pair(r->e, &ci, &cj, shift, &sid);
  if (ok <= 0) return ok;
  dopair1(r->e, ci, cj, sid, shift, loop);
  return 0;
}
API int orf_doself1_branch(struct runner *r, struct cell *c, int loop) {
  const struct engine *e = r->e;
  if (c->hydro.count == 0) return 0;
  if (!cell_is_active_hydro(c, e)) return 0;
  if (c->hydro.h_max_old * kernel_gamma > c->dmin) return -2;
  doself1(e, c, loop);
  return 0;
}
API int orf_dopair2_branch(struct runner *r, struct cell *ci, struct cell *cj) {
  double shift[3] = {0.0, 0.0, 0.0};
  int sid;
  const int ok = check_pair(r->e, &ci, &cj, shift, &sid);
  if (ok <= 0) return ok;
  dopair2(r->e, ci, cj, sid, shift);
  return 0;
}
API int orf_doself2_branch(struct runner *r, struct cell *c) {
  const struct engine *e = r->e;
  if (c->hydro.count == 0) return 0;
  if (!cell_is_active_hydro(c, e)) return 0;
  doself2(e, c);
  return 0;
}

/* DOSELF_SUBSET, runner_doiact_functions_hydro.h:949-1036 (density) */
API void orf_doself_subset(struct runner *r, struct cell *ci, struct part *parts,
                           const int *ind, int count) {
  const struct engine *e = r->e;
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  const int count_i = ci->hydro.count;
  struct part *parts_j = ci->hydro.parts;
  for (int pid = 0; pid < count; pid++) {
    struct part *pi = &parts[ind[pid]];
    const float pix[3] = {(float)(pi->x[0] - ci->loc[0]), (float)(pi->x[1] - ci->loc[1]),
                          (float)(pi->x[2] - ci->loc[2])};
    const float hi = pi->h;
    const float hig2 = hi * hi * kernel_gamma2;
    for (int pjd = 0; pjd < count_i; pjd++) {
      struct part *pj = &parts_j[pjd];
      if (pi == pj) continue;
      if (part_is_inhibited(pj)) continue;
      const float hj = pj->h;
      const float pjx[3] = {(float)(pj->x[0] - ci->loc[0]), (float)(pj->x[1] - ci->loc[1]),
                            (float)(pj->x[2] - ci->loc[2])};
      float dx[3] = {pix[0] - pjx[0], pix[1] - pjx[1], pix[2] - pjx[2]};
      const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
      if (r2 < hig2) iact_nonsym_density(r2, dx, hi, hj, pi, pj, a, H);
    }
  }
}

/* DOPAIR_SUBSET_NAIVE semantics (runner_doiact_functions_hydro.h:608-694):
 * every j of cj, periodic shift from the cell offsets. The sorted variant
 * (710-870) visits a superset window of the same in-range set. */
API void orf_dopair_subset(struct runner *r, struct cell *ci, struct part *parts_i,
                           const int *ind, int count, struct cell *cj) {
  const struct engine *e = r->e;
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  if (cj->hydro.count == 0) return;
  double shift[3] = {0.0, 0.0, 0.0};
  for (int k = 0; k < 3; k++) {
    if (cj->loc[k] - ci->loc[k] < -e->s->dim[k] / 2)
      shift[k] = e->s->dim[k];
    else if (cj->loc[k] - ci->loc[k] > e->s->dim[k] / 2)
      shift[k] = -e->s->dim[k];
  }
  const int count_j = cj->hydro.count;
  struct part *parts_j = cj->hydro.parts;
  for (int pid = 0; pid < count; pid++) {
    struct part *pi = &parts_i[ind[pid]];
    const double pix = pi->x[0] - shift[0];
    const double piy = pi->x[1] - shift[1];
    const double piz = pi->x[2] - shift[2];
    const float hi = pi->h;
    const float hig2 = hi * hi * kernel_gamma2;
    for (int pjd = 0; pjd < count_j; pjd++) {
      struct part *pj = &parts_j[pjd];
      if (part_is_inhibited(pj)) continue;
      const float hj = pj->h;
      float dx[3] = {(float)(pix - pj->x[0]), (float)(piy - pj->x[1]),
                     (float)(piz - pj->x[2])};
      const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
      if (r2 < hig2) iact_nonsym_density(r2, dx, hi, hj, pi, pj, a, H);
    }
  }
}

/* Brute-force oracles of the reference's tests, src/tools.c:198-700. */
API void orf_pairs_all_density(struct runner *r, struct cell *ci, struct cell *cj) {
  const struct engine *e = r->e;
  const double dim[3] = {e->s->dim[0], e->s->dim[1], e->s->dim[2]};
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  for (int i = 0; i < ci->hydro.count; ++i) {
    struct part *pi = &ci->hydro.parts[i];
    const float hi = pi->h, hig2 = hi * hi * kernel_gamma2;
    if (!PA(pi)) continue;
    for (int j = 0; j < cj->hydro.count; ++j) {
      struct part *pj = &cj->hydro.parts[j];
      float r2 = 0.0f, dx[3];
      for (int k = 0; k < 3; k++) {
        dx[k] = ci->hydro.parts[i].x[k] - cj->hydro.parts[j].x[k];
        dx[k] = nearest(dx[k], dim[k]);
        r2 += dx[k] * dx[k];
      }
      if (r2 < hig2 && !part_is_inhibited(pj))
        iact_nonsym_density(r2, dx, hi, pj->h, pi, pj, a, H);
    }
  }
  for (int j = 0; j < cj->hydro.count; ++j) {
    struct part *pj = &cj->hydro.parts[j];
    const float hj = pj->h, hjg2 = hj * hj * kernel_gamma2;
    if (!PA(pj)) continue;
    for (int i = 0; i < ci->hydro.count; ++i) {
      struct part *pi = &ci->hydro.parts[i];
      float r2 = 0.0f, dx[3];
      for (int k = 0; k < 3; k++) {
        dx[k] = cj->hydro.parts[j].x[k] - ci->hydro.parts[i].x[k];
        dx[k] = nearest(dx[k], dim[k]);
        r2 += dx[k] * dx[k];
      }
      if (r2 < hjg2 && !part_is_inhibited(pi))
        iact_nonsym_density(r2, dx, hj, pi->h, pj, pi, a, H);
    }
  }
}

API void orf_self_all_density(struct runner *r, struct cell *ci) {
  const struct engine *e = r->e;
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  for (int i = 0; i < ci->hydro.count; ++i) {
    struct part *pi = &ci->hydro.parts[i];
    const float hi = pi->h, hig2 = hi * hi * kernel_gamma2;
    for (int j = i + 1; j < ci->hydro.count; ++j) {
      struct part *pj = &ci->hydro.parts[j];
      const float hj = pj->h, hjg2 = hj * hj * kernel_gamma2;
      float r2 = 0.0f, dxi[3];
      for (int k = 0; k < 3; k++) {
        dxi[k] = ci->hydro.parts[i].x[k] - ci->hydro.parts[j].x[k];
        r2 += dxi[k] * dxi[k];
      }
      if (r2 < hig2 && PA(pi) && !part_is_inhibited(pj))
        iact_nonsym_density(r2, dxi, hi, hj, pi, pj, a, H);
      if (r2 < hjg2 && PA(pj) && !part_is_inhibited(pi)) {
        dxi[0] = -dxi[0];
        dxi[1] = -dxi[1];
        dxi[2] = -dxi[2];
        iact_nonsym_density(r2, dxi, hj, hi, pj, pi, a, H);
      }
    }
  }
}

API void orf_pairs_all_force(struct runner *r, struct cell *ci, struct cell *cj) {
  const struct engine *e = r->e;
  const double dim[3] = {e->s->dim[0], e->s->dim[1], e->s->dim[2]};
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  for (int i = 0; i < ci->hydro.count; ++i) {
    struct part *pi = &ci->hydro.parts[i];
    const float hi = pi->h, hig2 = hi * hi * kernel_gamma2;
    if (!PA(pi)) continue;
    for (int j = 0; j < cj->hydro.count; ++j) {
      struct part *pj = &cj->hydro.parts[j];
      const float hj = pj->h, hjg2 = hj * hj * kernel_gamma2;
      float r2 = 0.0f, dx[3];
      for (int k = 0; k < 3; k++) {
        dx[k] = ci->hydro.parts[i].x[k] - cj->hydro.parts[j].x[k];
        dx[k] = nearest(dx[k], dim[k]);
        r2 += dx[k] * dx[k];
      }
      if (r2 < hig2 || r2 < hjg2) {
        iact_nonsym_force(r2, dx, hi, hj, pi, pj, a, H);
        iact_nonsym_timebin(pi, pj);
      }
    }
  }
  for (int j = 0; j < cj->hydro.count; ++j) {
    struct part *pj = &cj->hydro.parts[j];
    const float hj = pj->h, hjg2 = hj * hj * kernel_gamma2;
    if (!PA(pj)) continue;
    for (int i = 0; i < ci->hydro.count; ++i) {
      struct part *pi = &ci->hydro.parts[i];
      const float hi = pi->h, hig2 = hi * hi * kernel_gamma2;
      float r2 = 0.0f, dx[3];
      for (int k = 0; k < 3; k++) {
        dx[k] = cj->hydro.parts[j].x[k] - ci->hydro.parts[i].x[k];
        dx[k] = nearest(dx[k], dim[k]);
        r2 += dx[k] * dx[k];
      }
      if (r2 < hjg2 || r2 < hig2) {
        iact_nonsym_force(r2, dx, hj, hi, pj, pi, a, H);
        iact_nonsym_timebin(pj, pi);
      }
    }
  }
}

API void orf_self_all_force(struct runner *r, struct cell *ci) {
  const struct engine *e = r->e;
  const float a = (float)e->cosmology->a, H = (float)e->cosmology->H;
  for (int i = 0; i < ci->hydro.count; ++i) {
    struct part *pi = &ci->hydro.parts[i];
    const float hi = pi->h, hig2 = hi * hi * kernel_gamma2;
    for (int j = i + 1; j < ci->hydro.count; ++j) {
      struct part *pj = &ci->hydro.parts[j];
      const float hj = pj->h, hjg2 = hj * hj * kernel_gamma2;
      float r2 = 0.0f, dxi[3];
      for (int k = 0; k < 3; k++) {
        dxi[k] = ci->hydro.parts[i].x[k] - ci->hydro.parts[j].x[k];
        r2 += dxi[k] * dxi[k];
      }
      if (r2 < hig2 || r2 < hjg2) {
        if (PA(pi) && PA(pj)) {
          iact_force(r2, dxi, hi, hj, pi, pj, a, H);
          iact_timebin(pi, pj);
        } else if (PA(pi)) {
          iact_nonsym_force(r2, dxi, hi, hj, pi, pj, a, H);
          iact_nonsym_timebin(pi, pj);
        } else if (PA(pj)) {
          dxi[0] = -dxi[0];
          dxi[1] = -dxi[1];
          dxi[2] = -dxi[2];
          iact_nonsym_force(r2, dxi, hj, hi, pj, pi, a, H);
          iact_nonsym_timebin(pj, pi);
        }
      }
    }
  }
}

/* Per-particle ops exposed for the cell-level tests (test125cells chain). */
API void orf_part_end_density(struct part *p, const struct oracle_params *P) {
  hydro_end_density(p, P);
}
API void orf_part_prepare_gradient(struct part *p, const struct oracle_params *P) {
  hydro_prepare_gradient(p, P);
  hydro_reset_gradient(p);
}
API void orf_part_extra_ghost(struct part *p, const struct oracle_params *P) {
  hydro_end_gradient(p);
  hydro_prepare_force(p, P, (float)dt_alpha_of(p->time_bin, P));
  timestep_limiter_prepare_force(p);
  hydro_reset_acceleration(p);
}
API void orf_part_end_force(struct part *p) { hydro_end_force(p); }
API void orf_part_init(struct part *p) { hydro_init_part(p); }

/* ------------------------------------------------------------------------ */
/* CPU baseline: the float restatement of DOSELF1/DOPAIR1 (density) and     */
/* DOSELF2/DOPAIR2 (force) over a periodic top-level cell grid, multi-      */
/* threaded with conflict-free scheduling: all self tasks in parallel; then */
/* for each of the 13 pair directions and each of the 8 parity classes of  */
/* the left cell, all pairs in parallel (two pairs of one (direction,      */
/* parity) group never share a cell when cdim is even).                    */
/* ------------------------------------------------------------------------ */
struct orf_cellgrid {
  int cdim;
  struct cell *cells;
  struct part *parts; /* cell-ordered copy */
  long long N;
};

static const int pair_dirs[13][3] = {{1, 1, 1}, {1, 1, 0}, {1, 1, -1}, {1, 0, 1},
                                     {1, 0, 0}, {1, 0, -1}, {1, -1, 1}, {1, -1, 0},
                                     {1, -1, -1}, {0, 1, 1}, {0, 1, 0}, {0, 1, -1},
                                     {0, 0, 1}};

/* Build a cdim^3 periodic grid of cells over a copy of the particles,
 * sorted in all 13 directions. */
API struct orf_cellgrid *orf_cellgrid_new(const struct part *parts, long long N,
                                          double box, int cdim) {
  struct orf_cellgrid *g = (struct orf_cellgrid *)calloc(1, sizeof(*g));
  g->cdim = cdim;
  g->N = N;
  const int nc = cdim * cdim * cdim;
  g->cells = (struct cell *)calloc((size_t)nc, sizeof(struct cell));
  g->parts = (struct part *)aligned_alloc(32, sizeof(struct part) * (size_t)(N > 0 ? N : 1));
  int *cnt = (int *)calloc((size_t)nc + 1, sizeof(int));
  int *cof = (int *)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
  const double w = box / cdim;
  for (long long i = 0; i < N; i++) {
    int c[3];
    for (int k = 0; k < 3; k++) {
      double xx = parts[i].x[k] - floor(parts[i].x[k] / box) * box;
      c[k] = (int)(xx / w);
      if (c[k] >= cdim) c[k] = cdim - 1;
    }
    cof[i] = (c[0] * cdim + c[1]) * cdim + c[2];
    cnt[cof[i] + 1]++;
  }
  for (int c = 0; c < nc; c++) cnt[c + 1] += cnt[c];
  int *fill = (int *)malloc(sizeof(int) * (size_t)nc);
  memcpy(fill, cnt, sizeof(int) * (size_t)nc);
  for (long long i = 0; i < N; i++) g->parts[fill[cof[i]]++] = parts[i];
  for (int cx = 0; cx < cdim; cx++)
    for (int cy = 0; cy < cdim; cy++)
      for (int cz = 0; cz < cdim; cz++) {
        const int id = (cx * cdim + cy) * cdim + cz;
        struct cell *c = &g->cells[id];
        c->loc[0] = cx * w;
        c->loc[1] = cy * w;
        c->loc[2] = cz * w;
        c->width[0] = c->width[1] = c->width[2] = w;
        c->dmin = (float)w;
        c->hydro.parts = g->parts + cnt[id];
        c->hydro.count = cnt[id + 1] - cnt[id];
        float hmax = 0.f;
        for (int k = 0; k < c->hydro.count; k++)
          if (c->hydro.parts[k].h > hmax) hmax = c->hydro.parts[k].h;
        c->hydro.h_max = c->hydro.h_max_old = c->hydro.h_max_active = hmax;
        c->hydro.ti_end_min = 8;
        c->hydro.ti_old_part = 8;
      }
#pragma omp parallel for schedule(dynamic, 8)
  for (int id = 0; id < nc; id++) orf_cell_sort(&g->cells[id], 0x1FFF);
  free(fill);
  free(cnt);
  free(cof);
  return g;
}

API void orf_cellgrid_free(struct orf_cellgrid *g) {
  const int nc = g->cdim * g->cdim * g->cdim;
  for (int id = 0; id < nc; id++) orf_cell_free_sorts(&g->cells[id]);
  free(g->cells);
  free(g->parts);
  free(g);
}

API struct part *orf_cellgrid_parts(struct orf_cellgrid *g) { return g->parts; }

/* Runs the full density (loop=0) or force (loop=2) pass over the grid with
 * `nthreads` threads. Returns elapsed wall seconds. */
API double orf_cellgrid_run(struct orf_cellgrid *g, struct runner *r, int loop,
                            int nthreads) {
  const int cdim = g->cdim;
  const int nc = cdim * cdim * cdim;
  struct timespec t0, t1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp parallel
  {
#pragma omp for schedule(dynamic, 4)
    for (int id = 0; id < nc; id++) {
      if (loop == LOOP_FORCE)
        orf_doself2_branch(r, &g->cells[id]);
      else
        orf_doself1_branch(r, &g->cells[id], loop);
    }
    for (int d = 0; d < 13; d++) {
      for (int par = 0; par < 8; par++) {
        const int px = par & 1, py = (par >> 1) & 1, pz = (par >> 2) & 1;
        const int h = cdim / 2;
#pragma omp for schedule(dynamic, 4)
        for (int t = 0; t < h * h * h; t++) {
          const int cx = 2 * (t / (h * h)) + px;
          const int cy = 2 * ((t / h) % h) + py;
          const int cz = 2 * (t % h) + pz;
          const int nx = (cx + pair_dirs[d][0] + cdim) % cdim;
          const int ny = (cy + pair_dirs[d][1] + cdim) % cdim;
          const int nz = (cz + pair_dirs[d][2] + cdim) % cdim;
          struct cell *ci = &g->cells[(cx * cdim + cy) * cdim + cz];
          struct cell *cj = &g->cells[(nx * cdim + ny) * cdim + nz];
          if (loop == LOOP_FORCE)
            orf_dopair2_branch(r, ci, cj);
          else
            orf_dopair1_branch(r, ci, cj, loop);
        }
      }
    }
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------------ */
/* CPU baseline on SWIFT's cell tree (clustered inputs): the top-level grid  */
/* as above, each top cell split into octants while it holds more than      */
/* splitsize particles (space_split, space_splitsize 400, space.h:49), every */
/* cell sorted, and the tasks run through the DOSUB recursion              */
/* (runner_doiact_functions_hydro.h:2524-2617 density, 2630-2720 force:     */
/* recurse while cell_can_recurse_in_{self,pair}_hydro_task, cell.h:761-782, */
/* over the touching progeny pairs of cell_split_pairs, cell.c:62; else the */
/* DOSELF/DOPAIR branch). Scheduling as orf_cellgrid_run, so two threads    */
/* never touch one top cell's subtree at once.                              */
/* ------------------------------------------------------------------------ */
struct orf_celltree {
  int cdim;
  struct cell *top;        /* cdim^3 top cells */
  struct cell **blocks;    /* arena of progeny cells (stable addresses) */
  int nblocks, used;       /* cells used in the last block */
  long long ncells;
  struct part *parts;      /* tree-ordered copy */
  long long N;
};
#define ORF_ARENA 4096

static struct cell *celltree_alloc(struct orf_celltree *t) {
  if (t->nblocks == 0 || t->used == ORF_ARENA) {
    t->blocks = (struct cell **)realloc(t->blocks, sizeof(struct cell *) * (size_t)(t->nblocks + 1));
    t->blocks[t->nblocks++] = (struct cell *)calloc(ORF_ARENA, sizeof(struct cell));
    t->used = 0;
  }
  t->ncells++;
  return &t->blocks[t->nblocks - 1][t->used++];
}

static void celltree_hmax(struct cell *c) {
  float hmax = 0.f;
  for (int k = 0; k < c->hydro.count; k++)
    if (c->hydro.parts[k].h > hmax) hmax = c->hydro.parts[k].h;
  c->hydro.h_max = c->hydro.h_max_old = c->hydro.h_max_active = hmax;
  c->hydro.ti_end_min = 8;
  c->hydro.ti_old_part = 8;
}

/* space_split's octants: progeny k at ((k >> 2) & 1, (k >> 1) & 1, k & 1)
 * half-widths from the cell's corner (space_split.c:233) */
static void celltree_split(struct orf_celltree *t, struct cell *c, double box, int splitsize,
                           int depth, struct part *tmp) {
  if (c->hydro.count <= splitsize || depth >= 24) return;
  const int n = c->hydro.count;
  int cnt[9] = {0};
  unsigned char *oct = (unsigned char *)malloc((size_t)n);
  const double half[3] = {0.5 * c->width[0], 0.5 * c->width[1], 0.5 * c->width[2]};
  for (int k = 0; k < n; k++) {
    int o = 0;
    for (int d = 0; d < 3; d++) {
      const double xx = c->hydro.parts[k].x[d] - floor(c->hydro.parts[k].x[d] / box) * box;
      o |= (xx >= c->loc[d] + half[d]) << (2 - d);
    }
    oct[k] = (unsigned char)o;
    cnt[o + 1]++;
  }
  for (int o = 0; o < 8; o++) cnt[o + 1] += cnt[o];
  int fill[8];
  memcpy(fill, cnt, sizeof(fill));
  for (int k = 0; k < n; k++) tmp[fill[oct[k]]++] = c->hydro.parts[k];
  memcpy(c->hydro.parts, tmp, sizeof(struct part) * (size_t)n);
  free(oct);
  c->split = 1;
  for (int o = 0; o < 8; o++) {
    struct cell *p = celltree_alloc(t);
    p->loc[0] = c->loc[0] + ((o >> 2) & 1) * half[0];
    p->loc[1] = c->loc[1] + ((o >> 1) & 1) * half[1];
    p->loc[2] = c->loc[2] + (o & 1) * half[2];
    for (int d = 0; d < 3; d++) p->width[d] = half[d];
    p->dmin = 0.5f * c->dmin;
    p->parent = c;
    p->hydro.parts = c->hydro.parts + cnt[o];
    p->hydro.count = cnt[o + 1] - cnt[o];
    celltree_hmax(p);
    c->progeny[o] = p;
    celltree_split(t, p, box, splitsize, depth + 1, tmp);
  }
}

static void celltree_sort_all(struct cell *c) {
  orf_cell_sort(c, 0x1FFF);
  if (c->split)
    for (int o = 0; o < 8; o++)
      if (c->progeny[o]) celltree_sort_all(c->progeny[o]);
}

API struct orf_celltree *orf_celltree_new(const struct part *parts, long long N, double box,
                                          int cdim, int splitsize) {
  struct orf_celltree *t = (struct orf_celltree *)calloc(1, sizeof(*t));
  struct orf_cellgrid *g = orf_cellgrid_new(parts, N, box, cdim);
  /* take over the grid's top cells and particle copy; the top cells' sorts
   * are rebuilt after the split reorders their particles */
  const int nc = cdim * cdim * cdim;
  for (int id = 0; id < nc; id++) orf_cell_free_sorts(&g->cells[id]);
  t->cdim = cdim;
  t->top = g->cells;
  t->parts = g->parts;
  t->N = N;
  t->ncells = nc;
  free(g);
  struct part *tmp = (struct part *)malloc(sizeof(struct part) * (size_t)(N > 0 ? N : 1));
  for (int id = 0; id < nc; id++) celltree_split(t, &t->top[id], box, splitsize, 0, tmp);
  free(tmp);
#pragma omp parallel for schedule(dynamic, 1)
  for (int id = 0; id < nc; id++) celltree_sort_all(&t->top[id]);
  return t;
}

static void celltree_free_sorts(struct cell *c) {
  orf_cell_free_sorts(c);
  if (c->split)
    for (int o = 0; o < 8; o++)
      if (c->progeny[o]) celltree_free_sorts(c->progeny[o]);
}

API void orf_celltree_free(struct orf_celltree *t) {
  const int nc = t->cdim * t->cdim * t->cdim;
  for (int id = 0; id < nc; id++) celltree_free_sorts(&t->top[id]);
  for (int b = 0; b < t->nblocks; b++) free(t->blocks[b]);
  free(t->blocks);
  free(t->top);
  free(t->parts);
  free(t);
}

API long long orf_celltree_ncells(const struct orf_celltree *t) { return t->ncells; }
API struct part *orf_celltree_parts(struct orf_celltree *t) { return t->parts; }

/* cell_split_pairs (cell.c:62) as a set: the progeny pairs (pid of ci, pjd of
 * cj) that touch across the face/edge/corner of direction sid */
static int split_pairs_n[13], split_pairs_ij[13][16][2];
static void split_pairs_make(void) {
  for (int sid = 0; sid < 13; sid++) {
    int n = 0;
    for (int a = 0; a < 8; a++)
      for (int b = 0; b < 8; b++) {
        int ok = 1;
        for (int k = 0; k < 3; k++) {
          const int d = 2 * pair_dirs[sid][k] + ((b >> (2 - k)) & 1) - ((a >> (2 - k)) & 1);
          if (d < -1 || d > 1) ok = 0;
        }
        if (ok) {
          split_pairs_ij[sid][n][0] = a;
          split_pairs_ij[sid][n][1] = b;
          n++;
        }
      }
    split_pairs_n[sid] = n;
  }
}

static int can_recurse_pair(const struct cell *c) { /* cell.h:761-769 */
  return c->split && (kernel_gamma * c->hydro.h_max_old + c->hydro.dx_max_part_old) < 0.5f * c->dmin;
}
static int can_recurse_self(const struct cell *c) { /* cell.h:778-782 */
  return c->split && (kernel_gamma * c->hydro.h_max_old < 0.5f * c->dmin);
}

static void dosub_pair(struct runner *r, struct cell *ci, struct cell *cj, int loop) {
  const struct engine *e = r->e;
  if (!cell_is_active_hydro(ci, e) && !cell_is_active_hydro(cj, e)) return;
  if (ci->hydro.count == 0 || cj->hydro.count == 0) return;
  double shift[3];
  const int sid = space_getsid(e->s, &ci, &cj, shift);
  if (can_recurse_pair(ci) && can_recurse_pair(cj)) {
    for (int k = 0; k < split_pairs_n[sid]; k++) {
      struct cell *pi = ci->progeny[split_pairs_ij[sid][k][0]];
      struct cell *pj = cj->progeny[split_pairs_ij[sid][k][1]];
      if (pi && pj) dosub_pair(r, pi, pj, loop);
    }
  } else if (loop == LOOP_FORCE) {
    orf_dopair2_branch(r, ci, cj);
  } else {
    orf_dopair1_branch(r, ci, cj, loop);
  }
}

static void dosub_self(struct runner *r, struct cell *c, int loop) {
  if (c->hydro.count == 0 || !cell_is_active_hydro(c, r->e)) return;
  if (can_recurse_self(c)) {
    for (int k = 0; k < 8; k++)
      if (c->progeny[k]) {
        dosub_self(r, c->progeny[k], loop);
        for (int j = k + 1; j < 8; j++)
          if (c->progeny[j]) dosub_pair(r, c->progeny[k], c->progeny[j], loop);
      }
  } else if (loop == LOOP_FORCE) {
    orf_doself2_branch(r, c);
  } else {
    orf_doself1_branch(r, c, loop);
  }
}

/* The density (loop 0) or force (loop 2) pass over the tree with `nthreads`
 * threads; returns elapsed wall seconds. */
API double orf_celltree_run(struct orf_celltree *t, struct runner *r, int loop, int nthreads) {
  if (!split_pairs_n[12]) split_pairs_make();
  const int cdim = t->cdim;
  const int nc = cdim * cdim * cdim;
  struct timespec t0, t1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp parallel
  {
#pragma omp for schedule(dynamic, 1)
    for (int id = 0; id < nc; id++) dosub_self(r, &t->top[id], loop);
    for (int d = 0; d < 13; d++) {
      for (int par = 0; par < 8; par++) {
        const int px = par & 1, py = (par >> 1) & 1, pz = (par >> 2) & 1;
        const int h = cdim / 2;
#pragma omp for schedule(dynamic, 1)
        for (int q = 0; q < h * h * h; q++) {
          const int cx = 2 * (q / (h * h)) + px;
          const int cy = 2 * ((q / h) % h) + py;
          const int cz = 2 * (q % h) + pz;
          const int nx = (cx + pair_dirs[d][0] + cdim) % cdim;
          const int ny = (cy + pair_dirs[d][1] + cdim) % cdim;
          const int nz = (cz + pair_dirs[d][2] + cdim) % cdim;
          dosub_pair(r, &t->top[(cx * cdim + cy) * cdim + cz],
                     &t->top[(nx * cdim + ny) * cdim + nz], loop);
        }
      }
    }
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
#endif /* ORACLE_F32 */

/* ======================================================================== */
/* Gravity P2P — src/runner_doiact_grav.c, src/gravity/MultiSoftening/      */
/* gravity_iact.h, src/kernel_gravity.h, src/kernel_long_gravity.h,         */
/* src/gravity_cache.h. Float restatement in the f32 build; the f64 build   */
/* promotes every temporary.                                                */
/* ======================================================================== */

/* kernel_gravity.h:48-70 (Wendland-C2) */
static inline real kernel_grav_pot_eval(real u) {
  real W = (real)3.f * u - (real)15.f;
  W = W * u + (real)28.f;
  W = W * u - (real)21.f;
  W = W * u;
  W = W * u + (real)7.f;
  W = W * u;
  W = W * u - (real)3.f;
  return W;
}
/* kernel_gravity.h:79-100 */
static inline real kernel_grav_force_eval(real u) {
  real W = (real)21.f * u - (real)90.f;
  W = W * u + (real)140.f;
  W = W * u - (real)84.f;
  W = W * u;
  W = W * u + (real)14.f;
  return W;
}
/* kernel_long_gravity.h:204-262 (default branch) */
static inline void kernel_long_grav_eval(real r_over_r_s, real *corr_f, real *corr_pot) {
  const real x = (real)2.f * r_over_r_s;
  const real exp_x = EXP(x);
  const real alpha = (real)1.f / ((real)1.f + exp_x);
  real W = (real)1.f - alpha * exp_x;
  W = W * (real)2.f;
  *corr_pot = W;
  W = (real)1.f - alpha;
  W = W * x - exp_x;
  W = W * alpha + (real)1.f;
  W = W * (real)2.f;
  *corr_f = W;
}
/* gravity_iact.h:47-81 */
static inline void iact_grav_pp_full(real r2, real h2, real h_inv, real h_inv3,
                                     real mass, real *f_ij, real *pot_ij) {
  const real r_inv = (real)1.f / SQRT(r2 + (real)FLT_MIN);
  if (r2 >= h2) {
    *f_ij = mass * r_inv * r_inv * r_inv;
    *pot_ij = -mass * r_inv;
  } else {
    const real r = r2 * r_inv;
    const real ui = r * h_inv;
    *f_ij = mass * h_inv3 * kernel_grav_force_eval(ui);
    *pot_ij = mass * h_inv * kernel_grav_pot_eval(ui);
  }
}
/* gravity_iact.h:91-135 */
static inline void iact_grav_pp_truncated(real r2, real h2, real h_inv, real h_inv3,
                                          real mass, real r_s_inv, real *f_ij,
                                          real *pot_ij) {
  const real r_inv = (real)1.f / SQRT(r2 + (real)FLT_MIN);
  const real r = r2 * r_inv;
  if (r2 >= h2) {
    *f_ij = mass * r_inv * r_inv * r_inv;
    *pot_ij = -mass * r_inv;
  } else {
    const real ui = r * h_inv;
    *f_ij = mass * h_inv3 * kernel_grav_force_eval(ui);
    *pot_ij = mass * h_inv * kernel_grav_pot_eval(ui);
  }
  const real u_lr = r * r_s_inv;
  real corr_f_lr, corr_pot_lr;
  kernel_long_grav_eval(u_lr, &corr_f_lr, &corr_pot_lr);
  *f_ij *= corr_f_lr;
  *pot_ij *= corr_pot_lr;
}

static inline real nearest_r(real dx, real box) {
  return ((dx > (real)0.5f * box) ? (dx - box)
                                  : ((dx < (real)-0.5f * box) ? (dx + box) : dx));
}

struct oracle_grav_params {
  int periodic;        /* e->mesh->periodic */
  float dim[3];        /* e->mesh->dim */
  float r_s_inv;       /* e->mesh->r_s_inv */
  double r_cut_min;    /* e->mesh->r_cut_min */
  int max_active_bin;
  /* gravity_props fields of gravity_M2P_accept */
  float theta_crit;
  float adaptive_tolerance;
  int use_advanced_MAC;
  int use_gadget_tolerance;
  int use_tree_below_softening;
  int consider_truncation_in_MAC;
  double r_cut_max;    /* e->mesh->r_cut_max */
};

/* ------------------------------------------------------------------------ */
/* Multipoles, order 4 (SELF_GRAVITY_MULTIPOLE_ORDER of the default build): */
/* struct multipole / gravity_tensors (src/multipole_struct.h:110-220) with */
/* the 35 terms in member order (dipole zero at 1..3), P2M                  */
/* (src/multipole.h:983-1266), the multipole power (878-972), the M2P       */
/* acceptance (src/multipole_accept.h:290-373) and M2P                      */
/* (src/multipole.h:2257-2480, src/gravity_derivatives.h:516-760).          */
/* ------------------------------------------------------------------------ */
struct oracle_multipole {
  double CoM[3];
  double r_max;
  float M[35];
  float power[5];
  float max_softening;
  float min_old_a_grav_norm;
};

static const int mp_a[35] = {0, 1, 0, 0, 2, 0, 0, 1, 1, 0, 3, 0, 0, 2, 2, 1, 0, 1,
                             0, 1, 4, 0, 0, 3, 3, 1, 0, 1, 0, 2, 2, 0, 2, 1, 1};
static const int mp_b[35] = {0, 0, 1, 0, 0, 2, 0, 1, 0, 1, 0, 3, 0, 1, 0, 2, 2, 0,
                             1, 1, 0, 4, 0, 1, 0, 3, 3, 0, 1, 2, 0, 2, 1, 2, 1};
static const int mp_c[35] = {0, 0, 0, 1, 0, 0, 2, 0, 1, 1, 0, 0, 3, 0, 1, 0, 1, 2,
                             2, 1, 0, 0, 4, 0, 1, 0, 1, 3, 3, 0, 2, 2, 1, 1, 2};

static double fact_d(int n) { return n <= 1 ? 1. : n * fact_d(n - 1); }

/* gravity_P2M: mass, CoM, then M_n = (-1)^|n| sum m X_n(dx) with X_n =
 * dx^n / n! (vector_power.h) about the CoM, accumulated in double and stored
 * as float; r_max; then gravity_multipole_compute_power (float squares for
 * unit weights, double products for the fractional ones, as written). */
/* gravity_multipole_compute_power (multipole.h:1220-1266) */
static void mpole_power(struct oracle_multipole *out) {
  double pw[5] = {0., 0., 0., 0., 0.};
  for (int t = 4; t < 35; t++) {
    const int a = mp_a[t], b = mp_b[t], c = mp_c[t], o = a + b + c;
    const double w = fact_d(a) * fact_d(b) * fact_d(c) / fact_d(o);
    const float M = out->M[t];
    if (w == 1.)
      pw[o] += (double)(M * M);
    else
      pw[o] += w * (double)M * (double)M;
  }
  out->power[0] = out->M[0];
  out->power[1] = 0.f;
  for (int o = 2; o <= 4; o++) out->power[o] = (float)sqrt(pw[o]);
}

API void PFX(grav_p2m)(const struct gpart *g, int n, struct oracle_multipole *out) {
  float eps_max = 0.f, oag_min = FLT_MAX;
  double mass = 0., com[3] = {0., 0., 0.};
  for (int k = 0; k < n; k++) {
    const double m = g[k].mass;
    eps_max = eps_max > g[k].epsilon ? eps_max : g[k].epsilon;
    oag_min = oag_min < g[k].old_a_grav_norm ? oag_min : g[k].old_a_grav_norm;
    mass += m;
    for (int d = 0; d < 3; d++) com[d] += g[k].x[d] * m;
  }
  const double imass = 1.0 / mass;
  for (int d = 0; d < 3; d++) com[d] *= imass;
  double Md[35] = {0.};
  double r_max2 = 0.;
  for (int k = 0; k < n; k++) {
    const double dx[3] = {g[k].x[0] - com[0], g[k].x[1] - com[1], g[k].x[2] - com[2]};
    r_max2 = fmax(r_max2, dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2]);
    const double m = g[k].mass;
    for (int t = 4; t < 35; t++) {
      const int a = mp_a[t], b = mp_b[t], c = mp_c[t];
      const double X = pow(dx[0], a) * pow(dx[1], b) * pow(dx[2], c) /
                       (fact_d(a) * fact_d(b) * fact_d(c));
      Md[t] += ((a + b + c) & 1) ? -m * X : m * X;
    }
  }
  for (int d = 0; d < 3; d++) out->CoM[d] = com[d];
  out->r_max = sqrt(r_max2);
  out->M[0] = (float)mass;
  out->M[1] = out->M[2] = out->M[3] = 0.f;
  for (int t = 4; t < 35; t++) out->M[t] = (float)Md[t];
  out->max_softening = eps_max;
  out->min_old_a_grav_norm = oag_min;
  mpole_power(out);
}

/* gravity_M2M (src/multipole.h:1278) + gravity_multipole_add (:352) of every
 * child of a split cell, with space_split's CoM, r_max and softening
 * (src/space_split.c:340-440). M'_n = sum_{m <= n} M_m X_{n-m}(CoM - CoM_k),
 * X_k(v) = v^k / k! (the zero dipole skipped); each child's shifted terms are
 * rounded to float and added in float, as the reference's temp multipole is
 * (the f64 build keeps the sum in double). */
API void PFX(grav_m2m)(const struct oracle_multipole *const *kids, int nkids,
                       const double loc[3], const double width[3],
                       struct oracle_multipole *out) {
  double mass = 0., com[3] = {0., 0., 0.};
  for (int k = 0; k < nkids; k++) {
    mass += kids[k]->M[0];
    for (int d = 0; d < 3; d++) com[d] += kids[k]->CoM[d] * kids[k]->M[0];
  }
  const double imass = 1. / mass;
  for (int d = 0; d < 3; d++) com[d] *= imass;
  real M[35];
  for (int t = 0; t < 35; t++) M[t] = 0;
  float eps_max = 0.f, oag_min = FLT_MAX;
  double r_max = 0.;
  for (int k = 0; k < nkids; k++) {
    const struct oracle_multipole *B = kids[k];
    const double dx[3] = {com[0] - B->CoM[0], com[1] - B->CoM[1], com[2] - B->CoM[2]};
    for (int t = 0; t < 35; t++) {
      if (t >= 1 && t <= 3) continue;
      double v = 0.;
      for (int q = 0; q < 35; q++) {
        if (q >= 1 && q <= 3) continue;
        const int a = mp_a[t] - mp_a[q], b = mp_b[t] - mp_b[q], c = mp_c[t] - mp_c[q];
        if (a < 0 || b < 0 || c < 0) continue;
        v += (double)B->M[q] * pow(dx[0], a) * pow(dx[1], b) * pow(dx[2], c) /
             (fact_d(a) * fact_d(b) * fact_d(c));
      }
      M[t] += (real)v;
    }
    eps_max = eps_max > B->max_softening ? eps_max : B->max_softening;
    oag_min = oag_min < B->min_old_a_grav_norm ? oag_min : B->min_old_a_grav_norm;
    const double r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
    r_max = fmax(r_max, B->r_max + sqrt(r2));
  }
  /* the alternative bound: the CoM's distance to the farthest corner */
  double c2 = 0.;
  for (int d = 0; d < 3; d++) {
    const double e = com[d] > loc[d] + width[d] / 2. ? com[d] - loc[d] : loc[d] + width[d] - com[d];
    c2 += e * e;
  }
  for (int d = 0; d < 3; d++) out->CoM[d] = com[d];
  out->r_max = fmin(r_max, sqrt(c2));
  for (int t = 0; t < 35; t++) out->M[t] = (float)M[t];
  out->M[0] = (float)mass;
  out->M[1] = out->M[2] = out->M[3] = 0.f;
  out->max_softening = eps_max;
  out->min_old_a_grav_norm = oag_min;
  mpole_power(out);
}

/* gravity_M2P_accept for a gpart at float cache position x (the float
 * arithmetic of the reference in both builds: the choice is discrete). */
static int m2p_accept(const struct oracle_grav_params *G, const struct gpart *pa,
                      const struct oracle_multipole *B, const float x[3], int periodic) {
  float dx[3];
  for (int k = 0; k < 3; k++) {
    dx[k] = x[k] - (float)B->CoM[k];
    if (periodic) {
      const float L = G->dim[k];
      dx[k] = (dx[k] > 0.5f * L) ? dx[k] - L : ((dx[k] < -0.5f * L) ? dx[k] + L : dx[k]);
    }
  }
  const float r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
  const float rho_B = (float)B->r_max;
  const float max_softening = B->max_softening > pa->epsilon ? B->max_softening : pa->epsilon;
  const float E_BA_term = 8.f * B->power[2];
  const float r_to_p = r2;
  float f_MAC_inv;
  if (periodic && G->consider_truncation_in_MAC) {
    const float H = max_softening;
    if (r2 < (25.f / 81.f) * H * H)
      f_MAC_inv = (25.f / 81.f) * H * H;
    else if (G->r_s_inv * G->r_s_inv * r2 > (25.f / 9.f))
      f_MAC_inv = (9.f / 25.f) * G->r_s_inv * G->r_s_inv * r2 * r2;
    else
      f_MAC_inv = r2;
  } else {
    f_MAC_inv = r2;
  }
  const float old_a_grav = pa->old_a_grav_norm;
  const float eps = G->adaptive_tolerance;
  const float theta_crit = G->theta_crit;
  const float theta_crit2 = theta_crit * theta_crit;
  const int cond_2 = G->use_tree_below_softening || max_softening * max_softening < r2;
  if (G->use_advanced_MAC && G->use_gadget_tolerance) {
    const float q = rho_B / sqrtf(r2);
    const float q2 = q * q;
    const float ratio = q2 * q2;
    return (B->M[0] * ratio < eps * old_a_grav * f_MAC_inv) && cond_2;
  } else if (G->use_advanced_MAC) {
    const int cond_1 = rho_B * rho_B < r2;
    const int cond_3 = E_BA_term < eps * old_a_grav * r_to_p * f_MAC_inv;
    return cond_1 && cond_2 && cond_3;
  }
  return (rho_B * rho_B < theta_crit2 * r2) && cond_2;
}

/* kernel_gravity.h:169-275: D_soft_1..6 */
static void d_soft_all(real u, real d[7]) {
  real p = (real)-3.f * u + (real)15.f;
  p = p * u - (real)28.f; p = p * u + (real)21.f; p = p * u; p = p * u - (real)7.f;
  p = p * u; p = p * u + (real)3.f;
  d[1] = p;
  p = (real)-21.f * u + (real)90.f;
  p = p * u - (real)140.f; p = p * u + (real)84.f; p = p * u; p = p * u - (real)14.f;
  p = p * u;
  d[2] = p;
  p = (real)-105.f * u + (real)360.f;
  p = p * u - (real)420.f; p = p * u + (real)168.f; p = p * u; p = p * u;
  d[3] = p;
  p = (real)-315.f * u + (real)720.f;
  p = p * u - (real)420.f; p = p * u; p = p * u;
  d[4] = p;
  p = (real)-315.f * u; p = p * u + (real)420.f; p = p * u;
  d[5] = p;
  p = (real)315.f * u; p = p * u - (real)1260.f;
  d[6] = p;
}

/* potential_derivatives_compute_M2P: the radial factors Dt_1..Dt_6, then
 * D_abc for a+b+c <= 5 in the reference's closed forms (by the shape of the
 * sorted exponents; the Dt are rescaled by r^-1 between orders exactly as
 * the reference does). */
struct m2p_derivs {
  real rr[3];     /* r_x / r, r_y / r, r_z / r */
  real Dt[6][7];  /* Dt[o][k]: Dt_k as scaled when order o is formed */
};

static void m2p_radial(real r_x, real r_y, real r_z, real r2, real r_inv, real eps,
                       int periodic, real r_s_inv, struct m2p_derivs *d) {
  real Dt[7];
  if (r2 < eps * eps) {
    const real eps_inv = (real)1.f / eps;
    const real r = r2 * r_inv;
    const real u = r * eps_inv;
    real ds[7];
    d_soft_all(u, ds);
    real e = eps_inv;
    for (int k = 1; k <= 6; k++) {
      Dt[k] = e * ds[k];
      e = e * eps_inv;
    }
  } else if (!periodic) {
    Dt[1] = r_inv;
    Dt[2] = (real)-1.f * Dt[1] * r_inv;
    Dt[3] = (real)-3.f * Dt[2] * r_inv;
    Dt[4] = (real)-5.f * Dt[3] * r_inv;
    Dt[5] = (real)-7.f * Dt[4] * r_inv;
    Dt[6] = (real)-9.f * Dt[5] * r_inv;
  } else {
    /* kernel_long_grav_derivatives, default branch (kernel_long_gravity.h:151-183) */
    const real r = r2 * r_inv;
    const real c1 = (real)2.f * r_s_inv;
    const real c2 = c1 * c1, c3 = c2 * c1, c4 = c3 * c1, c5 = c4 * c1;
    const real x = c1 * r;
    const real exp_x = EXP(x);
    const real a_inv = (real)1.f + exp_x;
    const real a1 = (real)1.f / a_inv;
    const real a2 = a1 * a1, a3 = a2 * a1, a4 = a3 * a1, a5 = a4 * a1, a6 = a5 * a1;
    const real chi0 = (real)-2.f * exp_x * a1 + (real)2.f;
    const real chi1 = (real)-2.f * exp_x * c1 * a2;
    const real chi2 = (real)-2.f * exp_x * c2 * ((real)2.f * a3 - a2);
    const real chi3 = (real)-2.f * exp_x * c3 * ((real)6.f * a4 - (real)6.f * a3 + a2);
    const real chi4 =
        (real)-2.f * exp_x * c4 * ((real)24.f * a5 - (real)36.f * a4 + (real)14.f * a3 - a2);
    const real chi5 = (real)-2.f * exp_x * c5 *
                      ((real)120.f * a6 - (real)240.f * a5 + (real)150.f * a4 -
                       (real)30.f * a3 + a2);
    Dt[1] = chi0 * r_inv;
    Dt[2] = (chi1 - chi0 * r_inv) * r_inv;
    Dt[3] = ((chi0 * r_inv - chi1) * (real)3.f * r_inv + chi2) * r_inv;
    Dt[4] = (((-chi0 * r_inv + chi1) * (real)15.f * r_inv - (real)6.f * chi2) * r_inv + chi3) *
            r_inv;
    Dt[5] = ((((chi0 * r_inv - chi1) * (real)105.f * r_inv + (real)45.f * chi2) * r_inv -
              (real)10.f * chi3) * r_inv + chi4) * r_inv;
    Dt[6] = (((((-chi0 * r_inv + chi1) * (real)945.f * r_inv - (real)420.f * chi2) * r_inv +
               (real)105.f * chi3) * r_inv - (real)15.f * chi4) * r_inv + chi5) * r_inv;
  }
  d->rr[0] = r_x * r_inv;
  d->rr[1] = r_y * r_inv;
  d->rr[2] = r_z * r_inv;
  /* the reference's in-place rescaling: before order 2 Dt_2 *= r^-1, before
   * order 3 Dt_3 *= r^-1, before 4 Dt_3, Dt_4 *= r^-1, before 5 Dt_4, Dt_5 */
  for (int o = 0; o < 6; o++) {
    if (o == 2) Dt[2] = Dt[2] * r_inv;
    if (o == 3) Dt[3] = Dt[3] * r_inv;
    if (o == 4) { Dt[3] = Dt[3] * r_inv; Dt[4] = Dt[4] * r_inv; }
    if (o == 5) { Dt[4] = Dt[4] * r_inv; Dt[5] = Dt[5] * r_inv; }
    for (int k = 0; k < 7; k++) d->Dt[o][k] = Dt[k];
  }
}

static real ipow(real x, int n) {
  real y = (real)1.f;
  for (int k = 0; k < n; k++) y = y * x;
  return y;
}

/* D_abc from the closed form of its shape: e = exponents, sorted so that
 * e[p[0]] >= e[p[1]] >= e[p[2]] */
static real m2p_D(const struct m2p_derivs *d, int a, int b, int c) {
  const int e[3] = {a, b, c};
  int p[3] = {0, 1, 2};
  for (int i = 0; i < 3; i++)
    for (int j = i + 1; j < 3; j++)
      if (e[p[j]] > e[p[i]]) { const int t = p[i]; p[i] = p[j]; p[j] = t; }
  const int n1 = e[p[0]], n2 = e[p[1]], n3 = e[p[2]], o = a + b + c;
  const real u = d->rr[p[0]], v = d->rr[p[1]], w = d->rr[p[2]];
  const real *Dt = d->Dt[o];
  switch (o) {
    case 0: return Dt[1];
    case 1: return u * Dt[2];
    case 2: return n1 == 2 ? u * u * Dt[3] + Dt[2] : u * v * Dt[3];
    case 3:
      if (n1 == 3) return ipow(u, 3) * Dt[4] + (real)3.f * u * Dt[3];
      if (n1 == 2) return u * u * v * Dt[4] + v * Dt[3];
      return u * v * w * Dt[4];
    case 4:
      if (n1 == 4) return ipow(u, 4) * Dt[5] + (real)6.f * u * u * Dt[4] + (real)3.f * Dt[3];
      if (n1 == 3) return ipow(u, 3) * v * Dt[5] + (real)3.f * u * v * Dt[4];
      if (n2 == 2) return u * u * v * v * Dt[5] + u * u * Dt[4] + v * v * Dt[4] + Dt[3];
      return u * u * v * w * Dt[5] + v * w * Dt[4];
    default:
      if (n1 == 5) return ipow(u, 5) * Dt[6] + (real)10.f * ipow(u, 3) * Dt[5] + (real)15.f * u * Dt[4];
      if (n1 == 4) return ipow(u, 4) * v * Dt[6] + (real)6.f * u * u * v * Dt[5] + (real)3.f * v * Dt[4];
      if (n1 == 3 && n2 == 2)
        return ipow(u, 3) * v * v * Dt[6] + ipow(u, 3) * Dt[5] + (real)3.f * u * v * v * Dt[5] +
               (real)3.f * u * Dt[4];
      if (n1 == 3) return ipow(u, 3) * v * w * Dt[6] + (real)3.f * u * v * w * Dt[5];
      (void)n3;
      return w * u * u * v * v * Dt[6] + w * u * u * Dt[5] + w * v * v * Dt[5] + w * Dt[4];
  }
}

/* gravity_M2P: F_000 -= M_000 D_000, ... with the sign of each order as the
 * reference writes it (orders 0, 2, 4 subtract; order 3 adds), i.e.
 * F = -sum_n (-1)^|n| M_n D_n and F_e = -sum_n (-1)^|n| M_n D_(n+e). */
static void grav_m2p(const struct oracle_multipole *m, real r_x, real r_y, real r_z, real r2,
                     real eps, int periodic, real r_s_inv, real F[4]) {
  const real r_inv = (real)1.f / SQRT(r2);
  struct m2p_derivs d;
  m2p_radial(r_x, r_y, r_z, r2, r_inv, eps, periodic, r_s_inv, &d);
  F[0] = F[1] = F[2] = F[3] = (real)0.f;
  for (int t = 0; t < 35; t++) {
    if (t >= 1 && t <= 3) continue;
    const int a = mp_a[t], b = mp_b[t], c = mp_c[t];
    const real M = ((a + b + c) & 1) ? -(real)m->M[t] : (real)m->M[t];
    F[0] -= M * m2p_D(&d, a, b, c);
    F[1] -= M * m2p_D(&d, a + 1, b, c);
    F[2] -= M * m2p_D(&d, a, b + 1, c);
    F[3] -= M * m2p_D(&d, a, b, c + 1);
  }
}

/* P2P of the (active) particles of gi against all of gj (no multipoles):
 * runner_dopair_grav_pp_full / _truncated (runner_doiact_grav.c:584-760),
 * on gravity caches (gravity_cache.h:310-379): positions relative to `shift`
 * cast to float, inhibited -> mass 0 / inactive; truncated selects the
 * erfc-like long-range factor. self: j == i skipped
 * (runner_doself_grav_pp_full, runner_doiact_grav.c:1500-1622). */
static long long grav_pp(struct gpart *gi, int ni, const struct gpart *gj, int nj,
                         int self, int truncated, const double shift_i[3],
                         const double shift_j[3], const struct oracle_grav_params *G,
                         const struct oracle_multipole *mj, long long *n_m2p) {
  long long n = 0;
  const real dim[3] = {(real)G->dim[0], (real)G->dim[1], (real)G->dim[2]};
  for (int pid = 0; pid < ni; pid++) {
    struct gpart *gp = &gi[pid];
    if (gp->time_bin == time_bin_inhibited) continue;
    if (gp->time_bin > G->max_active_bin) continue;
    const real x_i = (real)(gp->x[0] - shift_i[0]);
    const real y_i = (real)(gp->x[1] - shift_i[1]);
    const real z_i = (real)(gp->x[2] - shift_i[2]);
    const real h_i = gp->epsilon;
    real a_x = 0, a_y = 0, a_z = 0, pot = 0;
    if (mj) {
      /* gravity_cache_populate's use_mpole, then runner_dopair_grav_pm_*
       * (runner_doiact_grav.c:911-1200): dx = CoM_j - x_i, softening
       * max(eps_i, multipole max softening), truncated as the pair */
      const float xf[3] = {(float)(gp->x[0] - shift_i[0]), (float)(gp->x[1] - shift_i[1]),
                           (float)(gp->x[2] - shift_i[2])};
      if (m2p_accept(G, gp, mj, xf, G->periodic)) {
        real dx[3];
        for (int k = 0; k < 3; k++) {
          dx[k] = (real)(mj->CoM[k] - shift_j[k]) - (real)(gp->x[k] - shift_i[k]);
          if (G->periodic) dx[k] = nearest_r(dx[k], dim[k]);
        }
        const real r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
        const real eps = rmax(h_i, (real)mj->max_softening);
        real F[4];
        grav_m2p(mj, dx[0], dx[1], dx[2], r2, eps, truncated, (real)G->r_s_inv, F);
        gp->a_grav[0] += (float)F[1];
        gp->a_grav[1] += (float)F[2];
        gp->a_grav[2] += (float)F[3];
        gp->potential += (float)F[0];
        if (n_m2p) (*n_m2p)++;
        continue;
      }
    }
    for (int pjd = 0; pjd < nj; pjd++) {
      if (self && pid == pjd) continue;
      const struct gpart *gq = &gj[pjd];
      const real mass_j = (gq->time_bin == time_bin_inhibited) ? (real)0 : (real)gq->mass;
      real dx = (real)(gq->x[0] - shift_j[0]) - x_i;
      real dy = (real)(gq->x[1] - shift_j[1]) - y_i;
      real dz = (real)(gq->x[2] - shift_j[2]) - z_i;
      if (G->periodic && !self) {
        dx = nearest_r(dx, dim[0]);
        dy = nearest_r(dy, dim[1]);
        dz = nearest_r(dz, dim[2]);
      }
      const real r2 = dx * dx + dy * dy + dz * dz;
      const real h = rmax(h_i, (real)gq->epsilon);
      const real h2 = h * h;
      const real h_inv = (real)1.f / h;
      const real h_inv_3 = h_inv * h_inv * h_inv;
      real f_ij, pot_ij;
      if (truncated)
        iact_grav_pp_truncated(r2, h2, h_inv, h_inv_3, mass_j, (real)G->r_s_inv, &f_ij,
                               &pot_ij);
      else
        iact_grav_pp_full(r2, h2, h_inv, h_inv_3, mass_j, &f_ij, &pot_ij);
      a_x += f_ij * dx;
      a_y += f_ij * dy;
      a_z += f_ij * dz;
      pot += pot_ij;
      n++;
    }
    /* gravity_cache_write_back (gravity_cache.h:488-511): a_grav += cache */
    gp->a_grav[0] += (float)a_x;
    gp->a_grav[1] += (float)a_y;
    gp->a_grav[2] += (float)a_z;
    gp->potential += (float)pot;
  }
  return n;
}

/* All P2P tasks of a step over leaf cells at once: leaves[i] = {start,count}
 * ranges of `g`; for i-leaf l the source leaves are pairs[off[l]..off[l+1])
 * as {j, truncated}. Each active i accumulates over every source leaf in
 * `real` and is written back once (the per-task float write-back of
 * gravity_cache_write_back would add float rounding of every partial sum).
 * Positions: direct differences, nearest image when periodic. */
static long long PFX(grav_pp_leaves_impl)(struct gpart *g, const int *leaves, int nleaves,
                                          const int *off, const int *pairs,
                                          const struct oracle_grav_params *G,
                                          const struct oracle_multipole *mp, long long *n_m2p,
                                          long long *n_trunc) {
  long long total = 0, total_m2p = 0, total_trunc = 0;
  const real dim[3] = {(real)G->dim[0], (real)G->dim[1], (real)G->dim[2]};
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total, total_m2p, total_trunc)
  for (int l = 0; l < nleaves; l++) {
    /* a "leaf" without entries is left alone: in a tree's cell list the
     * split cells overlap their progeny's ranges, and another thread's
     * update of those gparts must not be overwritten by a += 0 */
    if (off[l] == off[l + 1]) continue;
    const int s = leaves[2 * l], c = leaves[2 * l + 1];
    for (int pid = s; pid < s + c; pid++) {
      struct gpart *gp = &g[pid];
      if (gp->time_bin == time_bin_inhibited || gp->time_bin > G->max_active_bin) continue;
      real a_x = 0, a_y = 0, a_z = 0, pot = 0;
      const real h_i = gp->epsilon;
      for (int q = off[l]; q < off[l + 1]; q++) {
        /* pairs: {j, truncated, allow_mpole} (swh_leaf_pair) */
        const int jl = pairs[3 * q], trunc = pairs[3 * q + 1], allow = pairs[3 * q + 2];
        const int sj = leaves[2 * jl], cj = leaves[2 * jl + 1];
        if (allow && mp && cj > 1) {
          const struct oracle_multipole *B = &mp[jl];
          const float xf[3] = {(float)gp->x[0], (float)gp->x[1], (float)gp->x[2]};
          if (m2p_accept(G, gp, B, xf, G->periodic)) {
            real dx[3];
            for (int k = 0; k < 3; k++) {
              dx[k] = (real)(B->CoM[k] - gp->x[k]);
              if (G->periodic) dx[k] = nearest_r(dx[k], dim[k]);
            }
            const real r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
            real F[4];
            grav_m2p(B, dx[0], dx[1], dx[2], r2, rmax(h_i, (real)B->max_softening), trunc,
                     (real)G->r_s_inv, F);
            a_x += F[1];
            a_y += F[2];
            a_z += F[3];
            pot += F[0];
            total_m2p++;
            continue;
          }
        }
        for (int pjd = sj; pjd < sj + cj; pjd++) {
          if (pjd == pid) continue;
          const struct gpart *gq = &g[pjd];
          const real mass_j = (gq->time_bin == time_bin_inhibited) ? (real)0 : (real)gq->mass;
          real dx = (real)(gq->x[0] - gp->x[0]);
          real dy = (real)(gq->x[1] - gp->x[1]);
          real dz = (real)(gq->x[2] - gp->x[2]);
          if (G->periodic) {
            dx = nearest_r(dx, dim[0]);
            dy = nearest_r(dy, dim[1]);
            dz = nearest_r(dz, dim[2]);
          }
          const real r2 = dx * dx + dy * dy + dz * dz;
          const real h = rmax(h_i, (real)gq->epsilon);
          const real h_inv = (real)1.f / h;
          const real h_inv_3 = h_inv * h_inv * h_inv;
          real f_ij, pot_ij;
          if (trunc)
            iact_grav_pp_truncated(r2, h * h, h_inv, h_inv_3, mass_j, (real)G->r_s_inv,
                                   &f_ij, &pot_ij);
          else
            iact_grav_pp_full(r2, h * h, h_inv, h_inv_3, mass_j, &f_ij, &pot_ij);
          a_x += f_ij * dx;
          a_y += f_ij * dy;
          a_z += f_ij * dz;
          pot += pot_ij;
          total++;
          total_trunc += trunc ? 1 : 0;
        }
      }
      gp->a_grav[0] += (float)a_x;
      gp->a_grav[1] += (float)a_y;
      gp->a_grav[2] += (float)a_z;
      gp->potential += (float)pot;
    }
  }
  if (n_m2p) *n_m2p = total_m2p;
  if (n_trunc) *n_trunc = total_trunc;
  return total;
}

API long long PFX(grav_pp_leaves)(struct gpart *g, const int *leaves, int nleaves,
                                  const int *off, const int *pairs,
                                  const struct oracle_grav_params *G,
                                  const struct oracle_multipole *mp, long long *n_m2p) {
  return PFX(grav_pp_leaves_impl)(g, leaves, nleaves, off, pairs, G, mp, n_m2p, NULL);
}

/* runner_doself_grav_pp (runner_doiact_grav.c:1788-1871): cache frame =
 * cell centre; truncated iff periodic && 2*r_max > r_cut_min. */
API long long PFX(grav_self_pp)(struct gpart *g, int n, const double loc[3],
                                const double width[3], double r_max,
                                const struct oracle_grav_params *G) {
  const double c[3] = {loc[0] + 0.5 * width[0], loc[1] + 0.5 * width[1],
                       loc[2] + 0.5 * width[2]};
  const int truncated = G->periodic && (2. * r_max > G->r_cut_min);
  return grav_pp(g, n, g, n, 1, truncated, c, c, G, NULL, NULL);
}

/* runner_dopair_grav_pp (runner_doiact_grav.c:1202-1425): absolute float
 * positions, nearest-image dx when periodic; truncated iff periodic &&
 * |CoM_i - CoM_j| + rmax_i + rmax_j > r_cut_min. Updates gi (and gj when
 * symmetric). With allow_mpole (mi, mj non-NULL) a cell of more than one
 * particle offers its multipole to the other cell's particles (1273-1274). */
API long long PFX(grav_pair_pp_mpole)(struct gpart *gi, int ni, struct gpart *gj, int nj,
                                      const struct oracle_multipole *mi,
                                      const struct oracle_multipole *mj, int symmetric,
                                      int allow_mpole, const struct oracle_grav_params *G,
                                      long long *n_m2p) {
  const double zero[3] = {0., 0., 0.};
  int truncated = 0;
  if (G->periodic) {
    double dx[3];
    for (int k = 0; k < 3; k++) {
      dx[k] = (float)mj->CoM[k] - (float)mi->CoM[k];
      dx[k] = nearest_r((real)dx[k], (real)G->dim[k]);
    }
    const double r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
    truncated = (sqrt(r2) + (float)mi->r_max + (float)mj->r_max) > G->r_cut_min;
  }
  const struct oracle_multipole *use_j = (allow_mpole && nj > 1) ? mj : NULL;
  const struct oracle_multipole *use_i = (allow_mpole && ni > 1) ? mi : NULL;
  long long n = grav_pp(gi, ni, gj, nj, 0, truncated, zero, zero, G, use_j, n_m2p);
  if (symmetric) n += grav_pp(gj, nj, gi, ni, 0, truncated, zero, zero, G, use_i, n_m2p);
  return n;
}

API long long PFX(grav_pair_pp)(struct gpart *gi, int ni, struct gpart *gj, int nj,
                                const double CoM_i[3], const double CoM_j[3],
                                double rmax_i, double rmax_j, int symmetric,
                                const struct oracle_grav_params *G) {
  const double zero[3] = {0., 0., 0.};
  int truncated = 0;
  if (G->periodic) {
    double dx[3];
    for (int k = 0; k < 3; k++) {
      dx[k] = (float)CoM_j[k] - (float)CoM_i[k];
      dx[k] = nearest_r((real)dx[k], (real)G->dim[k]);
    }
    const double r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
    truncated = (sqrt(r2) + rmax_i + rmax_j) > G->r_cut_min;
  }
  long long n = grav_pp(gi, ni, gj, nj, 0, truncated, zero, zero, G, NULL, NULL);
  if (symmetric) n += grav_pp(gj, nj, gi, ni, 0, truncated, zero, zero, G, NULL, NULL);
  return n;
}

/* ------------------------------------------------------------------------ */
/* Tree gravity: runner_doself_recursive_grav / runner_dopair_recursive_grav */
/* (src/runner_doiact_grav.c:2208-2431) over a cell tree, M2L                */
/* (gravity_M2L_nonsym / _symmetric + gravity_M2L_apply, multipole.h:        */
/* 1600-2095, with gravity_M2L_accept_symmetric, multipole_accept.h:78-199), */
/* and runner_do_grav_down (runner_doiact_grav.c:65-164: gravity_L2L,        */
/* gravity_L2P). Cell multipoles: gravity_P2M over each cell's gparts.       */
/* P-P entries run through grav_pp_leaves (above).                           */
/* ------------------------------------------------------------------------ */
struct oracle_gcell {
  int start, count, split, progeny[8];
  int reserved;
  double loc[3], width[3];
};

struct otree_walk {
  const struct oracle_gcell *cells;
  const struct oracle_multipole *mp;
  const char *act;
  const unsigned char *own; /* NULL: every cell owned (the decomposition stand-in) */
  const struct oracle_grav_params *G;
  int *pp;      /* entries of 4 ints: i-cell, j-cell, truncated, allow_mpole */
  long long npp, cap_pp;
  int *mm;      /* entries of 3 ints: target, source, symmetric */
  long long nmm, cap_mm;
  long long skipped;
};

static void otw_push_pp(struct otree_walk *w, int i, int j, int tr, int allow) {
  if (w->npp == w->cap_pp) {
    w->cap_pp = w->cap_pp ? 2 * w->cap_pp : 1024;
    w->pp = (int *)realloc(w->pp, sizeof(int) * 4 * (size_t)w->cap_pp);
  }
  int *e = w->pp + 4 * w->npp++;
  e[0] = i; e[1] = j; e[2] = tr; e[3] = allow;
}

static void otw_push_mm(struct otree_walk *w, int t, int s, int sym) {
  if (w->nmm == w->cap_mm) {
    w->cap_mm = w->cap_mm ? 2 * w->cap_mm : 1024;
    w->mm = (int *)realloc(w->mm, sizeof(int) * 3 * (size_t)w->cap_mm);
  }
  int *e = w->mm + 3 * w->nmm++;
  e[0] = t; e[1] = s; e[2] = sym;
}

/* gravity_M2L_accept (multipole_accept.h:78-176), float, p = 2 */
static int m2l_accept_o(const struct oracle_grav_params *G, const struct oracle_multipole *A,
                        const struct oracle_multipole *B, float r2) {
  const float rho_A = (float)A->r_max, rho_B = (float)B->r_max;
  const float rho_max = rho_A > rho_B ? rho_A : rho_B;
  const float max_softening =
      A->max_softening > B->max_softening ? A->max_softening : B->max_softening;
  /* sum_n binomial(2, n) power_B[n] integer_powf(rho_A, 2 - n) */
  const int binom[3] = {1, 2, 1};
  const float rpow[3] = {rho_A * rho_A, rho_A, 1.f};
  float E_BA_term = 0.f;
  for (int n = 0; n <= 2; n++) E_BA_term += (float)binom[n] * B->power[n] * rpow[n];
  E_BA_term *= 8.f;
  if (rho_A + rho_B > 0.f) {
    E_BA_term *= rho_max;
    E_BA_term /= (rho_A + rho_B);
  }
  const float r_to_p = r2;
  float f_MAC_inv = r2;
  if (G->periodic && G->consider_truncation_in_MAC) {
    const float H = max_softening;
    if (r2 < (25.f / 81.f) * H * H)
      f_MAC_inv = (25.f / 81.f) * H * H;
    else if (G->r_s_inv * G->r_s_inv * r2 > (25.f / 9.f))
      f_MAC_inv = (9.f / 25.f) * G->r_s_inv * G->r_s_inv * r2 * r2;
  }
  const float min_a_grav = A->min_old_a_grav_norm;
  const float M_max = A->M[0] > B->M[0] ? A->M[0] : B->M[0];
  const float eps = G->adaptive_tolerance;
  const float theta_crit2 = G->theta_crit * G->theta_crit;
  const float rho_sum = rho_A + rho_B;
  const int cond_2 = G->use_tree_below_softening || max_softening * max_softening < r2;
  if (G->use_advanced_MAC && G->use_gadget_tolerance) {
    const float q = rho_max / sqrtf(r2);
    const float ratio = q * q * q;
    return (M_max * ratio < eps * min_a_grav * f_MAC_inv) && cond_2;
  } else if (G->use_advanced_MAC) {
    const int cond_1 = rho_sum * rho_sum < r2;
    const int cond_3 = E_BA_term < eps * min_a_grav * r_to_p * f_MAC_inv;
    return cond_1 && cond_2 && cond_3;
  }
  return (rho_sum * rho_sum < theta_crit2 * r2) && cond_2;
}

static void otw_self(struct otree_walk *w, int c);
static void otw_pair(struct otree_walk *w, int ci, int cj);

/* an entry for cell c: active, and owned by this rank when the step is
 * sharded (runner_do*_grav run by the rank owning the i-cell) */
static int otw_emits(const struct otree_walk *w, int c) {
  return w->act[c] && (!w->own || w->own[c]);
}

static void otw_no_cache(struct otree_walk *w, int ci, int cj) {
  if (!otw_emits(w, ci)) return;
  if (w->cells[ci].count == 0 || w->cells[cj].count == 0) return;
  if (w->cells[ci].split) {
    for (int k = 0; k < 8; k++)
      if (w->cells[ci].progeny[k] >= 0) otw_no_cache(w, w->cells[ci].progeny[k], cj);
  } else {
    otw_push_pp(w, ci, cj, w->G->periodic ? 1 : 0, 0);
  }
}

static void otw_self(struct otree_walk *w, int c) {
  if (!otw_emits(w, c)) return;
  const struct oracle_gcell *C = &w->cells[c];
  if (C->split) {
    for (int j = 0; j < 8; j++) {
      if (C->progeny[j] < 0) continue;
      otw_self(w, C->progeny[j]);
      for (int k = j + 1; k < 8; k++)
        if (C->progeny[k] >= 0) otw_pair(w, C->progeny[j], C->progeny[k]);
    }
  } else {
    otw_push_pp(w, c, c, w->G->periodic && (2. * w->mp[c].r_max > w->G->r_cut_min), 0);
  }
}

static void otw_pair(struct otree_walk *w, int ci, int cj) {
  const struct oracle_grav_params *G = w->G;
  if (!(otw_emits(w, ci) || otw_emits(w, cj))) return;
  const struct oracle_multipole *A = &w->mp[ci], *B = &w->mp[cj];
  double d[3];
  for (int k = 0; k < 3; k++) {
    d[k] = A->CoM[k] - B->CoM[k];
    if (G->periodic) d[k] = nearest(d[k], (double)G->dim[k]);
  }
  const double r2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
  const double r_lr_check = sqrt(r2) - (A->r_max + B->r_max);
  if (G->periodic && r_lr_check > G->r_cut_max) {
    w->skipped++;
    return;
  }
  const struct oracle_gcell *Ci = &w->cells[ci], *Cj = &w->cells[cj];
  if (Ci->count <= 1 || Cj->count <= 1) {
    otw_no_cache(w, ci, cj);
    otw_no_cache(w, cj, ci);
  } else if (m2l_accept_o(G, A, B, (float)r2) && m2l_accept_o(G, B, A, (float)r2)) {
    /* runner_dopair_grav_mm: symmetric when both are active */
    const int sym = w->act[ci] && w->act[cj];
    if (otw_emits(w, ci)) otw_push_mm(w, ci, cj, sym);
    if (otw_emits(w, cj)) otw_push_mm(w, cj, ci, sym);
  } else if (!Ci->split && !Cj->split) {
    /* runner_dopair_grav_pp(ci, cj, 1, 1) */
    int tr = 0;
    if (G->periodic) {
      double dd[3];
      for (int k = 0; k < 3; k++) {
        dd[k] = (float)B->CoM[k] - (float)A->CoM[k];
        dd[k] = nearest_r((real)dd[k], (real)G->dim[k]);
      }
      const double rr2 = dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2];
      tr = (sqrt(rr2) + (float)A->r_max + (float)B->r_max) > G->r_cut_min;
    }
    if (otw_emits(w, ci)) otw_push_pp(w, ci, cj, tr, 1);
    if (otw_emits(w, cj)) otw_push_pp(w, cj, ci, tr, 1);
  } else if (A->r_max > B->r_max) {
    if (Ci->split) {
      for (int k = 0; k < 8; k++)
        if (Ci->progeny[k] >= 0) otw_pair(w, Ci->progeny[k], cj);
    } else {
      for (int k = 0; k < 8; k++)
        if (Cj->progeny[k] >= 0) otw_pair(w, ci, Cj->progeny[k]);
    }
  } else {
    if (Cj->split) {
      for (int k = 0; k < 8; k++)
        if (Cj->progeny[k] >= 0) otw_pair(w, ci, Cj->progeny[k]);
    } else {
      for (int k = 0; k < 8; k++)
        if (Ci->progeny[k] >= 0) otw_pair(w, Ci->progeny[k], cj);
    }
  }
}

static int mp_idx(int a, int b, int c) {
  for (int t = 0; t < 35; t++)
    if (mp_a[t] == a && mp_b[t] == b && mp_c[t] == c) return t;
  return -1;
}

static double xpow_o(const double dx[3], int t) {
  const int a = mp_a[t], b = mp_b[t], c = mp_c[t];
  return pow(dx[0], a) * pow(dx[1], b) * pow(dx[2], c) / (fact_d(a) * fact_d(b) * fact_d(c));
}

/* Field tensors of the whole walk: F (35 per cell, real) after the down
 * pass; stats = {n_pp, n_m2p, n_m2l, n_pp_tasks, n_skipped}. The gparts'
 * a_grav / potential receive P2P + M2P (grav_pp_leaves) and L2P. */
/* gravity_M2L_nonsym / gravity_M2L_symmetric + gravity_M2L_apply
 * (multipole.h:1600-2095): source A's field tensor at target B's CoM added
 * into Ft; sym: softening max(eps_A, eps_B), else eps_A. */
static void m2l_add(const struct oracle_grav_params *G, const struct oracle_multipole *Bm,
                    const struct oracle_multipole *Am, int sym, real *Ft) {
  real dx[3];
  for (int k = 0; k < 3; k++) {
    dx[k] = (real)(Bm->CoM[k] - Am->CoM[k]);
    if (G->periodic) dx[k] = nearest_r(dx[k], (real)G->dim[k]);
  }
  const real r2 = dx[0] * dx[0] + dx[1] * dx[1] + dx[2] * dx[2];
  const real r_inv = (real)(1. / SQRT(r2));
  const float eps_f = sym ? (Am->max_softening > Bm->max_softening ? Am->max_softening
                                                                   : Bm->max_softening)
                          : Am->max_softening;
  struct m2p_derivs d;
  m2p_radial(dx[0], dx[1], dx[2], r2, r_inv, (real)eps_f, G->periodic, (real)G->r_s_inv, &d);
  for (int kk = 0; kk < 35; kk++) {
    const int ok = mp_a[kk] + mp_b[kk] + mp_c[kk];
    for (int nn = 0; nn < 35; nn++) {
      if (nn >= 1 && nn <= 3) continue; /* dipole about the CoM */
      const int on = mp_a[nn] + mp_b[nn] + mp_c[nn];
      if (ok + on > 4) continue;
      Ft[kk] += (real)Am->M[nn] *
                m2p_D(&d, mp_a[kk] + mp_a[nn], mp_b[kk] + mp_b[nn], mp_c[kk] + mp_c[nn]);
    }
  }
}

/* M-M pairs {target, source, symmetric} of explicit multipoles (the
 * reference's runner_dopair_grav_mm_progenies / runner_do_grav_long_range
 * M-M calls, runner_doiact_grav.c:1881-2095, 2441-2530): F[35 t ..] = the
 * sums in pair order (zeroed first). */
API void PFX(grav_m2l_pairs)(const struct oracle_grav_params *G,
                             const struct oracle_multipole *mp, int nmp, const int *pairs,
                             int npairs, double *F) {
  memset(F, 0, sizeof(double) * 35 * (size_t)nmp);
  real Ft[35];
  for (int q = 0; q < npairs; q++) {
    const int t = pairs[3 * q], so = pairs[3 * q + 1], sym = pairs[3 * q + 2];
    for (int k = 0; k < 35; k++) Ft[k] = (real)F[35 * (size_t)t + k];
    m2l_add(G, &mp[t], &mp[so], sym, Ft);
    for (int k = 0; k < 35; k++) F[35 * (size_t)t + k] = (double)Ft[k];
  }
}

/* gravity_M2L_accept_symmetric (multipole_accept.h:190-205) */
API int PFX(grav_m2l_accept_symmetric)(const struct oracle_grav_params *G,
                                       const struct oracle_multipole *A,
                                       const struct oracle_multipole *B, double r2) {
  return m2l_accept_o(G, A, B, (float)r2) && m2l_accept_o(G, B, A, (float)r2);
}

/* owned (NULL: every cell): the decomposition stand-in of
 * swh_gspace_set_owned_cells -- entries only for owned targets */
API void PFX(grav_tree_owned)(struct gpart *g, int n, const struct oracle_gcell *cells,
                              int ncells, const int *self_cells, int nself, const int *pair_cells,
                              int npair, const struct oracle_grav_params *G, long long *stats,
                              float *ftens, const unsigned char *owned) {
  (void)n;
  struct oracle_multipole *mp =
      (struct oracle_multipole *)malloc(sizeof(struct oracle_multipole) * (size_t)ncells);
  char *act = (char *)calloc((size_t)ncells, 1);
  int *parent = (int *)malloc(sizeof(int) * (size_t)ncells);
  for (int c = 0; c < ncells; c++) parent[c] = -1;
  for (int c = 0; c < ncells; c++) {
    for (int k = 0; k < cells[c].count; k++) {
      const struct gpart *gp = &g[cells[c].start + k];
      if (gp->time_bin != time_bin_inhibited && gp->time_bin <= G->max_active_bin) act[c] = 1;
    }
    if (cells[c].split)
      for (int k = 0; k < 8; k++)
        if (cells[c].progeny[k] >= 0) parent[cells[c].progeny[k]] = c;
  }
  /* multipoles as space_split makes them: P2M at the leaves, M2M upwards
   * (children before parents: deepest cells first) */
  {
    int *dep = (int *)malloc(sizeof(int) * (size_t)(ncells > 0 ? ncells : 1));
    int maxdep = 0;
    for (int c = 0; c < ncells; c++) {
      int d = 0;
      for (int x = c; parent[x] >= 0; x = parent[x]) d++;
      dep[c] = d;
      if (d > maxdep) maxdep = d;
    }
    for (int d = maxdep; d >= 0; d--)
#pragma omp parallel for schedule(dynamic, 64)
      for (int c = 0; c < ncells; c++) {
        if (dep[c] != d) continue;
        if (!cells[c].split) {
          PFX(grav_p2m)(g + cells[c].start, cells[c].count, &mp[c]);
        } else {
          const struct oracle_multipole *kids[8];
          int nk = 0;
          for (int k = 0; k < 8; k++)
            if (cells[c].progeny[k] >= 0) kids[nk++] = &mp[cells[c].progeny[k]];
          PFX(grav_m2m)(kids, nk, cells[c].loc, cells[c].width, &mp[c]);
        }
      }
    free(dep);
  }
  struct otree_walk w;
  memset(&w, 0, sizeof(w));
  w.cells = cells;
  w.mp = mp;
  w.act = act;
  w.own = owned;
  w.G = G;
  /* the recursive tasks (independent, as SWIFT's runners execute them,
   * runner_main.c:207-208, 257-258) over the threads in chunks of 64
   * consecutive tasks; the chunks' entries are joined in task order, so the
   * lists equal a serial walk's */
  {
    const long long ntask = (long long)nself + npair, kChunk = 64;
    const long long nchunk = (ntask + kChunk - 1) / kChunk;
    struct otree_walk *part =
        (struct otree_walk *)calloc((size_t)(nchunk > 0 ? nchunk : 1), sizeof(struct otree_walk));
#pragma omp parallel for schedule(dynamic, 1)
    for (long long ch = 0; ch < nchunk; ch++) {
      struct otree_walk *pw = &part[ch];
      *pw = w;
      pw->pp = NULL;
      pw->mm = NULL;
      pw->npp = pw->cap_pp = pw->nmm = pw->cap_mm = pw->skipped = 0;
      const long long t1 = (ch + 1) * kChunk < ntask ? (ch + 1) * kChunk : ntask;
      for (long long t = ch * kChunk; t < t1; t++) {
        if (t < nself) otw_self(pw, self_cells[t]);
        else otw_pair(pw, pair_cells[2 * (t - nself)], pair_cells[2 * (t - nself) + 1]);
      }
    }
    long long npp = 0, nmm = 0;
    for (long long ch = 0; ch < nchunk; ch++) {
      npp += part[ch].npp;
      nmm += part[ch].nmm;
      w.skipped += part[ch].skipped;
    }
    w.pp = (int *)malloc(sizeof(int) * 4 * (size_t)(npp > 0 ? npp : 1));
    w.mm = (int *)malloc(sizeof(int) * 3 * (size_t)(nmm > 0 ? nmm : 1));
    for (long long ch = 0; ch < nchunk; ch++) {
      if (part[ch].npp)
        memcpy(w.pp + 4 * w.npp, part[ch].pp, sizeof(int) * 4 * (size_t)part[ch].npp);
      if (part[ch].nmm)
        memcpy(w.mm + 3 * w.nmm, part[ch].mm, sizeof(int) * 3 * (size_t)part[ch].nmm);
      w.npp += part[ch].npp;
      w.nmm += part[ch].nmm;
      free(part[ch].pp);
      free(part[ch].mm);
    }
    w.cap_pp = w.npp;
    w.cap_mm = w.nmm;
    free(part);
  }
  /* P-P: CSR over i-cells in walk order per cell */
  int *leaves = (int *)malloc(sizeof(int) * 2 * (size_t)ncells);
  int *off = (int *)calloc((size_t)ncells + 1, sizeof(int));
  int *pairs = (int *)malloc(sizeof(int) * 3 * (size_t)(w.npp > 0 ? w.npp : 1));
  for (int c = 0; c < ncells; c++) {
    leaves[2 * c] = cells[c].start;
    leaves[2 * c + 1] = cells[c].count;
  }
  for (long long q = 0; q < w.npp; q++) off[w.pp[4 * q] + 1]++;
  for (int c = 0; c < ncells; c++) off[c + 1] += off[c];
  int *fill = (int *)malloc(sizeof(int) * (size_t)(ncells > 0 ? ncells : 1));
  memcpy(fill, off, sizeof(int) * (size_t)ncells);
  for (long long q = 0; q < w.npp; q++) {
    const int i = w.pp[4 * q];
    int *e = pairs + 3 * fill[i]++;
    e[0] = w.pp[4 * q + 1];
    e[1] = w.pp[4 * q + 2];
    e[2] = w.pp[4 * q + 3];
  }
  long long n_m2p = 0, n_trunc = 0;
  const long long n_pp =
      PFX(grav_pp_leaves_impl)(g, leaves, ncells, off, pairs, G, mp, &n_m2p, &n_trunc);
  /* M2L (field tensor at the target's CoM) */
  real *F = (real *)calloc((size_t)ncells * 35, sizeof(real));
  /* by target (a stable counting sort: each target sums its sources in walk
   * order, so the threads change no result) */
  long long *moff = (long long *)calloc((size_t)ncells + 1, sizeof(long long));
  long long *mord = (long long *)malloc(sizeof(long long) * (size_t)(w.nmm > 0 ? w.nmm : 1));
  for (long long q = 0; q < w.nmm; q++) moff[w.mm[3 * q] + 1]++;
  for (int c = 0; c < ncells; c++) moff[c + 1] += moff[c];
  {
    long long *mfill = (long long *)malloc(sizeof(long long) * (size_t)(ncells > 0 ? ncells : 1));
    memcpy(mfill, moff, sizeof(long long) * (size_t)ncells);
    for (long long q = 0; q < w.nmm; q++) mord[mfill[w.mm[3 * q]]++] = q;
    free(mfill);
  }
#pragma omp parallel for schedule(dynamic, 16)
  for (int tc = 0; tc < ncells; tc++)
  for (long long qq = moff[tc]; qq < moff[tc + 1]; qq++) {
    const long long q = mord[qq];
    const int t = w.mm[3 * q], s = w.mm[3 * q + 1], sym = w.mm[3 * q + 2];
    m2l_add(G, &mp[t], &mp[s], sym, F + 35 * (size_t)t);
  }
  /* down pass: parents before children (depth order), then L2P */
  int *depth = (int *)malloc(sizeof(int) * (size_t)ncells);
  int maxd = 0;
  for (int c = 0; c < ncells; c++) {
    int dd = 0, x = c;
    while (parent[x] >= 0) { x = parent[x]; dd++; }
    depth[c] = dd;
    if (dd > maxd) maxd = dd;
  }
  for (int dd = 1; dd <= maxd; dd++) {
    /* the cells of one depth are independent (each reads only its parent) */
#pragma omp parallel for schedule(dynamic, 64)
    for (int c = 0; c < ncells; c++) {
      if (depth[c] != dd) continue;
      const int p = parent[c];
      const real *Fp = F + 35 * (size_t)p;
      int any = 0;
      for (int t = 0; t < 35; t++) any |= Fp[t] != 0;
      if (!any) continue;
      const double dx[3] = {mp[c].CoM[0] - mp[p].CoM[0], mp[c].CoM[1] - mp[p].CoM[1],
                            mp[c].CoM[2] - mp[p].CoM[2]};
      real *Fc = F + 35 * (size_t)c;
      for (int kk = 0; kk < 35; kk++)
        for (int nn = 0; nn < 35; nn++) {
          const int m = mp_idx(mp_a[kk] + mp_a[nn], mp_b[kk] + mp_b[nn], mp_c[kk] + mp_c[nn]);
          if (m < 0) continue;
          Fc[kk] += (real)xpow_o(dx, nn) * Fp[m];
        }
    }
  }
#pragma omp parallel for schedule(dynamic, 64)
  for (int c = 0; c < ncells; c++) {
    if (cells[c].split) continue;
    const real *Fc = F + 35 * (size_t)c;
    int any = 0;
    for (int t = 0; t < 35; t++) any |= Fc[t] != 0;
    if (!any) continue;
    for (int k = 0; k < cells[c].count; k++) {
      struct gpart *gp = &g[cells[c].start + k];
      if (gp->time_bin == time_bin_inhibited || gp->time_bin > G->max_active_bin) continue;
      const double dx[3] = {gp->x[0] - mp[c].CoM[0], gp->x[1] - mp[c].CoM[1],
                            gp->x[2] - mp[c].CoM[2]};
      double a[3] = {0., 0., 0.}, pot = 0.;
      for (int t = 0; t < 35; t++) {
        const double X = xpow_o(dx, t);
        pot -= X * (double)Fc[t];
        if (mp_a[t] + mp_b[t] + mp_c[t] <= 3) {
          a[0] += X * (double)Fc[mp_idx(mp_a[t] + 1, mp_b[t], mp_c[t])];
          a[1] += X * (double)Fc[mp_idx(mp_a[t], mp_b[t] + 1, mp_c[t])];
          a[2] += X * (double)Fc[mp_idx(mp_a[t], mp_b[t], mp_c[t] + 1)];
        }
      }
      gp->a_grav[0] += (float)a[0];
      gp->a_grav[1] += (float)a[1];
      gp->a_grav[2] += (float)a[2];
      gp->potential += (float)pot;
    }
  }
  if (ftens)
    for (size_t k = 0; k < (size_t)ncells * 35; k++) ftens[k] = (float)F[k];
  if (stats) {
    stats[0] = n_pp;
    stats[1] = n_m2p;
    stats[2] = w.nmm;
    stats[3] = w.npp;
    stats[4] = w.skipped;
    stats[5] = n_trunc; /* P2P pairs of truncated entries (swh_grav_tree_stats.n_pp_truncated) */
  }
  free(F); free(moff); free(mord); free(depth); free(fill); free(pairs); free(off); free(leaves);
  free(w.pp); free(w.mm); free(parent); free(act); free(mp);
}

API void PFX(grav_tree)(struct gpart *g, int n, const struct oracle_gcell *cells, int ncells,
                        const int *self_cells, int nself, const int *pair_cells, int npair,
                        const struct oracle_grav_params *G, long long *stats, float *ftens) {
  PFX(grav_tree_owned)(g, n, cells, ncells, self_cells, nself, pair_cells, npair, G, stats, ftens,
                       NULL);
}

/* ======================================================================== */
/* PM mesh gravity — src/mesh_gravity.c compute_potential_global (844-1041) */
/* on a non-distributed mesh without neutrinos: CIC assignment              */
/* (gpart_to_mesh_CIC, 137-182, CIC_set 103-125), r2c FFT,                  */
/* mesh_apply_Green_function (519-638) with fourier_kernel_long_grav_eval   */
/* (kernel_long_gravity.h:310-319, default sinh branch), c2r FFT, and       */
/* mesh_to_gpart_CIC (308-394: CIC potential, 5-point stencil accelerations)*/
/* + the const_G scaling of mesh_to_gpart_CIC_mapper (428-470). All double, */
/* as the reference, in both oracle builds. FFTW (third-party, not under    */
/* /root/reference) computes the unnormalised DFT; this restates it with a  */
/* plain radix-2 complex transform over the full N^3 spectrum (a plain DFT */
/* for other N, e.g. odd meshes), applying the Green function to every k (the factor is even in each*/
/* component, so the spectrum stays Hermitian and the real part is the c2r */
/* result).                                                                 */
/* ======================================================================== */
static int pm_id(int i, int j, int k, int N) { /* row_major_id_periodic (row_major_id.h:39-43) */
  return ((i + N) % N) * N * N + ((j + N) % N) * N + ((k + N) % N);
}

static void pm_fft_line(double *re, double *im, int n, int sign) {
  if (n & (n - 1)) { /* not a power of two (odd meshes): the plain O(n^2) DFT */
    double *tr = malloc(n * sizeof(double)), *ti = malloc(n * sizeof(double));
    for (int k = 0; k < n; k++) {
      double sr = 0., si = 0.;
      for (int t = 0; t < n; t++) {
        const double ang = sign * 2. * M_PI * (double)(((long long)k * t) % n) / n;
        const double c = cos(ang), sn = sin(ang);
        sr += re[t] * c - im[t] * sn;
        si += re[t] * sn + im[t] * c;
      }
      tr[k] = sr;
      ti[k] = si;
    }
    memcpy(re, tr, n * sizeof(double));
    memcpy(im, ti, n * sizeof(double));
    free(tr);
    free(ti);
    return;
  }
  for (int i = 1, j = 0; i < n; i++) {
    int bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      double t = re[i]; re[i] = re[j]; re[j] = t;
      t = im[i]; im[i] = im[j]; im[j] = t;
    }
  }
  for (int len = 2; len <= n; len <<= 1) {
    const double ang = sign * 2. * M_PI / len;
    for (int i = 0; i < n; i += len)
      for (int k = 0; k < len / 2; k++) {
        const double wr = cos(ang * k), wi = sin(ang * k);
        const int a = i + k, b = i + k + len / 2;
        const double xr = re[b] * wr - im[b] * wi, xi = re[b] * wi + im[b] * wr;
        re[b] = re[a] - xr; im[b] = im[a] - xi;
        re[a] += xr; im[a] += xi;
      }
  }
}

/* sign -1: forward (FFTW_FORWARD, e^{-2 pi i jk/N}); +1: backward, unnormalised */
static void pm_fft3d(double *re, double *im, int N, int sign) {
  double *lr = malloc(N * sizeof(double)), *li = malloc(N * sizeof(double));
  const int st[3] = {N * N, N, 1};
  for (int ax = 0; ax < 3; ax++) {
    const int s = st[ax], o1 = st[(ax + 1) % 3], o2 = st[(ax + 2) % 3];
    for (int a = 0; a < N; a++)
      for (int b = 0; b < N; b++) {
        const int base = a * o1 + b * o2;
        for (int t = 0; t < N; t++) { lr[t] = re[base + t * s]; li[t] = im[base + t * s]; }
        pm_fft_line(lr, li, N, sign);
        for (int t = 0; t < N; t++) { re[base + t * s] = lr[t]; im[base + t * s] = li[t]; }
      }
  }
  free(lr);
  free(li);
}

static double pm_cic_get(const double *pot, int N, int i, int j, int k, double tx, double ty,
                         double tz, double dx, double dy, double dz) { /* CIC_get, 69-85 */
  double temp;
  temp = pot[pm_id(i + 0, j + 0, k + 0, N)] * tx * ty * tz;
  temp += pot[pm_id(i + 0, j + 0, k + 1, N)] * tx * ty * dz;
  temp += pot[pm_id(i + 0, j + 1, k + 0, N)] * tx * dy * tz;
  temp += pot[pm_id(i + 0, j + 1, k + 1, N)] * tx * dy * dz;
  temp += pot[pm_id(i + 1, j + 0, k + 0, N)] * dx * ty * tz;
  temp += pot[pm_id(i + 1, j + 0, k + 1, N)] * dx * ty * dz;
  temp += pot[pm_id(i + 1, j + 1, k + 0, N)] * dx * dy * tz;
  temp += pot[pm_id(i + 1, j + 1, k + 1, N)] * dx * dy * dz;
  return temp;
}

static void pm_cic_coeffs(const double x[3], const double dim[3], int N, double fac, int ijk[3],
                          double t[3], double d[3]) {
  for (int a = 0; a < 3; a++) {
    const double p = x[a] < 0. ? x[a] + dim[a] : (x[a] >= dim[a] ? x[a] - dim[a] : x[a]);
    int i = (int)(fac * p);
    if (i >= N) i = N - 1;
    ijk[a] = i;
    d[a] = fac * p - i;
    t[a] = 1. - d[a];
  }
}

API void PFX(pm_mesh)(struct gpart *g, int n, int N, double box, double r_s, float const_G,
                      double *pot_out) {
  const size_t N3 = (size_t)N * N * N;
  double *re = calloc(N3, sizeof(double)), *im = calloc(N3, sizeof(double));
  const double fac = N / box, dim[3] = {box, box, box};
  /* CIC assignment (gpart_to_mesh_CIC) */
  for (int p = 0; p < n; p++) {
    if (g[p].time_bin == time_bin_inhibited) continue;
    int c[3];
    double t[3], d[3];
    pm_cic_coeffs(g[p].x, dim, N, fac, c, t, d);
    const double value = (double)g[p].mass * 1.0;
    const int i = c[0], j = c[1], k = c[2];
    re[pm_id(i + 0, j + 0, k + 0, N)] += value * t[0] * t[1] * t[2];
    re[pm_id(i + 0, j + 0, k + 1, N)] += value * t[0] * t[1] * d[2];
    re[pm_id(i + 0, j + 1, k + 0, N)] += value * t[0] * d[1] * t[2];
    re[pm_id(i + 0, j + 1, k + 1, N)] += value * t[0] * d[1] * d[2];
    re[pm_id(i + 1, j + 0, k + 0, N)] += value * d[0] * t[1] * t[2];
    re[pm_id(i + 1, j + 0, k + 1, N)] += value * d[0] * t[1] * d[2];
    re[pm_id(i + 1, j + 1, k + 0, N)] += value * d[0] * d[1] * t[2];
    re[pm_id(i + 1, j + 1, k + 1, N)] += value * d[0] * d[1] * d[2];
  }
  pm_fft3d(re, im, N, -1);
  /* mesh_apply_Green_function */
  const double green_fac = -1. / (M_PI * box);
  const double a_smooth2 = 4. * M_PI * M_PI * r_s * r_s / (box * box);
  const double k_fac = M_PI / (double)N;
  const int Nh = N / 2;
  for (int i = 0; i < N; i++) {
    const int kx = i > Nh ? i - N : i;
    const double fx = k_fac * kx;
    const double sx = kx != 0 ? fx / sin(fx) : 1.;
    for (int j = 0; j < N; j++) {
      const int ky = j > Nh ? j - N : j;
      const double fy = k_fac * ky;
      const double sy = ky != 0 ? fy / sin(fy) : 1.;
      for (int k = 0; k < N; k++) {
        const int kz = k > Nh ? k - N : k;
        const double fz = k_fac * kz;
        const double sz = kz != 0 ? fz / (sin(fz) + FLT_MIN) : 1.;
        const double k2 = (double)kx * kx + (double)ky * ky + (double)kz * kz;
        if (k2 == 0.) continue;
        const double u = sqrt(k2 * a_smooth2);
        const double arg = M_PI_2 * u;
        const double W = arg / (sinh(arg) + FLT_MIN);
        const double green_cor = green_fac * W / (k2 + FLT_MIN);
        const double cic = sx * sy * sz, cic2 = cic * cic, cic4 = cic2 * cic2;
        const double tot = green_cor * cic4;
        re[(size_t)i * N * N + j * N + k] *= tot;
        im[(size_t)i * N * N + j * N + k] *= tot;
      }
    }
  }
  re[0] = 0.;
  im[0] = 0.;
  pm_fft3d(re, im, N, +1);
  /* mesh_to_gpart_CIC + const_G */
  for (int p = 0; p < n; p++) {
    struct gpart *gp = &g[p];
    if (gp->time_bin == time_bin_inhibited) continue;
    int c[3];
    double t[3], d[3];
    pm_cic_coeffs(gp->x, dim, N, fac, c, t, d);
    const int i = c[0], j = c[1], k = c[2];
#define PMG(a, b, cc) pm_cic_get(re, N, i + (a), j + (b), k + (cc), t[0], t[1], t[2], d[0], d[1], d[2])
    double pp = 0., a[3] = {0., 0., 0.};
    pp += PMG(0, 0, 0);
    a[0] += (1. / 12.) * PMG(2, 0, 0);
    a[0] -= (2. / 3.) * PMG(1, 0, 0);
    a[0] += (2. / 3.) * PMG(-1, 0, 0);
    a[0] -= (1. / 12.) * PMG(-2, 0, 0);
    a[1] += (1. / 12.) * PMG(0, 2, 0);
    a[1] -= (2. / 3.) * PMG(0, 1, 0);
    a[1] += (2. / 3.) * PMG(0, -1, 0);
    a[1] -= (1. / 12.) * PMG(0, -2, 0);
    a[2] += (1. / 12.) * PMG(0, 0, 2);
    a[2] -= (2. / 3.) * PMG(0, 0, 1);
    a[2] += (2. / 3.) * PMG(0, 0, -1);
    a[2] -= (1. / 12.) * PMG(0, 0, -2);
#undef PMG
    for (int q = 0; q < 3; q++) {
      gp->a_grav_mesh[q] = (float)(fac * a[q]);
      gp->a_grav_mesh[q] *= const_G;
    }
    gp->potential_mesh = 0.f;
    gp->potential_mesh += (float)pp;
    gp->potential_mesh *= const_G;
  }
  if (pot_out) memcpy(pot_out, re, N3 * sizeof(double));
  free(re);
  free(im);
}
