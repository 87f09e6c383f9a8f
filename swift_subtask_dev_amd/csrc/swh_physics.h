// swh_physics.h — device-side SPHENIX physics with the cubic-spline or
// Wendland-C2 SPH kernel (build-time choice), and Wendland-C2 gravity softening,
// templated on the arithmetic type T (double = the fp64 path, float = the
// reference's own precision). Constants are the reference's float values
// (same expressions as the macros they cite), promoted to T.
//
// References (/root/reference/src):
//   kernel_hydro.h:45-64,121-147,195-284   cubic spline, Wendland C2, kernel_deval
//   hydro/SPHENIX/hydro_iact.h     runner_iact_nonsym_{density,gradient,force}
//   hydro/SPHENIX/hydro.h          end_density / prepare_gradient / prepare_force ...
//   kernel_gravity.h:48-100, kernel_long_gravity.h:204-262, gravity/MultiSoftening/gravity_iact.h
#pragma once

#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdint>

namespace swh {

// --- constants: the SPH kernel (3D), gamma = 5/3 ---------------------------
// The kernel is a build-time choice, as SWIFT's configure --with-kernel
// (configure.ac:2107-2137): cubic spline (default, libswifthip.so) or
// Wendland C2 (-DSWH_KERNEL_WENDLAND_C2, libswifthip_wc2.so).
constexpr double kPi = 3.14159265358979323846;
#if defined(SWH_KERNEL_WENDLAND_C2)
// kernel_hydro.h:121-147: degree 5, one branch, W(x) = (1-x)^4 (1+4x)
constexpr float kGamma = (float)(1.936492);
constexpr float kConstant = (float)(21. * (1. / kPi) / 2.);
constexpr float kKernelW0 = 1.f;  // kernel_coeffs[kernel_degree]
#define SWH_KERNEL_NAME "wendland-c2"
#else
// kernel_hydro.h:45-64: degree 3, two branches
constexpr float kGamma = (float)(1.825742);
constexpr float kConstant = (float)(16. * (1. / kPi));
constexpr float kKernelW0 = 0.5f;  // kernel_coeffs[kernel_degree]
#define SWH_KERNEL_NAME "cubic-spline"
#endif
constexpr float kGammaInv = (float)(1. / kGamma);
constexpr float kGamma2 = kGamma * kGamma;
constexpr float kGammaInvDim = (float)(1. / (kGamma * kGamma * kGamma));
constexpr float kGammaInvDimPlusOne = (float)(1. / (kGamma * kGamma * kGamma * kGamma));
constexpr float kRoot = kKernelW0 * kConstant * kGammaInvDim;  // W(0), kernel_root
constexpr float kDim = 3.f;
constexpr float kDimInv = 0.3333333333f;
constexpr float kHydroGamma = 1.66666666666666667f;
constexpr float kHydroGammaMinusOne = 0.66666666666666667f;
constexpr float kViscBeta = 3.0f;
constexpr int kNumTimeBins = 56;
constexpr int kTimeBinInhibited = kNumTimeBins + 2;

template <typename T>
__device__ __forceinline__ T tmax(T a, T b) { return a > b ? a : b; }
template <typename T>
__device__ __forceinline__ T tmin(T a, T b) { return a < b ? a : b; }

template <typename T> __device__ __forceinline__ T tsqrt(T x);
template <> __device__ __forceinline__ double tsqrt<double>(double x) { return sqrt(x); }
template <> __device__ __forceinline__ float tsqrt<float>(float x) { return sqrtf(x); }

// fp64 reciprocal and reciprocal square root: the hardware approximation
// (v_rcp_f64 / v_rsq_f64) refined by two Newton steps to ~1 ulp, a third of
// the instructions of an IEEE division / sqrt. The float path keeps the
// reference's own operations (it is compared with the float oracle).
__device__ __forceinline__ double rcp_f64(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
__device__ __forceinline__ double rsqrt_f64(double x) {  // x > 0
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double e = fma(-h * y, y, 0.5);
  y = fma(y, e, y);
  e = fma(-h * y, y, 0.5);
  return fma(y, e, y);
}
// One-Newton-step forms for the pair loops: v_rcp_f64 / v_rsq_f64 are good
// to ~5e-8 relative on gfx950 and one step takes that to 2e-15 / 4e-15
// (measured over x in [1e-6, 1e6], tools/probe/rcp_acc.hip) -- far below
// the float storage of the results (6e-8) the loops accumulate into.
__device__ __forceinline__ double rcp1_f64(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(r, fma(-x, r, 1.0), r);
}
__device__ __forceinline__ double rsqrt1_f64(double x) {  // x > 0
  const double y = __builtin_amdgcn_rsq(x);
  return fma(y, fma(-0.5 * x * y, y, 0.5), y);
}

// a / b: fp64 through rcp1_f64, float as the reference writes it.
template <typename T> __device__ __forceinline__ T tdiv(T a, T b);
template <> __device__ __forceinline__ double tdiv<double>(double a, double b) {
  return a * rcp1_f64(b);
}
template <> __device__ __forceinline__ float tdiv<float>(float a, float b) { return a / b; }

// r = |dx| and 1/r (0 for r = 0, as the loops' r > 0 guard).
template <typename T> __device__ __forceinline__ void r_and_inv(T r2, T& r, T& r_inv);
template <>
__device__ __forceinline__ void r_and_inv<double>(double r2, double& r, double& r_inv) {
  r_inv = r2 > 0. ? rsqrt1_f64(r2) : 0.;
  r = r2 * r_inv;
}
template <>
__device__ __forceinline__ void r_and_inv<float>(float r2, float& r, float& r_inv) {
  r = sqrtf(r2);
  r_inv = r > 0.f ? 1.f / r : 0.f;
}

// kernel_deval (kernel_hydro.h:257-284): W(u), dW/du from the kernel's
// coefficient table by Horner, the branch index (int)(x * kernel_ivals)
// clamped to kernel_ivals (an all-zero row: outside the support).
template <typename T>
__device__ __forceinline__ void kernel_deval(T u, T& W, T& dW_dx);

#if defined(SWH_KERNEL_WENDLAND_C2)
// fp64: (1-x)^4 (1+4x) and its derivative -20 x (1-x)^3 in closed form
// (equal to the table's Horner form on [0,1), zero beyond).
template <>
__device__ __forceinline__ void kernel_deval<double>(double u, double& W, double& dW_dx) {
  const double x = u * (double)kGammaInv;
  const double t = fmax(1. - x, 0.);
  const double t2 = t * t;
  const double t3 = t2 * t;
  W = t3 * t * fma(4., x, 1.) * ((double)kConstant * (double)kGammaInvDim);
  dW_dx = -20. * x * t3 * ((double)kConstant * (double)kGammaInvDimPlusOne);
}

// float: the reference's Horner evaluation of {4, -15, 20, -10, 0, 1} on
// branch 0 and the zero row beyond (kernel_hydro.h:143-146).
template <>
__device__ __forceinline__ void kernel_deval<float>(float u, float& W, float& dW_dx) {
  using T = float;
  const T x = u * (T)kGammaInv;
  const int temp = (int)(x * (T)1);
  const bool in = (temp > 1 ? 1 : temp) == 0;
  const T c0 = in ? (T)4 : (T)0, c1 = in ? (T)-15 : (T)0, c2 = in ? (T)20 : (T)0;
  const T c3 = in ? (T)-10 : (T)0, c4 = (T)0, c5 = in ? (T)1 : (T)0;
  T w = c0 * x + c1;
  T dw = c0;
  dw = dw * x + w;
  w = x * w + c2;
  dw = dw * x + w;
  w = x * w + c3;
  dw = dw * x + w;
  w = x * w + c4;
  dw = dw * x + w;
  w = x * w + c5;
  w = tmax(w, (T)0);
  dw = tmin(dw, (T)0);
  W = w * (T)kConstant * (T)kGammaInvDim;
  dW_dx = dw * (T)kConstant * (T)kGammaInvDimPlusOne;
}
#else
// fp64: the same piecewise cubic in closed form, w = (1-x)^3_+ - 4 (1/2-x)^3_+
// (equal to the table's Horner forms on [0,1/2) and [1/2,1), zero beyond),
// without the index selects.
template <>
__device__ __forceinline__ void kernel_deval<double>(double u, double& W, double& dW_dx) {
  const double x = u * (double)kGammaInv;
  const double t = fmax(1. - x, 0.);
  const double q = fmax(0.5 - x, 0.);
  const double t2 = t * t, q2 = q * q;
  W = fma(-4. * q2, q, t2 * t) * ((double)kConstant * (double)kGammaInvDim);
  dW_dx = fma(12., q2, -3. * t2) * ((double)kConstant * (double)kGammaInvDimPlusOne);
}

// float: branch 0: u/H < 1/2, branch 1: < 1, branch 2 (outside support):
// all-zero coefficients, picked with selects instead of a table load.
template <>
__device__ __forceinline__ void kernel_deval<float>(float u, float& W, float& dW_dx) {
  using T = float;
  const T x = u * (T)kGammaInv;
  const int temp = (int)(x * (T)2);
  const int ind = temp > 2 ? 2 : temp;
  const T c0 = ind == 0 ? (T)3 : (ind == 1 ? (T)-1 : (T)0);
  const T c1 = ind == 0 ? (T)-3 : (ind == 1 ? (T)3 : (T)0);
  const T c2 = ind == 0 ? (T)0 : (ind == 1 ? (T)-3 : (T)0);
  const T c3 = ind == 0 ? (T)0.5 : (ind == 1 ? (T)1 : (T)0);
  T w = c0 * x + c1;
  T dw = c0;
  dw = dw * x + w;
  w = x * w + c2;
  dw = dw * x + w;
  w = x * w + c3;
  w = tmax(w, (T)0);
  dw = tmin(dw, (T)0);
  W = w * (T)kConstant * (T)kGammaInvDim;
  dW_dx = dw * (T)kConstant * (T)kGammaInvDimPlusOne;
}
#endif

// ---------------------------------------------------------------------------
// Accumulators of one i-particle for each loop (registers for the duration of
// the gather).
// ---------------------------------------------------------------------------
template <typename T>
struct DensityAcc {
  T rho, rho_dh, wcount, wcount_dh, div_v, rot_x, rot_y, rot_z;
  __device__ void zero() { rho = rho_dh = wcount = wcount_dh = div_v = rot_x = rot_y = rot_z = (T)0; }
};

// runner_iact_nonsym_density (hydro_iact.h:130-178). dx = x_i - x_j.
template <typename T>
__device__ __forceinline__ void iact_nonsym_density(T r2, T dx, T dy, T dz, T hi_inv,
                                                    T vix, T viy, T viz, T mj, T vjx,
                                                    T vjy, T vjz, DensityAcc<T>& A) {
  T r, r_inv;
  r_and_inv(r2, r, r_inv);
  const T ui = r * hi_inv;
  T wi, wi_dx;
  kernel_deval(ui, wi, wi_dx);
  A.rho += mj * wi;
  A.rho_dh -= mj * ((T)kDim * wi + ui * wi_dx);
  A.wcount += wi;
  A.wcount_dh -= ((T)kDim * wi + ui * wi_dx);
  const T faci = mj * wi_dx * r_inv;
  const T dvx = vix - vjx, dvy = viy - vjy, dvz = viz - vjz;
  const T dvdr = dvx * dx + dvy * dy + dvz * dz;
  A.div_v -= faci * dvdr;
  A.rot_x += faci * (dvy * dz - dvz * dy);
  A.rot_y += faci * (dvz * dx - dvx * dz);
  A.rot_z += faci * (dvx * dy - dvy * dx);
}

// The fp64 batch loops' form of runner_iact_nonsym_density: the same sums
// with the kernel's constant factors taken out of the per-pair work
// (density_finalize puts them back at the store; fp64 rounding only).
//   A.rho = sum m_j w        A.wcount = sum w           (w  = W / C_W)
//   A.rho_dh = sum m_j u dw  A.wcount_dh = sum u dw     (dw = dW/du / C_dW)
//   A.div_v, A.rot_*: the sums of m_j dw / r (dv . dx), m_j dw / r (dv x dx)
// with x = u / gamma, w = (1 - x)^3_+ - 4 (1/2 - x)^3_+, dw = 12 (1/2 - x)^2_+
// - 3 (1 - x)^2_+ for the cubic spline (Wendland C2: w = (1 - x)^4 (1 + 4x),
// dw = -20 x (1 - x)^3), C_W = kConstant gamma^-3, C_dW = kConstant gamma^-4.
__device__ __forceinline__ void iact_nonsym_density_raw(double r2, double dx, double dy, double dz,
                                                        double hi_inv, double vix, double viy,
                                                        double viz, double mj, double vjx,
                                                        double vjy, double vjz,
                                                        DensityAcc<double>& A) {
  double r, r_inv;
  r_and_inv(r2, r, r_inv);
  const double ui = r * hi_inv;
  const double x = ui * (double)kGammaInv;
  const double t = fmax(1. - x, 0.);
#if defined(SWH_KERNEL_WENDLAND_C2)
  const double t3 = t * t * t;
  const double w = t3 * t * fma(4., x, 1.);
  const double dw = -20. * x * t3;
#else
  const double q = fmax(0.5 - x, 0.);
  const double t2 = t * t, q2 = q * q;
  const double w = fma(-4. * q2, q, t2 * t);
  const double dw = fma(12., q2, -3. * t2);
#endif
  const double udw = ui * dw;
  A.wcount += w;
  A.rho = fma(mj, w, A.rho);
  A.wcount_dh += udw;
  A.rho_dh = fma(mj, udw, A.rho_dh);
  const double faci = mj * dw * r_inv;
  const double dvx = vix - vjx, dvy = viy - vjy, dvz = viz - vjz;
  const double dvdr = dvx * dx + dvy * dy + dvz * dz;
  A.div_v -= faci * dvdr;
  A.rot_x += faci * (dvy * dz - dvz * dy);
  A.rot_y += faci * (dvz * dx - dvx * dz);
  A.rot_z += faci * (dvx * dy - dvy * dx);
}

// The runner_iact_nonsym_density sums from iact_nonsym_density_raw's.
__device__ __forceinline__ DensityAcc<double> density_finalize(const DensityAcc<double>& R) {
  constexpr double cw = (double)kConstant * (double)kGammaInvDim;
  constexpr double cdw = (double)kConstant * (double)kGammaInvDimPlusOne;
  DensityAcc<double> A;
  A.rho = cw * R.rho;
  A.wcount = cw * R.wcount;
  A.rho_dh = -fma((double)kDim * cw, R.rho, cdw * R.rho_dh);
  A.wcount_dh = -fma((double)kDim * cw, R.wcount, cdw * R.wcount_dh);
  A.div_v = cdw * R.div_v;
  A.rot_x = cdw * R.rot_x;
  A.rot_y = cdw * R.rot_y;
  A.rot_z = cdw * R.rot_z;
  return A;
}

template <typename T>
struct GradientAcc {
  T v_sig, laplace_u, alpha_visc_max_ngb;
};

// runner_iact_nonsym_gradient (hydro_iact.h:276-329); signal velocity
// hydro.h:490-498 with beta = const_viscosity_beta; gamma=5/3 -> fac_mu = 1.
template <typename T>
__device__ __forceinline__ void iact_nonsym_gradient(T r2, T dx, T dy, T dz, T hi,
                                                     T vix, T viy, T viz, T ui_energy,
                                                     T ci, T mj, T vjx, T vjy, T vjz,
                                                     T uj_energy, T rhoj, T cj,
                                                     T alphaj, T a2_Hubble,
                                                     GradientAcc<T>& A) {
  T r, r_inv;
  r_and_inv(r2, r, r_inv);
  const T dvdr = (vix - vjx) * dx + (viy - vjy) * dy + (viz - vjz) * dz;
  const T dvdr_Hubble = dvdr + a2_Hubble * r2;
  const T omega_ij = tmin(dvdr_Hubble, (T)0);
  const T mu_ij = r_inv * omega_ij;
  const T new_v_sig = ci + cj - (T)kViscBeta * mu_ij;
  A.v_sig = tmax(A.v_sig, new_v_sig);
  T wi, wi_dx;
  const T ui = tdiv(r, hi);
  kernel_deval(ui, wi, wi_dx);
  const T delta_u_factor = (ui_energy - uj_energy) * r_inv;
  A.laplace_u += tdiv(mj * delta_u_factor * wi_dx, rhoj);
  A.alpha_visc_max_ngb = tmax(A.alpha_visc_max_ngb, alphaj);
}

// Per-particle force-side inputs (i or j).
template <typename T>
struct ForceIn {
  T m, h, rho, P, c, f, balsara, alpha_visc, alpha_diff, u;
  T vx, vy, vz;
  T m_inv, rho_inv, P_rho2;  // i side, fp64 path only (force_prep_i)
};

// The i-particle's reciprocals, once per gather instead of once per pair
// (fp64 path; the float path keeps the reference's per-pair divisions).
template <typename T>
__device__ __forceinline__ void force_prep_i(ForceIn<T>& I) {
  if constexpr (sizeof(T) == 8) {
    I.m_inv = rcp_f64(I.m);
    I.rho_inv = rcp_f64(I.rho);
    I.P_rho2 = I.P * I.rho_inv * I.rho_inv;
  } else {
    I.m_inv = I.rho_inv = I.P_rho2 = (T)0;
  }
}

template <typename T>
struct ForceAcc {
  T ax, ay, az, u_dt, h_dt;
  int min_ngb_time_bin;
};

// fp64 form of runner_iact_nonsym_force: the same terms with one
// reciprocal per distinct denominator (1/h_j, 1/m_j, 1/rho_j, 1/(rho_i +
// rho_j), 1/(P_i + P_j)), the i-side ones precomputed (force_prep_i), and
// sqrt(x) as x rsqrt(x).
__device__ __forceinline__ void iact_nonsym_force_f64(double r2, double dx, double dy,
                                                      double dz, const ForceIn<double>& I,
                                                      double hid_inv, double hi_inv,
                                                      const ForceIn<double>& J,
                                                      double a2_Hubble, ForceAcc<double>& A) {
  double r, r_inv;
  r_and_inv(r2, r, r_inv);
  const double mj = J.m;
  const double xi = r * hi_inv;
  double wi, wi_dx;
  kernel_deval(xi, wi, wi_dx);
  const double wi_dr = hid_inv * wi_dx;
  const double hj_inv = rcp1_f64(J.h);
  const double hj2 = hj_inv * hj_inv;
  const double hjd_inv = hj2 * hj2;
  double wj, wj_dx;
  kernel_deval(r * hj_inv, wj, wj_dx);
  const double wj_dr = hjd_inv * wj_dx;
  const double dvdr = (I.vx - J.vx) * dx + (I.vy - J.vy) * dy + (I.vz - J.vz) * dz;
  const double dvdr_Hubble = dvdr + a2_Hubble * r2;
  const double omega_ij = fmin(dvdr_Hubble, 0.);
  const double mu_ij = r_inv * omega_ij;
  const double v_sig = I.c + J.c - (double)kViscBeta * mu_ij;
  const double f_ij = 1. - I.f * rcp1_f64(mj);
  const double f_ji = 1. - J.f * I.m_inv;
  const double rhoj_inv = rcp1_f64(J.rho);
  const double rho_ij = I.rho + J.rho;
  const double rho_ij_inv = rcp1_f64(rho_ij);
  const double alpha = I.alpha_visc + J.alpha_visc;
  const double visc = -0.25 * alpha * v_sig * mu_ij * (I.balsara + J.balsara) * rho_ij_inv;
  const double visc_acc_term = 0.5 * visc * (wi_dr * f_ij + wj_dr * f_ji) * r_inv;
  const double P_over_rho2_i = I.P_rho2 * f_ij;
  const double P_over_rho2_j = J.P * rhoj_inv * rhoj_inv * f_ji;
  const double sph_acc_term = (P_over_rho2_i * wi_dr + P_over_rho2_j * wj_dr) * r_inv;
  const double acc = sph_acc_term + visc_acc_term;
  A.ax -= mj * acc * dx;
  A.ay -= mj * acc * dy;
  A.az -= mj * acc * dz;
  const double sph_du_term_i = P_over_rho2_i * dvdr * r_inv * wi_dr;
  const double visc_du_term = 0.5 * visc_acc_term * dvdr_Hubble;
  const double alpha_diff = (I.P * I.alpha_diff + J.P * J.alpha_diff) * rcp1_f64(I.P + J.P);
  const double q = 2. * fabs(I.P - J.P) * rho_ij_inv;
  const double sq = q > 0. ? q * rsqrt1_f64(q) : 0.;
  const double v_diff = alpha_diff * 0.5 * (sq + fabs(r_inv * dvdr_Hubble));
  const double diff_du_term =
      v_diff * (I.u - J.u) * (f_ij * wi_dr * I.rho_inv + f_ji * wj_dr * rhoj_inv);
  const double du_dt_i = sph_du_term_i + visc_du_term + diff_du_term;
  A.u_dt += du_dt_i * mj;
  A.h_dt -= mj * dvdr * r_inv * rhoj_inv * wi_dr;
}

// runner_iact_nonsym_force (hydro_iact.h:488-609). dx = x_i - x_j. The
// float path is the reference's operation order; fp64 takes the form above.
template <typename T>
__device__ __forceinline__ void iact_nonsym_force(T r2, T dx, T dy, T dz,
                                                  const ForceIn<T>& I, T hid_inv,
                                                  T hi_inv, const ForceIn<T>& J,
                                                  T a2_Hubble, ForceAcc<T>& A) {
  if constexpr (sizeof(T) == 8) {
    iact_nonsym_force_f64(r2, dx, dy, dz, I, hid_inv, hi_inv, J, a2_Hubble, A);
    return;
  }
  T r, r_inv;
  r_and_inv(r2, r, r_inv);
  const T mi = I.m, mj = J.m;
  const T rhoi = I.rho, rhoj = J.rho;
  const T pressurei = I.P, pressurej = J.P;
  const T xi = r * hi_inv;
  T wi, wi_dx;
  kernel_deval(xi, wi, wi_dx);
  const T wi_dr = hid_inv * wi_dx;
  const T hj_inv = tdiv((T)1, J.h);
  const T hj2 = hj_inv * hj_inv;
  const T hjd_inv = hj2 * hj2;
  const T xj = r * hj_inv;
  T wj, wj_dx;
  kernel_deval(xj, wj, wj_dx);
  const T wj_dr = hjd_inv * wj_dx;
  const T dvdr = (I.vx - J.vx) * dx + (I.vy - J.vy) * dy + (I.vz - J.vz) * dz;
  const T dvdr_Hubble = dvdr + a2_Hubble * r2;
  const T omega_ij = tmin(dvdr_Hubble, (T)0);
  const T mu_ij = r_inv * omega_ij;
  const T v_sig = I.c + J.c - (T)kViscBeta * mu_ij;
  const T f_ij = (T)1 - tdiv(I.f, mj);
  const T f_ji = (T)1 - tdiv(J.f, mi);
  const T rho_ij = rhoi + rhoj;
  const T alpha = I.alpha_visc + J.alpha_visc;
  const T visc = tdiv((T)-0.25 * alpha * v_sig * mu_ij * (I.balsara + J.balsara), rho_ij);
  const T visc_acc_term = (T)0.5 * visc * (wi_dr * f_ij + wj_dr * f_ji) * r_inv;
  const T P_over_rho2_i = tdiv(pressurei, rhoi * rhoi) * f_ij;
  const T P_over_rho2_j = tdiv(pressurej, rhoj * rhoj) * f_ji;
  const T sph_acc_term = (P_over_rho2_i * wi_dr + P_over_rho2_j * wj_dr) * r_inv;
  const T acc = sph_acc_term + visc_acc_term;
  A.ax -= mj * acc * dx;
  A.ay -= mj * acc * dy;
  A.az -= mj * acc * dz;
  const T sph_du_term_i = P_over_rho2_i * dvdr * r_inv * wi_dr;
  const T visc_du_term = (T)0.5 * visc_acc_term * dvdr_Hubble;
  const T alpha_diff = tdiv(pressurei * I.alpha_diff + pressurej * J.alpha_diff,
                            pressurei + pressurej);
  const T v_diff = alpha_diff * (T)0.5 *
                   (tsqrt(tdiv((T)2 * fabs(pressurei - pressurej), rho_ij)) +
                    fabs(r_inv * dvdr_Hubble));
  const T diff_du_term =
      v_diff * (I.u - J.u) * (tdiv(f_ij * wi_dr, rhoi) + tdiv(f_ji * wj_dr, rhoj));
  const T du_dt_i = sph_du_term_i + visc_du_term + diff_du_term;
  A.u_dt += du_dt_i * mj;
  A.h_dt -= tdiv(mj * dvdr * r_inv, rhoj) * wi_dr;
}

// ---------------------------------------------------------------------------
// Gravity (Wendland-C2 softening, erfc-like long-range truncation)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T grav_pot_eval(T u) {  // kernel_gravity.h:48-70
  T W = (T)3 * u - (T)15;
  W = W * u + (T)28;
  W = W * u - (T)21;
  W = W * u;
  W = W * u + (T)7;
  W = W * u;
  W = W * u - (T)3;
  return W;
}
template <typename T>
__device__ __forceinline__ T grav_force_eval(T u) {  // kernel_gravity.h:79-100
  T W = (T)21 * u - (T)90;
  W = W * u + (T)140;
  W = W * u - (T)84;
  W = W * u;
  W = W * u + (T)14;
  return W;
}

template <typename T> __device__ __forceinline__ T texp(T x);
template <> __device__ __forceinline__ double texp<double>(double x) { return exp(x); }
template <> __device__ __forceinline__ float texp<float>(float x) { return expf(x); }

// runner_iact_grav_pp_full / _truncated (gravity_iact.h:47-135)
template <typename T, bool TRUNC>
__device__ __forceinline__ void iact_grav_pp(T r2, T h2, T h_inv, T h_inv3, T mass,
                                             T r_s_inv, T& f_ij, T& pot_ij) {
  const T r_inv = (T)1 / tsqrt(r2 + (T)FLT_MIN);
  if (r2 >= h2) {
    f_ij = mass * r_inv * r_inv * r_inv;
    pot_ij = -mass * r_inv;
  } else {
    const T r = r2 * r_inv;
    const T ui = r * h_inv;
    f_ij = mass * h_inv3 * grav_force_eval(ui);
    pot_ij = mass * h_inv * grav_pot_eval(ui);
  }
  if (TRUNC) {
    const T r = r2 * r_inv;
    const T x = (T)2 * (r * r_s_inv);
    const T exp_x = texp(x);
    const T alpha = (T)1 / ((T)1 + exp_x);
    T W = (T)1 - alpha * exp_x;
    const T corr_pot = W * (T)2;
    W = (T)1 - alpha;
    W = W * x - exp_x;
    W = W * alpha + (T)1;
    const T corr_f = W * (T)2;
    f_ij *= corr_f;
    pot_ij *= corr_pot;
  }
}

}  // namespace swh
