// swh_mpole.h — multipole side of the gravity path: the M2P acceptance test
// (gravity_M2P_accept, src/multipole_accept.h:290-373, as evaluated by
// gravity_cache_populate, src/gravity_cache.h:200-290), the M2P kernel
// (gravity_M2P + potential_derivatives_compute_M2P, src/multipole.h:2257-2480,
// src/gravity_derivatives.h:516-760) and leaf P2M (gravity_P2M +
// gravity_multipole_compute_power, src/multipole.h:878-1266), order 4.
//
// The acceptance test is a discrete choice between two approximations, so it
// is evaluated in float, operation by operation as the reference does
// (contraction off): the GPU takes the M2P route for exactly the particles
// SWIFT does. The M2P itself is written differently from the reference's
// term-by-term listing: with g_m = (r^-1 d/dr)^m phi the derivative tensor of
// a radial potential is
//   D_abc = sum_{i,j,k} C(a,i) C(b,j) C(c,k) x^(a-2i) y^(b-2j) z^(c-2k) g_(a+b+c-i-j-k),
//   C(a,i) = a! / (2^i i! (a-2i)!),
// and the field is F_000 = -sum_n (-1)^|n| M_n D_n, F_e = -sum_n (-1)^|n| M_n
// D_(n+e) over the 35 terms n of the order-4 expansion; the loops are
// compile-time, so the compiler emits straight-line FMA code.
#pragma once

#include <algorithm>
#include <cmath>

#include "swh_physics.h"
#include "swifthip.h"

namespace swh {

// Multi-indices of swh_multipole::M (include/swifthip.h), struct multipole's
// member order.
constexpr int kMpA[SWH_MPOLE_TERMS] = {0, 1, 0, 0, 2, 0, 0, 1, 1, 0, 3, 0, 0, 2, 2, 1, 0, 1,
                                       0, 1, 4, 0, 0, 3, 3, 1, 0, 1, 0, 2, 2, 0, 2, 1, 1};
constexpr int kMpB[SWH_MPOLE_TERMS] = {0, 0, 1, 0, 0, 2, 0, 1, 0, 1, 0, 3, 0, 1, 0, 2, 2, 0,
                                       1, 1, 0, 4, 0, 1, 0, 3, 3, 0, 1, 2, 0, 2, 1, 2, 1};
constexpr int kMpC[SWH_MPOLE_TERMS] = {0, 0, 0, 1, 0, 0, 2, 0, 1, 1, 0, 0, 3, 0, 1, 0, 1, 2,
                                       2, 1, 0, 0, 4, 0, 1, 0, 1, 3, 3, 0, 2, 2, 1, 1, 2};

// C(a, i) = a! / (2^i i! (a - 2i)!), a <= 5.
__host__ __device__ constexpr double herm_coef(int a, int i) {
  return a == 2 ? 1.
       : a == 3 ? (i == 0 ? 1. : 3.)
       : a == 4 ? (i == 0 ? 1. : (i == 1 ? 6. : 3.))
       : a == 5 ? (i == 0 ? 1. : (i == 1 ? 10. : 15.))
                : 1.;
}

// n! for n <= 4
__host__ __device__ constexpr double fact(int n) { return n <= 1 ? 1. : n * fact(n - 1); }

// MAC parameters (swh_grav_params) in the float form the reference uses.
struct MacParams {
  float theta_crit2, eps, r_s_inv;
  int advanced, gadget, below_soft, trunc_mac, periodic;
  float dim[3];
};

inline MacParams mac_params(const swh_grav_params* G) {
  MacParams m;
  const float th = G->theta_crit;
  m.theta_crit2 = th * th;
  m.eps = G->adaptive_tolerance;
  m.r_s_inv = G->r_s_inv;
  m.advanced = G->use_advanced_MAC;
  m.gadget = G->use_gadget_tolerance;
  m.below_soft = G->use_tree_below_softening;
  m.trunc_mac = G->consider_truncation_in_MAC;
  m.periodic = G->periodic;
  for (int k = 0; k < 3; k++) m.dim[k] = G->dim[k];
  return m;
}

// The multipole fields the acceptance test reads, as floats.
struct MacSource {
  float CoM[3];
  float rho;        // r_max
  float max_soft;   // m_pole.max_softening
  float power2;     // m_pole.power[2]
  float M000;
};

__host__ __device__ inline MacSource mac_source(const swh_multipole& m) {
  MacSource s;
  for (int k = 0; k < 3; k++) s.CoM[k] = (float)m.CoM[k];
  s.rho = (float)m.r_max;
  s.max_soft = m.max_softening;
  s.power2 = m.power[2];
  s.M000 = m.M[0];
  return s;
}

// gravity_cache_populate's use_mpole for one particle at float position
// (x, y, z) with softening eps_i and old_a_grav_norm old_a.
__device__ inline bool m2p_accept(const MacParams& P, const MacSource& B, float x, float y,
                                  float z, float eps_i, float old_a) {
#pragma clang fp contract(off)
  float dx = x - B.CoM[0];
  float dy = y - B.CoM[1];
  float dz = z - B.CoM[2];
  if (P.periodic) {
    dx = dx > 0.5f * P.dim[0] ? dx - P.dim[0] : (dx < -0.5f * P.dim[0] ? dx + P.dim[0] : dx);
    dy = dy > 0.5f * P.dim[1] ? dy - P.dim[1] : (dy < -0.5f * P.dim[1] ? dy + P.dim[1] : dy);
    dz = dz > 0.5f * P.dim[2] ? dz - P.dim[2] : (dz < -0.5f * P.dim[2] ? dz + P.dim[2] : dz);
  }
  const float r2 = dx * dx + dy * dy + dz * dz;
  const float max_soft = fmaxf(B.max_soft, eps_i);
  const float E_BA_term = 8.f * B.power2;
  float f_MAC_inv = r2;
  if (P.periodic && P.trunc_mac) {  // gravity_f_MAC_inverse
    const float H = max_soft;
    if (r2 < (25.f / 81.f) * H * H)
      f_MAC_inv = (25.f / 81.f) * H * H;
    else if (P.r_s_inv * P.r_s_inv * r2 > (25.f / 9.f))
      f_MAC_inv = (9.f / 25.f) * P.r_s_inv * P.r_s_inv * r2 * r2;
  }
  const bool cond_2 = P.below_soft || max_soft * max_soft < r2;
  if (P.advanced && P.gadget) {
    const float q = B.rho / sqrtf(r2);
    const float q2 = q * q;
    const float ratio = q2 * q2;  // integer_powf(q, 4)
    return (B.M000 * ratio < P.eps * old_a * f_MAC_inv) && cond_2;
  }
  if (P.advanced) {
    const bool cond_1 = B.rho * B.rho < r2;
    const bool cond_3 = E_BA_term < P.eps * old_a * r2 * f_MAC_inv;
    return cond_1 && cond_2 && cond_3;
  }
  return (B.rho * B.rho < P.theta_crit2 * r2) && cond_2;
}

// 2 exp(-x) for x >= 0 (the truncation's argument, a finite distance ratio):
// Cody-Waite reduction by ln 2 in one fma (|k| <= x / ln2 keeps k times
// ln2's rounding error below 1e-15 of f for every x the truncation meets),
// then e^f = 1 + f (1 + f q(f)) on |f| <= ln2/2 with q of degree 6 fitted for
// the least maximum relative error (Lawson-weighted least squares on 4,000
// Chebyshev nodes in extended precision; max relative error 1.3e-12 checked on
// 200,001 points, four orders below the float a_grav / potential it feeds),
// every coefficient doubled so the result is 2 e^-x at no cost: 12
// instructions where the library exp takes ~30, no overflow / NaN handling.
// (Horner steps as three-operand v_fma_f64: the compiler otherwise copies
// each loop-invariant coefficient register before a two-operand v_fmac_f64,
// a move per term.)
__device__ __forceinline__ double fma3(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
template <bool FMA3>
__device__ __forceinline__ double horner_step(double p, double f, double c) {
  return FMA3 ? fma3(p, f, c) : fma(p, f, c);
}
// FMA3: the three-operand form (the batch kernel, whose registers hold the
// coefficients; the 256-thread tile kernel keeps fma and its register budget)
template <bool FMA3>
__device__ __forceinline__ double exp_neg_f64_x2(double x) {
  // k = rint(-x / ln 2) by the 1.5 * 2^52 shifter: one fma rounds to an
  // integer held in the low word (no conversion for the ldexp)
  const double kd = fma(x, -1.4426950408889634, 6755399441055744.0);
  const double k = kd - 6755399441055744.0;
  const double f = fma(k, -0.6931471805599453, -x);
  double q = horner_step<FMA3>(2 * 2.4778829221708597e-05, f, 2 * 0.00019908923481541454);
  q = horner_step<FMA3>(q, f, 2 * 0.0013889023827227704);
  q = horner_step<FMA3>(q, f, 2 * 0.008333281839354719);
  q = horner_step<FMA3>(q, f, 2 * 0.04166666572724781);
  q = horner_step<FMA3>(q, f, 2 * 0.16666666784287604);
  q = horner_step<FMA3>(q, f, 2 * 0.500000000012381);
  const double p = fma(f, fma(f, q, 2.), 2.);
  return __builtin_ldexp(p, __double2loint(kd));
}

// D_soft_k(u) of the Wendland-C2 softening (kernel_gravity.h:169-275).
template <typename T>
__device__ __forceinline__ void d_soft(T u, T* d) {
  const T u2 = u * u;
  d[1] = ((((-(T)3 * u + (T)15) * u - (T)28) * u + (T)21) * u2 - (T)7) * u2 + (T)3;
  d[2] = (((-(T)21 * u + (T)90) * u - (T)140) * u + (T)84) * u2 * u - (T)14 * u;
  d[3] = (((-(T)105 * u + (T)360) * u - (T)420) * u + (T)168) * u2;
  d[4] = ((-(T)315 * u + (T)720) * u - (T)420) * u2;
  d[5] = (-(T)315 * u2 + (T)420) * u;
  d[6] = (T)315 * u2 - (T)1260;
}

// g_m = Dt_(m+1) r^-m, m = 0..5 (Dt of potential_derivatives_compute_M2P):
// softened below eps, Newtonian, or truncated by the long-range kernel
// (kernel_long_grav_derivatives, default branch, kernel_long_gravity.h:151-183).
template <typename T>
__device__ __forceinline__ void radial_chain(T r2, T r_inv, T eps, bool periodic, T r_s_inv,
                                             T* g) {
  T Dt[7];
  if (r2 < eps * eps) {
    const T eps_inv = (T)1 / eps;
    const T u = r2 * r_inv * eps_inv;
    T d[7];
    d_soft<T>(u, d);
    T e = eps_inv;
    for (int k = 1; k <= 6; k++) {
      Dt[k] = e * d[k];
      e *= eps_inv;
    }
  } else if (!periodic) {
    Dt[1] = r_inv;
    for (int k = 2; k <= 6; k++) Dt[k] = -(T)(2 * k - 3) * Dt[k - 1] * r_inv;
  } else if constexpr (sizeof(T) == 8) {
    // alpha = 1 / (1 + e^x) = E r and e^x alpha = 1 - alpha = r with E =
    // e^-x, r = 1 / (1 + E) (as p2p_trunc): chi_k = -2 e^x alpha^(k+1) P_k =
    // -2 r alpha^k P_k(alpha), no overflow, one reciprocal
    const double x = 2. * r_s_inv * (r2 * r_inv);
    const double E2 = exp_neg_f64_x2<false>(x);  // 2 E
    const double om = rcp1_f64(fma(E2, 0.5, 1.));  // 1 - alpha
    const double al = 0.5 * E2 * om;
    const double c1 = 2. * r_s_inv, c2 = c1 * c1, c3 = c2 * c1, c4 = c3 * c1, c5 = c4 * c1;
    const double b = -2. * om * al;
    T chi[6];
    chi[0] = 2. * al;
    chi[1] = b * c1;
    chi[2] = b * c2 * fma(2., al, -1.);
    chi[3] = b * c3 * fma(fma(6., al, -6.), al, 1.);
    chi[4] = b * c4 * fma(fma(fma(24., al, -36.), al, 14.), al, -1.);
    chi[5] = b * c5 * fma(fma(fma(fma(120., al, -240.), al, 150.), al, -30.), al, 1.);
    const T ri = r_inv;
    Dt[1] = chi[0] * ri;
    Dt[2] = (chi[1] - chi[0] * ri) * ri;
    Dt[3] = ((chi[0] * ri - chi[1]) * (T)3 * ri + chi[2]) * ri;
    Dt[4] = (((-chi[0] * ri + chi[1]) * (T)15 * ri - (T)6 * chi[2]) * ri + chi[3]) * ri;
    Dt[5] = ((((chi[0] * ri - chi[1]) * (T)105 * ri + (T)45 * chi[2]) * ri - (T)10 * chi[3]) *
                 ri + chi[4]) * ri;
    Dt[6] = (((((-chi[0] * ri + chi[1]) * (T)945 * ri - (T)420 * chi[2]) * ri +
               (T)105 * chi[3]) * ri - (T)15 * chi[4]) * ri + chi[5]) * ri;
  } else {
    const T r = r2 * r_inv;
    const T c1 = (T)2 * r_s_inv;
    const T x = c1 * r;
    const T exp_x = exp(x);
    const T a1 = (T)1 / ((T)1 + exp_x);
    const T a2 = a1 * a1, a3 = a2 * a1, a4 = a3 * a1, a5 = a4 * a1, a6 = a5 * a1;
    const T c2 = c1 * c1, c3 = c2 * c1, c4 = c3 * c1, c5 = c4 * c1;
    const T m2e = -(T)2 * exp_x;
    T chi[6];
    chi[0] = m2e * a1 + (T)2;
    chi[1] = m2e * c1 * a2;
    chi[2] = m2e * c2 * ((T)2 * a3 - a2);
    chi[3] = m2e * c3 * ((T)6 * a4 - (T)6 * a3 + a2);
    chi[4] = m2e * c4 * ((T)24 * a5 - (T)36 * a4 + (T)14 * a3 - a2);
    chi[5] = m2e * c5 * ((T)120 * a6 - (T)240 * a5 + (T)150 * a4 - (T)30 * a3 + a2);
    // Dt_k from chi_0..chi_(k-1), nested in r^-1 as the reference does
    const T ri = r_inv;
    Dt[1] = chi[0] * ri;
    Dt[2] = (chi[1] - chi[0] * ri) * ri;
    Dt[3] = ((chi[0] * ri - chi[1]) * (T)3 * ri + chi[2]) * ri;
    Dt[4] = (((-chi[0] * ri + chi[1]) * (T)15 * ri - (T)6 * chi[2]) * ri + chi[3]) * ri;
    Dt[5] = ((((chi[0] * ri - chi[1]) * (T)105 * ri + (T)45 * chi[2]) * ri - (T)10 * chi[3]) *
                 ri + chi[4]) * ri;
    Dt[6] = (((((-chi[0] * ri + chi[1]) * (T)945 * ri - (T)420 * chi[2]) * ri +
               (T)105 * chi[3]) * ri - (T)15 * chi[4]) * ri + chi[5]) * ri;
  }
  T rp = (T)1;
  for (int m = 0; m <= 5; m++) {
    g[m] = Dt[m + 1] * rp;
    rp *= r_inv;
  }
}

// D_abc from the powers of the separation and the radial chain.
template <typename T, int A, int B, int C>
__device__ __forceinline__ T dtensor(const T* xp, const T* yp, const T* zp, const T* g) {
  T d = (T)0;
#pragma unroll
  for (int i = 0; 2 * i <= A; i++)
#pragma unroll
    for (int j = 0; 2 * j <= B; j++)
#pragma unroll
      for (int k = 0; 2 * k <= C; k++)
        d += (T)(herm_coef(A, i) * herm_coef(B, j) * herm_coef(C, k)) * xp[A - 2 * i] *
             yp[B - 2 * j] * zp[C - 2 * k] * g[A + B + C - i - j - k];
  return d;
}

template <typename T, int t>
__device__ __forceinline__ void m2p_term(const float* M, const T* xp, const T* yp, const T* zp,
                                         const T* g, T* F) {
  constexpr int a = kMpA[t], b = kMpB[t], c = kMpC[t];
  const T m = ((a + b + c) & 1) ? -(T)M[t] : (T)M[t];  // (-1)^|n| M_n
  F[0] -= m * dtensor<T, a, b, c>(xp, yp, zp, g);
  F[1] -= m * dtensor<T, a + 1, b, c>(xp, yp, zp, g);
  F[2] -= m * dtensor<T, a, b + 1, c>(xp, yp, zp, g);
  F[3] -= m * dtensor<T, a, b, c + 1>(xp, yp, zp, g);
}

template <typename T, int t>
__device__ __forceinline__ void m2p_terms(const float* M, const T* xp, const T* yp,
                                          const T* zp, const T* g, T* F) {
  if constexpr (t < SWH_MPOLE_TERMS) {
    if constexpr (t == 0 || t > 3) m2p_term<T, t>(M, xp, yp, zp, g, F);  // dipole is zero
    m2p_terms<T, t + 1>(M, xp, yp, zp, g, F);
  }
}

// runner_iact_grav_pm_full / _truncated (MultiSoftening/gravity_iact.h:142-
// 210): (r_x, r_y, r_z) = CoM - x_i, softening eps = max(eps_i, multipole's
// max softening). F = {potential, a_x, a_y, a_z}.
template <typename T>
__device__ __forceinline__ void m2p(const float* M, T rx, T ry, T rz, T eps, bool truncated,
                                    T r_s_inv, T* F) {
  const T r2 = rx * rx + ry * ry + rz * rz;
  T r_inv;
  if constexpr (sizeof(T) == 8) r_inv = rsqrt1_f64(r2);  // r2 > 0: the MAC passed
  else r_inv = (T)1 / sqrt(r2);
  T g[6];
  radial_chain<T>(r2, r_inv, eps, truncated, r_s_inv, g);
  T xp[6], yp[6], zp[6];
  xp[0] = yp[0] = zp[0] = (T)1;
#pragma unroll
  for (int k = 1; k < 6; k++) {
    xp[k] = xp[k - 1] * rx;
    yp[k] = yp[k - 1] * ry;
    zp[k] = zp[k - 1] * rz;
  }
  F[0] = F[1] = F[2] = F[3] = (T)0;
  m2p_terms<T, 0>(M, xp, yp, zp, g, F);
}

// ---------------------------------------------------------------------------
// M2L, L2L, L2P (order 4; gravity_M2L_apply, gravity_L2L, gravity_L2P,
// src/multipole.h:1600-2100, 2513-3018). Field tensors F_k, |k| <= 4, in
// swh_multipole::M's index order. With D_m the potential derivative tensor
// at r = (field centre - multipole centre) and X_n(d) = d^n / n!:
//   M2L: F_k += sum_{|n|+|k| <= 4} M_n D_(n+k)   (dipole M_1 = 0 about the CoM)
//   L2L: F'_k = sum_{|n|+|k| <= 4} X_n(c' - c) F_(n+k)
//   L2P: pot = -sum_n X_n(x - c) F_n,  a_e = sum_{|n| <= 3} X_n(x - c) F_(n+e)
// The (k, n) loops are compile-time, so each is straight-line FMA code.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int mp_index(int a, int b, int c) {
  int t = 0;
  while (t < SWH_MPOLE_TERMS && !(kMpA[t] == a && kMpB[t] == b && kMpC[t] == c)) t++;
  return t;
}
__host__ __device__ constexpr int mp_order(int t) { return kMpA[t] + kMpB[t] + kMpC[t]; }

// gravity_M2M (src/multipole.h:1278): M'_t += sum_{q <= t} M_q X_(t-q)(dx),
// dx = the new centre - the old one, X as in xpowers, the zero dipole skipped.
template <int t, int q>
__device__ __forceinline__ void m2m_tq(const float* M, const double* X, double* Mt) {
  if constexpr (q < SWH_MPOLE_TERMS) {
    if constexpr ((q == 0 || q > 3) && kMpA[q] <= kMpA[t] && kMpB[q] <= kMpB[t] &&
                  kMpC[q] <= kMpC[t]) {
      constexpr int d = mp_index(kMpA[t] - kMpA[q], kMpB[t] - kMpB[q], kMpC[t] - kMpC[q]);
      Mt[t] += (double)M[q] * X[d];
    }
    m2m_tq<t, q + 1>(M, X, Mt);
  }
}
template <int t>
__device__ __forceinline__ void m2m_t(const float* M, const double* X, double* Mt) {
  if constexpr (t < SWH_MPOLE_TERMS) {
    if constexpr (t == 0 || t > 3) m2m_tq<t, 0>(M, X, Mt);
    m2m_t<t + 1>(M, X, Mt);
  }
}

// D_m for the 35 multi-indices, |m| <= 4, from powers of r and the chain g
template <typename T, int t>
__device__ __forceinline__ void dtensors(const T* xp, const T* yp, const T* zp, const T* g,
                                         T* D) {
  if constexpr (t < SWH_MPOLE_TERMS) {
    D[t] = dtensor<T, kMpA[t], kMpB[t], kMpC[t]>(xp, yp, zp, g);
    dtensors<T, t + 1>(xp, yp, zp, g, D);
  }
}

template <typename T, int k, int n>
__device__ __forceinline__ void m2l_kn(const float* M, const T* D, T* F) {
  if constexpr (n < SWH_MPOLE_TERMS) {
    if constexpr ((n == 0 || n > 3) && mp_order(k) + mp_order(n) <= 4) {
      constexpr int m = mp_index(kMpA[k] + kMpA[n], kMpB[k] + kMpB[n], kMpC[k] + kMpC[n]);
      F[k] += (T)M[n] * D[m];
    }
    m2l_kn<T, k, n + 1>(M, D, F);
  }
}
template <typename T, int k>
__device__ __forceinline__ void m2l_k(const float* M, const T* D, T* F) {
  if constexpr (k < SWH_MPOLE_TERMS) {
    m2l_kn<T, k, 0>(M, D, F);
    m2l_k<T, k + 1>(M, D, F);
  }
}

// gravity_M2L_nonsym / _symmetric's per-direction work: (rx, ry, rz) = field
// centre - multipole centre (nearest image applied), eps the softening of
// the pair (potential_derivatives_compute_M2L, gravity_derivatives.h:217-515).
template <typename T>
__device__ __forceinline__ void m2l(const float* M, T rx, T ry, T rz, T eps, bool periodic,
                                    T r_s_inv, T* F) {
  const T r2 = rx * rx + ry * ry + rz * rz;
  T r_inv;
  if constexpr (sizeof(T) == 8) r_inv = rsqrt1_f64(r2);  // r2 > 0: the MAC passed
  else r_inv = (T)1 / sqrt(r2);
  T g[6];
  radial_chain<T>(r2, r_inv, eps, periodic, r_s_inv, g);
  T xp[5], yp[5], zp[5];
  xp[0] = yp[0] = zp[0] = (T)1;
#pragma unroll
  for (int q = 1; q < 5; q++) {
    xp[q] = xp[q - 1] * rx;
    yp[q] = yp[q - 1] * ry;
    zp[q] = zp[q - 1] * rz;
  }
  T D[SWH_MPOLE_TERMS];
  dtensors<T, 0>(xp, yp, zp, g, D);
  m2l_k<T, 0>(M, D, F);
}

// X_n(d) = d^n / n! for the 35 multi-indices (compile-time recursion: every
// index is a constant, so the arrays stay in registers)
template <typename T, int t>
__device__ __forceinline__ void xpowers_t(const T* xp, const T* yp, const T* zp, T* X) {
  if constexpr (t < SWH_MPOLE_TERMS) {
    constexpr double inv = 1. / (fact(kMpA[t]) * fact(kMpB[t]) * fact(kMpC[t]));
    X[t] = xp[kMpA[t]] * yp[kMpB[t]] * zp[kMpC[t]] * (T)inv;
    xpowers_t<T, t + 1>(xp, yp, zp, X);
  }
}
template <typename T>
__device__ __forceinline__ void xpowers(T dx, T dy, T dz, T* X) {
  T xp[5], yp[5], zp[5];
  xp[0] = yp[0] = zp[0] = (T)1;
#pragma unroll
  for (int q = 1; q < 5; q++) {
    xp[q] = xp[q - 1] * dx;
    yp[q] = yp[q - 1] * dy;
    zp[q] = zp[q - 1] * dz;
  }
  xpowers_t<T, 0>(xp, yp, zp, X);
}

template <typename T, int k, int n>
__device__ __forceinline__ void l2l_kn(const T* X, const T* Fp, T* F) {
  if constexpr (n < SWH_MPOLE_TERMS) {
    if constexpr (mp_order(k) + mp_order(n) <= 4) {
      constexpr int m = mp_index(kMpA[k] + kMpA[n], kMpB[k] + kMpB[n], kMpC[k] + kMpC[n]);
      F[k] += X[n] * Fp[m];
    }
    l2l_kn<T, k, n + 1>(X, Fp, F);
  }
}
template <typename T, int k>
__device__ __forceinline__ void l2l_k(const T* X, const T* Fp, T* F) {
  if constexpr (k < SWH_MPOLE_TERMS) {
    l2l_kn<T, k, 0>(X, Fp, F);
    l2l_k<T, k + 1>(X, Fp, F);
  }
}

// gravity_L2P: {potential, a_x, a_y, a_z} at offset d from the tensor's centre
// (F: the tensor in fp64, e.g. staged in LDS)
template <typename T, int t>
__device__ __forceinline__ void l2p_t(const double* F, const T* X, T& pot, T& ax, T& ay, T& az) {
  if constexpr (t < SWH_MPOLE_TERMS) {
    pot -= X[t] * (T)F[t];
    if constexpr (mp_order(t) <= 3) {
      constexpr int ix = mp_index(kMpA[t] + 1, kMpB[t], kMpC[t]);
      constexpr int iy = mp_index(kMpA[t], kMpB[t] + 1, kMpC[t]);
      constexpr int iz = mp_index(kMpA[t], kMpB[t], kMpC[t] + 1);
      ax += X[t] * (T)F[ix];
      ay += X[t] * (T)F[iy];
      az += X[t] * (T)F[iz];
    }
    l2p_t<T, t + 1>(F, X, pot, ax, ay, az);
  }
}
template <typename T>
__device__ __forceinline__ void l2p(const double* F, T dx, T dy, T dz, T* out) {
  T X[SWH_MPOLE_TERMS];
  xpowers<T>(dx, dy, dz, X);
  T pot = (T)0, ax = (T)0, ay = (T)0, az = (T)0;
  l2p_t<T, 0>(F, X, pot, ax, ay, az);
  out[0] = pot;
  out[1] = ax;
  out[2] = ay;
  out[3] = az;
}

// gravity_M2L_accept (multipole_accept.h:78-176) for sink A, source B, in the
// reference's float arithmetic (host side: the tree walk's decision).
struct M2LSide {
  float rho, max_soft, min_a, M000, power[3];
};
__host__ __device__ inline M2LSide m2l_side(const swh_multipole& m) {
  M2LSide s;
  s.rho = (float)m.r_max;
  s.max_soft = m.max_softening;
  s.min_a = m.min_old_a_grav_norm;
  s.M000 = m.M[0];
  for (int k = 0; k < 3; k++) s.power[k] = m.power[k];
  return s;
}
__host__ __device__ inline bool m2l_accept(const MacParams& P, const M2LSide& A, const M2LSide& B,
                                           float r2) {
#pragma clang fp contract(off)
  const float rho_A = A.rho, rho_B = B.rho;
  const float rho_max = rho_A > rho_B ? rho_A : rho_B;
  const float max_softening = A.max_soft > B.max_soft ? A.max_soft : B.max_soft;
  // p = 2: sum_n binomial(2, n) power_B[n] rho_A^(2 - n)
  float E_BA_term = 0.f;
  E_BA_term += 1.f * B.power[0] * (rho_A * rho_A);
  E_BA_term += 2.f * B.power[1] * rho_A;
  E_BA_term += 1.f * B.power[2] * 1.f;
  E_BA_term *= 8.f;
  if (rho_A + rho_B > 0.f) {
    E_BA_term *= rho_max;
    E_BA_term /= (rho_A + rho_B);
  }
  const float r_to_p = r2;
  float f_MAC_inv = r2;
  if (P.periodic && P.trunc_mac) {  // gravity_f_MAC_inverse
    const float H = max_softening;
    if (r2 < (25.f / 81.f) * H * H)
      f_MAC_inv = (25.f / 81.f) * H * H;
    else if (P.r_s_inv * P.r_s_inv * r2 > (25.f / 9.f))
      f_MAC_inv = (9.f / 25.f) * P.r_s_inv * P.r_s_inv * r2 * r2;
  }
  const float min_a_grav = A.min_a;
  const float M_max = A.M000 > B.M000 ? A.M000 : B.M000;
  const float rho_sum = rho_A + rho_B;
  const bool cond_2 = P.below_soft || max_softening * max_softening < r2;
  if (P.advanced && P.gadget) {
    const float q = rho_max / sqrtf(r2);
    const float ratio = q * q * q;  // integer_powf(q, SELF_GRAVITY_MULTIPOLE_ORDER - 1)
    return (M_max * ratio < P.eps * min_a_grav * f_MAC_inv) && cond_2;
  }
  if (P.advanced) {
    const bool cond_1 = rho_sum * rho_sum < r2;
    const bool cond_3 = E_BA_term < P.eps * min_a_grav * r_to_p * f_MAC_inv;
    return cond_1 && cond_2 && cond_3;
  }
  return (rho_sum * rho_sum < P.theta_crit2 * r2) && cond_2;
}

// gravity_multipole_compute_power (multipole.h:878-972) on the stored
// float terms, with the reference's mixed float/double arithmetic: unit
// weights square in float, fractional weights multiply in double.
__host__ __device__ inline void mpole_power(swh_multipole& m) {
  double p[5] = {0., 0., 0., 0., 0.};
  for (int t = 4; t < SWH_MPOLE_TERMS; t++) {
    const int a = kMpA[t], b = kMpB[t], c = kMpC[t], o = a + b + c;
    const double w = fact(a) * fact(b) * fact(c) / fact(o);
    const float M = m.M[t];
    if (w == 1.)
      p[o] += (double)(M * M);
    else
      p[o] += w * (double)M * (double)M;
  }
  m.power[0] = m.M[0];
  m.power[1] = 0.f;
  for (int o = 2; o <= 4; o++) m.power[o] = (float)sqrt(p[o]);
}

}  // namespace swh
