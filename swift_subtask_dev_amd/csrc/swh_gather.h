// swh_gather.h — device-side neighbour gathers of the batch hydro loops.
//
// Each loop (density / gradient / force) is a state class with
//   load_i()   : i-particle inputs + accumulator initial values
//   accept()   : the loop's in-range test for a candidate j
//                (density, gradient: r < H_i; force: r < max(H_i, H_j))
//   interact() : the non-symmetric iact (hydro_iact.h:130, 276, 488)
//   store()    : accumulate into the particle's fields (SWIFT "+=" semantics)
//   kPay / load_j() / interact_staged(): the j-side record a list walk loads
//                (kPay float4s + one int) and the iact on it
//
// The list walks (swh_list.h) evaluate these states entry by entry; the
// wave-per-particle search of list overflow and ghost reruns walks the grid
// cells with cell_range / wrap_cell / separation.
#pragma once

#include "swh_physics.h"
#include "swh_space.h"

namespace swh {

enum { LOOP_DENSITY = 0, LOOP_GRADIENT = 1, LOOP_FORCE = 2 };

__device__ __forceinline__ double wrap_nearest(double d, double box) {
  return d > 0.5 * box ? d - box : (d < -0.5 * box ? d + box : d);
}

template <int LOOP, typename T>
struct LoopState;

// j-side record of a loop as loaded by a list walk.
template <int N>
struct JRec {
  float4 p[N];
  int meta;
};

// fp64 (the batch path): the sums of iact_nonsym_density_raw, finalized at
// the store; fp32 (SWH_PRECISION_F32): the reference's own arithmetic.
#ifndef SWH_DENS_RAW
#define SWH_DENS_RAW 1
#endif
template <typename T>
struct LoopState<LOOP_DENSITY, T> {
  static constexpr bool kRaw = SWH_DENS_RAW && sizeof(T) == 8;
  int self, n;
  double reach;
  T hig2, hi_inv, vix, viy, viz;
  DensityAcc<T> A;
  __device__ __forceinline__ void load_i(const SoA& a, int i, T, const unsigned int*) {
    const double4 p = a.pos[i];
    const float4 vm = a.vm[i];
    const T hi = (T)p.w;
    self = i;
    n = 0;
    hig2 = hi * hi * (T)kGamma2;
    hi_inv = (T)1 / hi;
    vix = vm.x; viy = vm.y; viz = vm.z;
    reach = p.w * (double)kGamma;
    A.zero();
  }
  __device__ __forceinline__ void iact(T r2, T dx, T dy, T dz, T mj, T vjx, T vjy, T vjz) {
    if constexpr (kRaw)
      iact_nonsym_density_raw(r2, dx, dy, dz, hi_inv, vix, viy, viz, mj, vjx, vjy, vjz, A);
    else
      iact_nonsym_density<T>(r2, dx, dy, dz, hi_inv, vix, viy, viz, mj, vjx, vjy, vjz, A);
  }
  __device__ __forceinline__ bool accept(int j, const double4&, T r2) const {
    return (r2 < hig2) & (j != self);
  }
  __device__ __forceinline__ void interact(const SoA& a, int j, const double4&, T dx, T dy,
                                           T dz, T r2) {
    const float4 v = a.vm[j];
    iact(r2, dx, dy, dz, (T)v.w, (T)v.x, (T)v.y, (T)v.z);
    n++;
  }
  static constexpr int kPay = 1;
  __device__ static __forceinline__ JRec<1> load_j(const SoA& a, int j) {
    JRec<1> r;
    r.p[0] = a.vm[j];
    r.meta = 0;
    return r;
  }
  __device__ __forceinline__ void interact_staged(const float4* p, int, const double4&, T dx,
                                                  T dy, T dz, T r2) {
    iact(r2, dx, dy, dz, (T)p[0].w, (T)p[0].x, (T)p[0].y, (T)p[0].z);
    n++;
  }
  __device__ __forceinline__ void store(SoA& a, int i) const {
    DensityAcc<T> A = this->A;
    if constexpr (kRaw) A = density_finalize(this->A);
    float4 d = a.dens[i];
    float4 r = a.rot[i];
    a.th[i].y = (float)((T)a.th[i].y + A.rho);
    d.x = (float)((T)d.x + A.rho_dh);
    d.y = (float)((T)d.y + A.wcount);
    d.z = (float)((T)d.z + A.wcount_dh);
    d.w = (float)((T)d.w + A.div_v);
    r.x = (float)((T)r.x + A.rot_x);
    r.y = (float)((T)r.y + A.rot_y);
    r.z = (float)((T)r.z + A.rot_z);
    a.dens[i] = d;
    a.rot[i] = r;
  }
};

template <typename T>
struct LoopState<LOOP_GRADIENT, T> {
  int self, n;
  double reach;
  T hi, hig2, vix, viy, viz, ui, ci, a2H;
  float gz, gw;
  GradientAcc<T> A;
  __device__ __forceinline__ void load_i(const SoA& a, int i, T a2H_, const unsigned int*) {
    const double4 p = a.pos[i];
    const float4 vm = a.vm[i];
    const float4 th = a.th[i];
    const float4 g = a.grad[i];
    self = i;
    n = 0;
    hi = (T)p.w;
    hig2 = hi * hi * (T)kGamma2;
    vix = vm.x; viy = vm.y; viz = vm.z;
    ui = th.x;
    ci = th.w;
    a2H = a2H_;
    reach = p.w * (double)kGamma;
    A.v_sig = g.x;
    A.alpha_visc_max_ngb = g.y;
    A.laplace_u = (T)0;
    gz = g.z;
    gw = g.w;
  }
  __device__ __forceinline__ bool accept(int j, const double4&, T r2) const {
    return (r2 < hig2) & (j != self);
  }
  __device__ __forceinline__ void interact(const SoA& a, int j, const double4&, T dx, T dy,
                                           T dz, T r2) {
    const float4 v = a.vm[j];
    const float4 t = a.th[j];
    iact_nonsym_gradient<T>(r2, dx, dy, dz, hi, vix, viy, viz, ui, ci, (T)v.w, (T)v.x, (T)v.y,
                            (T)v.z, (T)t.x, (T)t.y, (T)t.w, (T)a.fc[j].z, a2H, A);
    n++;
  }
  static constexpr int kPay = 2;
  __device__ static __forceinline__ JRec<2> load_j(const SoA& a, int j) {
    const float4 t = a.th[j];
    JRec<2> r;
    r.p[0] = a.vm[j];
    r.p[1] = make_float4(t.x, t.y, t.w, a.fc[j].z);  // u, rho, c, alpha_visc
    r.meta = 0;
    return r;
  }
  __device__ __forceinline__ void interact_staged(const float4* p, int, const double4&, T dx,
                                                  T dy, T dz, T r2) {
    iact_nonsym_gradient<T>(r2, dx, dy, dz, hi, vix, viy, viz, ui, ci, (T)p[0].w, (T)p[0].x,
                            (T)p[0].y, (T)p[0].z, (T)p[1].x, (T)p[1].y, (T)p[1].z, (T)p[1].w,
                            a2H, A);
    n++;
  }
  __device__ __forceinline__ void store(SoA& a, int i) const {
    a.grad[i] = make_float4((float)A.v_sig, (float)A.alpha_visc_max_ngb, gz, gw);
    a.rot[i].w = (float)((T)a.rot[i].w + A.laplace_u);
  }
};

template <typename T>
struct LoopState<LOOP_FORCE, T> {
  int self, n;
  double reach;
  T hig2, hi_inv, hid_inv, a2H;
  ForceIn<T> I;
  ForceAcc<T> A;
  __device__ __forceinline__ void load_i(const SoA& a, int i, T a2H_,
                                         const unsigned int* hmax_bits) {
    const double4 p = a.pos[i];
    const float4 vm = a.vm[i];
    const float4 th = a.th[i];
    const float4 fc = a.fc[i];
    const T hi = (T)p.w;
    self = i;
    n = 0;
    hig2 = hi * hi * (T)kGamma2;
    hi_inv = (T)1 / hi;
    const T hi2 = hi_inv * hi_inv;
    hid_inv = hi2 * hi2;
    a2H = a2H_;
    I.vx = vm.x; I.vy = vm.y; I.vz = vm.z; I.m = vm.w;
    I.h = hi;
    I.u = th.x; I.rho = th.y; I.P = th.z; I.c = th.w;
    I.f = fc.x; I.balsara = fc.y; I.alpha_visc = fc.z; I.alpha_diff = fc.w;
    force_prep_i(I);
    A.ax = A.ay = A.az = A.u_dt = A.h_dt = (T)0;
    A.min_ngb_time_bin = a.mintb[i];
    const double hmax = (double)__uint_as_float(*hmax_bits) * (double)kGamma;
    reach = fmax(hmax, p.w * (double)kGamma);
  }
  __device__ __forceinline__ bool accept(int j, const double4& pj, T r2) const {
    const T hj = (T)pj.w;
    return ((r2 < hig2) | (r2 < hj * hj * (T)kGamma2)) & (j != self);
  }
  __device__ __forceinline__ void interact(const SoA& a, int j, const double4& pj, T dx, T dy,
                                           T dz, T r2) {
    ForceIn<T> J;
    const float4 v = a.vm[j];
    const float4 t = a.th[j];
    const float4 c = a.fc[j];
    J.vx = v.x; J.vy = v.y; J.vz = v.z; J.m = v.w;
    J.h = (T)pj.w;
    J.u = t.x; J.rho = t.y; J.P = t.z; J.c = t.w;
    J.f = c.x; J.balsara = c.y; J.alpha_visc = c.z; J.alpha_diff = c.w;
    iact_nonsym_force<T>(r2, dx, dy, dz, I, hid_inv, hi_inv, J, a2H, A);
    const int tbj = a.tb[j];
    if (tbj > 0 && tbj < A.min_ngb_time_bin) A.min_ngb_time_bin = tbj;
    n++;
  }
  static constexpr int kPay = 3;
  __device__ static __forceinline__ JRec<3> load_j(const SoA& a, int j) {
    JRec<3> r;
    r.p[0] = a.vm[j];
    r.p[1] = a.th[j];
    r.p[2] = a.fc[j];
    r.meta = a.tb[j];
    return r;
  }
  __device__ __forceinline__ void interact_staged(const float4* p, int tbj, const double4& pj,
                                                  T dx, T dy, T dz, T r2) {
    ForceIn<T> J;
    J.vx = p[0].x; J.vy = p[0].y; J.vz = p[0].z; J.m = p[0].w;
    J.h = (T)pj.w;
    J.u = p[1].x; J.rho = p[1].y; J.P = p[1].z; J.c = p[1].w;
    J.f = p[2].x; J.balsara = p[2].y; J.alpha_visc = p[2].z; J.alpha_diff = p[2].w;
    iact_nonsym_force<T>(r2, dx, dy, dz, I, hid_inv, hi_inv, J, a2H, A);
    if (tbj > 0 && tbj < A.min_ngb_time_bin) A.min_ngb_time_bin = tbj;
    n++;
  }
  __device__ __forceinline__ void store(SoA& a, int i) const {
    float4 ac = a.acc[i];
    ac.x = (float)((T)ac.x + A.ax);
    ac.y = (float)((T)ac.y + A.ay);
    ac.z = (float)((T)ac.z + A.az);
    ac.w = (float)((T)ac.w + A.u_dt);
    a.acc[i] = ac;
    a.hdt[i] = (float)((T)a.hdt[i] + A.h_dt);
    a.mintb[i] = (int8_t)A.min_ngb_time_bin;
  }
};

// Grid-cell range of one particle: cells overlapping [x - R, x + R] per
// dimension. Periodic dimensions whose range covers the whole box switch to
// the nearest-image convention (tools.c pairs_all_*).
struct CellRange {
  int lo[3], hi[3];
  bool full[3];
};

__device__ __forceinline__ void cell_range(const GridDev& g, double xi, double yi, double zi,
                                           double reach, CellRange& c) {
  const double xs[3] = {xi, yi, zi};
  for (int k = 0; k < 3; k++) {
    const double rel = xs[k] - g.origin[k];
    // particles may sit up to g.dx outside their cell after a drift
    c.lo[k] = (int)floor((rel - reach - g.dx) * g.inv_w[k]);
    c.hi[k] = (int)floor((rel + reach + g.dx) * g.inv_w[k]);
    if (g.periodic) {
      c.full[k] = (c.hi[k] - c.lo[k] + 1 >= g.cdim[k]);
      if (c.full[k]) {
        c.lo[k] = 0;
        c.hi[k] = g.cdim[k] - 1;
      }
    } else {
      c.full[k] = false;
      c.lo[k] = c.lo[k] < 0 ? 0 : c.lo[k];
      c.hi[k] = c.hi[k] > g.cdim[k] - 1 ? g.cdim[k] - 1 : c.hi[k];
    }
  }
}

// Wrap grid coordinate ck of dimension k into the grid (periodic, not
// nearest-image) and return the image shift of the particles it holds.
__device__ __forceinline__ int wrap_cell(const GridDev& g, const CellRange& c, int k, int ck,
                                         double& shift) {
  shift = 0.;
  if (g.periodic && !c.full[k]) {
    if (ck < 0) {
      ck += g.cdim[k];
      shift = -g.dim[k];
    } else if (ck >= g.cdim[k]) {
      ck -= g.cdim[k];
      shift = g.dim[k];
    }
  }
  return ck;
}

// Separation x_i - x_j of candidate j under the row's image shifts.
template <typename T>
__device__ __forceinline__ T separation(const GridDev& g, const CellRange& c, const double4& pi,
                                        const double4& pj, double sx, double sy, double sz,
                                        T& tdx, T& tdy, T& tdz) {
  double dx = pi.x - (pj.x + sx);
  double dy = pi.y - (pj.y + sy);
  double dz = pi.z - (pj.z + sz);
  if (c.full[0]) dx = wrap_nearest(dx, g.dim[0]);
  if (c.full[1]) dy = wrap_nearest(dy, g.dim[1]);
  if (c.full[2]) dz = wrap_nearest(dz, g.dim[2]);
  tdx = (T)dx;
  tdy = (T)dy;
  tdz = (T)dz;
  return tdx * tdx + tdy * tdy + tdz * tdz;
}

}  // namespace swh
