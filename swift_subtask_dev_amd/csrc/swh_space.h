// swh_space.h — device views of the batch-path particle set and grid.
#pragma once

#include "swh_internal.h"

namespace swh {

// Sorted SoA arrays of a swh_space (device pointers, passed by value).
struct SoA {
  double4* pos;   // x, y, z, h
  float4* vm;     // vx, vy, vz, mass
  float4* th;     // u, rho, pressure, soundspeed
  float4* fc;     // f (grad-h), balsara, alpha_visc, alpha_diff
  int8_t* tb;     // time_bin
  float4* dens;   // rho_dh, wcount, wcount_dh, div_v
  float4* rot;    // rot_v[3], laplace_u
  float4* grad;   // v_sig, alpha_visc_max_ngb, div_v_previous_step, div_v_dt
  float4* acc;    // a_hydro[3], u_dt
  float* hdt;     // h_dt
  int8_t* mintb;  // limiter min_ngb_time_bin
  int* perm;      // sorted index -> caller index
  int* iperm;     // caller index -> sorted index
  int n_owned;    // caller indices >= n_owned are foreign (read-only halo)
};

// part_is_active (src/active.h:357-373) for a particle this space owns:
// foreign halo copies (another rank's particles, SWIFT's foreign cells) are
// neighbours of the loops but are never updated.
__device__ __forceinline__ bool active_part(const SoA& a, int64_t i, int max_active_bin) {
  return a.tb[i] <= max_active_bin && a.perm[i] < a.n_owned;
}

struct GridDev {
  int cdim[3];
  int periodic;
  double w[3];
  double inv_w[3];
  double origin[3];
  double dim[3];
  double dx;         // largest displacement since the rebuild: added to every reach
  const int2* span;  // linear (x-fastest) cell -> its sorted range [x, y)
};

// Sorted range of grid cell (cx, cy, cz) (already wrapped into the grid).
__device__ __forceinline__ int2 cell_range_of(const GridDev& g, int cx, int cy, int cz) {
  return g.span[(cz * g.cdim[1] + cy) * g.cdim[0] + cx];
}

inline GridDev grid_dev(const swh_space* s) {
  const SwhGrid& g = s->grid;
  GridDev d;
  d.span = s->cell_span.as<const int2>();
  for (int k = 0; k < 3; k++) {
    d.cdim[k] = g.cdim[k];
    d.w[k] = g.w[k];
    d.inv_w[k] = 1.0 / g.w[k];
    d.origin[k] = g.origin[k];
    d.dim[k] = g.dim[k];
  }
  d.periodic = g.periodic;
  d.dx = g.dx;
  return d;
}

SoA soa_of(swh_space* s);
// Recompute max h over the set into the device slot counters[2] (float bits).
swh_status space_hmax_to_device(swh_space* s);

}  // namespace swh
