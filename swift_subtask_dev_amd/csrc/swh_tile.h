// swh_tile.h — helpers shared by the wave-level neighbour loops (swh_tile4.h,
// swh_tile5.h, swh_list.h): wave barriers, row reductions, periodic image
// shifts and the staging geometry.
#pragma once

#include "swh_gather.h"

namespace swh {

// Staged candidate slots per wave and candidates fetched per lane per pass.
template <int LOOP>
struct TileSlots {
  static constexpr int value = 256;
};
#ifndef SWH_TILE_FETCH
#define SWH_TILE_FETCH 2
#endif
template <int LOOP>
struct TileFetch {
  static constexpr int value = SWH_TILE_FETCH;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Reductions within a row of SG lanes (xor offsets < SG stay in the row).
template <int SG>
__device__ __forceinline__ double row_min(double v) {
  for (int o = SG / 2; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}
template <int SG>
__device__ __forceinline__ double row_max(double v) {
  for (int o = SG / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ double shift_of(int code, double box) {
  return code == 1 ? -box : (code == 2 ? box : 0.);
}

// XCD-aware workgroup order: workgroups are dealt round-robin to the 8 XCDs
// (workgroup w runs on XCD w % 8); give each XCD a contiguous stretch of the
// Morton-ordered work so neighbouring work items share that XCD's L2.
__device__ __forceinline__ int xcd_block_id() {
  const int nwg = gridDim.x;
  const int per_xcd = (nwg + 7) / 8;
  const int xcd = blockIdx.x % 8, slot_in_xcd = blockIdx.x / 8;
  const int full_xcds = nwg - (per_xcd - 1) * 8;  // XCDs that get per_xcd blocks
  return xcd < full_xcds ? xcd * per_xcd + slot_in_xcd
                         : full_xcds * per_xcd + (xcd - full_xcds) * (per_xcd - 1) + slot_in_xcd;
}

}  // namespace swh
