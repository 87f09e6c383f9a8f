// swh_wave.h — wave-level helpers of the batch neighbour loops (swh_list.h)
// and the gravity kernels: wave barriers and reductions, wave-uniform
// broadcasts, stream compaction, the fp32 rounding constants of the list
// build's candidate tests, XCD-aware workgroup order and the combination of
// the lanes' partial loop states.
#pragma once

#include "swh_gather.h"

namespace swh {

// Counted launches add their per-wave counts into kCounterStripes stripes of
// 8 counters (a block's stripe by its index), summed afterwards by
// stripe_reduce_kernel: with one address for every wave's atomics the adds
// serialise at the L2 (~10 ns each: a 1M-wave launch spent 11 ms on them).
// Max / flag updates on one word from every wave: issue the atomic only when
// it changes the word (a relaxed load first; the atomics would serialise).
__device__ __forceinline__ void atomic_max_bits_if(unsigned int* p, unsigned int v) {
  if (v > __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(p, v);
}
__device__ __forceinline__ void atomic_flag_if(unsigned int* p) {
  if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(p, 1u);
}
// Max of v over a 256-thread block (every thread must call it), then one
// conditional atomic per block on p (float bits, v >= 0). sm: 4 floats of LDS.
__device__ __forceinline__ void block_max_bits(unsigned int* p, float v, float* sm) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float m = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    if (m > 0.f) atomic_max_bits_if(p, __float_as_uint(m));
  }
}
// Grid of the max / flag reductions: grid-stride loops over this many blocks
// keep the atomics on one word to a few thousand per launch.
constexpr int kReduceBlocks = 1024;
constexpr int kCounterStripes = 256;
__device__ __forceinline__ unsigned long long* counter_stripe(unsigned long long* c) {
  return c + (size_t)(blockIdx.x & (kCounterStripes - 1)) * 8;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

// Rounding bound of the list build's fp32 candidate tests: separations are
// formed from fp32 coordinates relative to the group centre, so a test of
// r2 < (R + 16 u D)^2 (1 + 8u) (u = 2^-24, D bounds the coordinates' size)
// accepts every pair whose exact fp64 separation is below R.
constexpr double kUnitRound = 5.9604644775390625e-8;   // u = 2^-24
constexpr float kThrSlack = 1.f + 8.f * 5.9604645e-8f;  // (1 + 8u)

// Work counters of a counted launch (swh_space_info.loop_stats): candidates
// loaded, candidates staged, test wave steps and list-flush lane steps.
struct TileStats {
  unsigned int loaded = 0, staged = 0, asteps = 0, bsteps = 0;
};

__device__ __forceinline__ float wrap_nearest_f(float d, float box) {
  return d > 0.5f * box ? d - box : (d < -0.5f * box ? d + box : d);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_*)

// The same nearest image by selects (no divergent branch).
__device__ __forceinline__ float wrap_nearest_sel(float d, float box) {
  const float hb = 0.5f * box;
  d = d > hb ? d - box : d;
  return d < -hb ? d + box : d;
}

__device__ __forceinline__ int uni_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uni_f(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ double uni_d(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned int lo = (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)b);
  const unsigned int hi =
      (unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double wave_min_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
// Wave-uniform max / min of a double that is equal within each quad of
// lanes (the list build's four lanes per i): two DPP mirrors combine the
// quads of each 16-lane row, four readlanes the rows -- no LDS round trip
// (__shfl_xor is a ds_bpermute).
__device__ __forceinline__ double dpp_d(double v, int ctrl_is_mirror) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  int l2, h2;
  if (ctrl_is_mirror) {
    l2 = __builtin_amdgcn_mov_dpp(lo, 0x140, 0xF, 0xF, false);  // row_mirror
    h2 = __builtin_amdgcn_mov_dpp(hi, 0x140, 0xF, 0xF, false);
  } else {
    l2 = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xF, 0xF, false);  // row_half_mirror
    h2 = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xF, 0xF, false);
  }
  return __hiloint2double(h2, l2);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
// (compare + select, not fmax/fmin: those canonicalize both operands first,
// three v_max_f64 per call; the inputs here are finite coordinates and reaches)
__device__ __forceinline__ double sel_max_d(double a, double b) { return b > a ? b : a; }
__device__ __forceinline__ double sel_min_d(double a, double b) { return b < a ? b : a; }
__device__ __forceinline__ double quad_group_max_d(double v) {
  v = sel_max_d(v, dpp_d(v, 0));
  v = sel_max_d(v, dpp_d(v, 1));
  return sel_max_d(sel_max_d(readlane_d(v, 0), readlane_d(v, 16)),
                   sel_max_d(readlane_d(v, 32), readlane_d(v, 48)));
}
__device__ __forceinline__ double quad_group_min_d(double v) {
  v = sel_min_d(v, dpp_d(v, 0));
  v = sel_min_d(v, dpp_d(v, 1));
  return sel_min_d(sel_min_d(readlane_d(v, 0), readlane_d(v, 16)),
                   sel_min_d(readlane_d(v, 32), readlane_d(v, 48)));
}

// Inclusive prefix sum over the 64 lanes by DPP (GFX9 row shifts within
// each 16-lane row, then row_bcast:15 / row_bcast:31 across rows).
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

__device__ __forceinline__ int wave_max_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// Stream compaction with one atomic per workgroup (blockDim.x <= 1024): the
// threads with `pred` get consecutive slots, in thread order. Every thread of
// the block must call it (it synchronises the block). Same-address atomics
// serialise in L2, so per-wave appends of millions of items cost ~0.3 ms.
template <typename C>
__device__ __forceinline__ int block_append(bool pred, C* counter) {
  __shared__ int wcnt[16];
  __shared__ int wbase[16];
  const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
  const int nw = (int)((blockDim.x + 63) >> 6);
  const unsigned long long m = __ballot(pred);
  if (lane == 0) wcnt[w] = (int)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int k = 0; k < nw; k++) {
      wbase[k] = tot;
      tot += wcnt[k];
    }
    const int b = tot ? (int)atomicAdd(counter, (C)tot) : 0;
    for (int k = 0; k < nw; k++) wbase[k] += b;
  }
  __syncthreads();
  return pred ? wbase[w] + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// Stream compaction with one atomic per wave: the lanes with `pred` get
// consecutive slots (in lane order) of the list whose length is *counter.
// Every lane of the wave must call it.
template <typename C>
__device__ __forceinline__ int wave_append(bool pred, C* counter) {
  const unsigned long long m = __ballot(pred);
  if (m == 0ull) return -1;
  const int lane = (int)(threadIdx.x & 63);
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = (int)atomicAdd(counter, (C)__popcll(m));
  base = __shfl(base, leader);
  return pred ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// Combine the LPI partial states of one i-particle (lanes differing in the
// low log2(LPI) bits): sums add, v_sig / alpha_max take the max, the limiter
// takes the min.
template <int W, typename T>
__device__ __forceinline__ void reduce_lanes(LoopState<LOOP_DENSITY, T>& s) {
  for (int o = 1; o < W; o <<= 1) {
    s.A.rho += __shfl_xor(s.A.rho, o);
    s.A.rho_dh += __shfl_xor(s.A.rho_dh, o);
    s.A.wcount += __shfl_xor(s.A.wcount, o);
    s.A.wcount_dh += __shfl_xor(s.A.wcount_dh, o);
    s.A.div_v += __shfl_xor(s.A.div_v, o);
    s.A.rot_x += __shfl_xor(s.A.rot_x, o);
    s.A.rot_y += __shfl_xor(s.A.rot_y, o);
    s.A.rot_z += __shfl_xor(s.A.rot_z, o);
    s.n += __shfl_xor(s.n, o);
  }
}
template <int W, typename T>
__device__ __forceinline__ void reduce_lanes(LoopState<LOOP_GRADIENT, T>& s) {
  for (int o = 1; o < W; o <<= 1) {
    s.A.v_sig = tmax(s.A.v_sig, (T)__shfl_xor(s.A.v_sig, o));
    s.A.alpha_visc_max_ngb =
        tmax(s.A.alpha_visc_max_ngb, (T)__shfl_xor(s.A.alpha_visc_max_ngb, o));
    s.A.laplace_u += __shfl_xor(s.A.laplace_u, o);
    s.n += __shfl_xor(s.n, o);
  }
}
template <int W, typename T>
__device__ __forceinline__ void reduce_lanes(LoopState<LOOP_FORCE, T>& s) {
  for (int o = 1; o < W; o <<= 1) {
    s.A.ax += __shfl_xor(s.A.ax, o);
    s.A.ay += __shfl_xor(s.A.ay, o);
    s.A.az += __shfl_xor(s.A.az, o);
    s.A.u_dt += __shfl_xor(s.A.u_dt, o);
    s.A.h_dt += __shfl_xor(s.A.h_dt, o);
    s.A.min_ngb_time_bin = min(s.A.min_ngb_time_bin, __shfl_xor(s.A.min_ngb_time_bin, o));
    s.n += __shfl_xor(s.n, o);
  }
}

}  // namespace swh
