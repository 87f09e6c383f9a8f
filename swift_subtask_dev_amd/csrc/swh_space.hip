// swh_space.hip — device-resident particle set of the batch path:
// AoS <-> SoA marshalling (the caller keeps SWIFT's struct part layout), and
// the neighbour-grid rebuild that replaces space_rebuild + runner_do_hydro_sort
// (src/space.c, src/runner_sort.c:201-431) for this path: particles are
// binned into a uniform grid of cells of width >= max(H)/cell_factor and
// stably radix-sorted by the Morton rank of their cell, so every cell is one
// contiguous range of the SoA arrays and consecutive cells are close in space.
// The tile loops' i-groups are cut from that order the way SWIFT splits its
// cell tree into leaves (space_split, cell.c): runs of consecutive cells of
// one aligned Morton block holding <= 64 particles.
#include <cmath>
#include <cstdlib>
#include <hipcub/hipcub.hpp>

#include <cstring>

#include "swh_internal.h"
#include "swh_physics.h"
#include "swh_space.h"
#include "swh_wave.h"

namespace swh {

__device__ __forceinline__ float aos_f(const char* r, int off) {
  return off >= 0 ? *reinterpret_cast<const float*>(r + off) : 0.f;
}

__global__ void unpack_kernel(Layout L, const char* __restrict__ aos, int64_t n, SoA a,
                              int8_t* __restrict__ hasg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const char* r = aos + i * L.stride;
  hasg[i] = (L.gpart >= 0 && *reinterpret_cast<void* const*>(r + L.gpart) != nullptr) ? 1 : 0;
  const double* x = reinterpret_cast<const double*>(r + L.x);
  a.pos[i] = make_double4(x[0], x[1], x[2], (double)aos_f(r, L.h));
  a.vm[i] = make_float4(aos_f(r, L.v), aos_f(r, L.v + 4), aos_f(r, L.v + 8), aos_f(r, L.mass));
  a.th[i] = make_float4(aos_f(r, L.u), aos_f(r, L.rho), aos_f(r, L.pressure),
                        aos_f(r, L.soundspeed));
  a.fc[i] = make_float4(aos_f(r, L.f), aos_f(r, L.balsara), aos_f(r, L.visc_alpha),
                        aos_f(r, L.diff_alpha));
  a.tb[i] = *reinterpret_cast<const int8_t*>(r + L.time_bin);
  a.dens[i] = make_float4(aos_f(r, L.rho_dh), aos_f(r, L.wcount), aos_f(r, L.wcount_dh),
                          aos_f(r, L.div_v));
  a.rot[i] = make_float4(aos_f(r, L.rot_v), aos_f(r, L.rot_v + 4), aos_f(r, L.rot_v + 8),
                         aos_f(r, L.laplace_u));
  a.grad[i] = make_float4(aos_f(r, L.v_sig), aos_f(r, L.avmn), aos_f(r, L.div_v_prev),
                          aos_f(r, L.div_v_dt));
  a.acc[i] = make_float4(aos_f(r, L.a_hydro), aos_f(r, L.a_hydro + 4),
                         aos_f(r, L.a_hydro + 8), aos_f(r, L.u_dt));
  a.hdt[i] = aos_f(r, L.h_dt);
  a.mintb[i] = L.min_tb >= 0 ? *reinterpret_cast<const int8_t*>(r + L.min_tb) : (int8_t)0;
  a.perm[i] = (int)i;
}

__device__ __forceinline__ void put_f(char* r, int off, float v) {
  if (off >= 0) *reinterpret_cast<float*>(r + off) = v;
}

__global__ void pack_kernel(Layout L, char* __restrict__ aos, int64_t n, SoA a, int fields) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  char* r = aos + (int64_t)a.perm[s] * L.stride;
  const double4 p = a.pos[s];
  const float4 th = a.th[s];
  if (fields & SWH_FIELDS_DENSITY) {
    const float4 d = a.dens[s];
    const float4 rt = a.rot[s];
    put_f(r, L.h, (float)p.w);
    put_f(r, L.rho, th.y);
    put_f(r, L.rho_dh, d.x);
    put_f(r, L.wcount, d.y);
    put_f(r, L.wcount_dh, d.z);
    put_f(r, L.div_v, d.w);
    put_f(r, L.rot_v, rt.x);
    put_f(r, L.rot_v + 4, rt.y);
    put_f(r, L.rot_v + 8, rt.z);
    put_f(r, L.laplace_u, rt.w);
  }
  if (fields & SWH_FIELDS_GRADIENT) {
    const float4 d = a.dens[s];
    const float4 rt = a.rot[s];
    const float4 g = a.grad[s];
    const float4 fc = a.fc[s];
    put_f(r, L.h, (float)p.w);
    put_f(r, L.rho, th.y);
    put_f(r, L.div_v, d.w);
    put_f(r, L.laplace_u, rt.w);
    put_f(r, L.v_sig, g.x);
    put_f(r, L.avmn, g.y);
    put_f(r, L.div_v_prev, g.z);
    put_f(r, L.div_v_dt, g.w);
    put_f(r, L.f, fc.x);
    put_f(r, L.balsara, fc.y);
    put_f(r, L.visc_alpha, fc.z);
    put_f(r, L.diff_alpha, fc.w);
    put_f(r, L.pressure, th.z);
    put_f(r, L.soundspeed, th.w);
  }
  if (fields & SWH_FIELDS_FORCE) {
    const float4 ac = a.acc[s];
    put_f(r, L.a_hydro, ac.x);
    put_f(r, L.a_hydro + 4, ac.y);
    put_f(r, L.a_hydro + 8, ac.z);
    put_f(r, L.u_dt, ac.w);
    put_f(r, L.h_dt, a.hdt[s]);
    if (L.min_tb >= 0) *reinterpret_cast<int8_t*>(r + L.min_tb) = a.mintb[s];
  }
  if (fields & SWH_FIELDS_DRIFT) {
    double* x = reinterpret_cast<double*>(r + L.x);
    x[0] = p.x;
    x[1] = p.y;
    x[2] = p.z;
    const float4 vm = a.vm[s];
    put_f(r, L.v, vm.x);
    put_f(r, L.v + 4, vm.y);
    put_f(r, L.v + 8, vm.z);
    put_f(r, L.h, (float)p.w);
    put_f(r, L.u, th.x);
    put_f(r, L.rho, th.y);
    put_f(r, L.pressure, th.z);
    put_f(r, L.soundspeed, th.w);
    put_f(r, L.v_sig, a.grad[s].x);
  }
}

// Per-block partial bounding box + max h over non-inhibited particles.
__global__ void bbox_kernel(const double4* __restrict__ pos, const int8_t* __restrict__ tb,
                            int64_t n, double* out) {
  // per block: min x,y,z; max x,y,z; max h; sum of log h (the grid's typical h)
  __shared__ double red[8][256];
  double v[8] = {1e300, 1e300, 1e300, -1e300, -1e300, -1e300, 0., 0.};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (tb[i] == kTimeBinInhibited) continue;
    const double4 p = pos[i];
    v[0] = fmin(v[0], p.x); v[1] = fmin(v[1], p.y); v[2] = fmin(v[2], p.z);
    v[3] = fmax(v[3], p.x); v[4] = fmax(v[4], p.y); v[5] = fmax(v[5], p.z);
    v[6] = fmax(v[6], p.w);
    v[7] += p.w > 0. ? log(p.w) : 0.;
  }
  for (int k = 0; k < 8; k++) red[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      for (int k = 0; k < 3; k++)
        red[k][threadIdx.x] = fmin(red[k][threadIdx.x], red[k][threadIdx.x + s]);
      for (int k = 3; k < 7; k++)
        red[k][threadIdx.x] = fmax(red[k][threadIdx.x], red[k][threadIdx.x + s]);
      red[7][threadIdx.x] += red[7][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int k = 0; k < 8; k++) out[blockIdx.x * 8 + k] = red[k][0];
}

// Inhibited particles get key = ncell: they sort behind every cell and are
// never visited as neighbours (the loops' part_is_inhibited skip).
__device__ __forceinline__ uint32_t spread3(uint32_t v);

// The key is the cell's Morton rank followed by `sb` bits per dimension of
// the particle's Morton position inside its cell: a cell stays one
// contiguous range, and inside it particles close in space are close in
// memory, so the neighbours a list entry names sit in few cache lines.
__global__ void key_kernel(GridDev g, const int* __restrict__ rank, double4* __restrict__ pos,
                           const int8_t* __restrict__ tb, int64_t n, int ncell, int sb,
                           uint32_t* __restrict__ keys, int* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  idx[i] = (int)i;
  if (tb[i] == kTimeBinInhibited) {
    keys[i] = (uint32_t)ncell << (3 * sb);
    return;
  }
  double4 p = pos[i];
  if (g.periodic) {  // box-wrap as space_rebuild does
    p.x -= floor(p.x / g.dim[0]) * g.dim[0];
    p.y -= floor(p.y / g.dim[1]) * g.dim[1];
    p.z -= floor(p.z / g.dim[2]) * g.dim[2];
    if (p.x >= g.dim[0]) p.x = 0.;
    if (p.y >= g.dim[1]) p.y = 0.;
    if (p.z >= g.dim[2]) p.z = 0.;
    pos[i] = p;
  }
  int c[3];
  uint32_t sub[3];
  const double xs[3] = {p.x, p.y, p.z};
  const int smax = (1 << sb) - 1;
  for (int k = 0; k < 3; k++) {
    const double u = (xs[k] - g.origin[k]) * g.inv_w[k];
    int ck = (int)floor(u);
    ck = ck < 0 ? 0 : (ck >= g.cdim[k] ? g.cdim[k] - 1 : ck);
    c[k] = ck;
    int sk = (int)floor((u - ck) * (double)(1 << sb));
    sub[k] = (uint32_t)(sk < 0 ? 0 : (sk > smax ? smax : sk));
  }
  const uint32_t sm = spread3(sub[0]) | (spread3(sub[1]) << 1) | (spread3(sub[2]) << 2);
  keys[i] = ((uint32_t)rank[(c[2] * g.cdim[1] + c[1]) * g.cdim[0] + c[0]] << (3 * sb)) | sm;
}

// Drop the in-cell bits of the sorted keys: keys become cell ranks again.
__global__ void key_shift_kernel(uint32_t* __restrict__ keys, int64_t n, int shift) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keys[i] >>= shift;
}

__device__ __forceinline__ uint32_t spread3(uint32_t v) {  // 10 bits -> every 3rd bit
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// Morton code of every linear cell (cdim <= 1024 per dimension).
__global__ void morton_kernel(int cx, int cy, int ncell, uint32_t* __restrict__ code,
                              int* __restrict__ lin) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncell) return;
  const uint32_t x = c % cx, y = (c / cx) % cy, z = c / (cx * cy);
  code[c] = spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
  lin[c] = c;
}

__global__ void span_kernel(const int* __restrict__ rank, const int* __restrict__ cs, int ncell,
                            int2* __restrict__ span) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncell) return;
  const int r = rank[c];
  span[c] = make_int2(cs[r], cs[r + 1]);
}

__global__ void rank_scatter_kernel(const int* __restrict__ sorted_lin, int ncell,
                                    int* __restrict__ rank) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < ncell) rank[sorted_lin[k]] = k;
}

// i-groups of the tile loops: the leaves of the octree over the Morton-ordered
// cells with at most kGroupMax (= the tile row width) particles (space_split's rule with
// space_splitsize = kGroupMax), consecutive sibling leaves merged while they
// fit. A block at level L = the aligned 2^L-cube of cells sharing code >> 3L;
// its cells are one contiguous rank range (ranks sorted by code). One thread
// per cell; the first cell of a leaf block emits its group. Cells holding more
// than kGroupMax particles are split into full chunks of kGroupMax; the
// remainder joins the sibling run that follows it (round 6: at the 128^3
// lattice's 18-particle cells it no longer takes a build wave of its own).
constexpr int kMaxLevel = 10;  // 30-bit codes
#ifndef SWH_GROUP_TAIL_MERGE
#define SWH_GROUP_TAIL_MERGE 1
#endif

__device__ __forceinline__ int lower_bound_u32(const uint32_t* __restrict__ a, int n,
                                               uint32_t v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

struct BlockSpan {
  int r0, r1;  // rank range
  int count;   // particles
};

__device__ __forceinline__ BlockSpan block_span(const uint32_t* __restrict__ code,
                                                const int* __restrict__ cs, int ncell,
                                                uint32_t lo_code, int level) {
  BlockSpan b;
  const uint64_t hi_code = (uint64_t)lo_code + (1ull << (3 * level));
  b.r0 = lower_bound_u32(code, ncell, lo_code);
  b.r1 = hi_code > 0xffffffffull ? ncell : lower_bound_u32(code, ncell, (uint32_t)hi_code);
  b.count = cs[b.r1] - cs[b.r0];
  return b;
}

template <bool WRITE>
__global__ void group_kernel(const uint32_t* __restrict__ code, const int* __restrict__ cs,
                             int ncell, int kGroupMax, int* __restrict__ ngroup,
                             const int* __restrict__ off, int2* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= ncell) return;
  const uint32_t c = code[r];
  int ng = 0;
  const int n0 = cs[r + 1] - cs[r];
  auto emit = [&](int start, int count) {
    if (WRITE) out[off[r] + ng] = make_int2(start, count);
    ng++;
  };
  // the level of the largest block around this cell that holds <= kGroupMax
  // particles (an oversized cell: level 0, the cell itself, split into chunks)
  int L = 0;
  BlockSpan leaf;
  leaf.r0 = r;
  leaf.r1 = r + 1;
  leaf.count = n0;
  if (n0 <= kGroupMax) {
    for (int l = 1; l <= kMaxLevel; l++) {
      const BlockSpan b = block_span(code, cs, ncell, (c >> (3 * l)) << (3 * l), l);
      if (b.count > kGroupMax) break;
      L = l;
      leaf = b;
    }
  }
  if (leaf.r0 == r && leaf.count > 0) {  // head of a non-empty leaf
    if (L == kMaxLevel) {
      emit(cs[leaf.r0], leaf.count);
    } else {
      // greedy merge over the parent's children, in order. A child holding
      // more than kGroupMax particles breaks the run; at the cell level
      // (L = 0) an oversized cell is cut into full chunks (emitted by its own
      // thread) and its remainder -- the END of its range, contiguous with
      // the next cell's -- starts the next run, so a 2-particle tail shares
      // a wave with its sibling cell instead of taking a build wave alone
      const int mine = (int)((c >> (3 * L)) & 7u);
      const uint32_t parent = (c >> (3 * (L + 1))) << (3 * (L + 1));
      int run_start = -1, run_p0 = 0, sum = 0;
      for (int o = 0; o < 8; o++) {
        const BlockSpan ch = block_span(code, cs, ncell, parent + ((uint32_t)o << (3 * L)), L);
        int cnt = ch.count, p0 = cs[ch.r0];
        if (cnt > kGroupMax) {
          if (run_start == mine) emit(run_p0, sum);
          run_start = -1;
          sum = 0;
          if (L > 0) continue;  // a block of several cells: split at a lower level
#if !SWH_GROUP_TAIL_MERGE
          if (o == mine)  // rounds 1-5: the remainder is a group of its own
            for (int q = 0; q < cnt; q += kGroupMax) emit(p0 + q, min(kGroupMax, cnt - q));
          continue;
#endif
          const int full = cnt / kGroupMax * kGroupMax;
          if (o == mine)
            for (int q = 0; q < full; q += kGroupMax) emit(p0 + q, kGroupMax);
          cnt -= full;  // the remainder joins the run that follows
          p0 += full;
        }
        if (cnt == 0) continue;
        if (run_start >= 0 && sum + cnt > kGroupMax) {
          if (run_start == mine) emit(run_p0, sum);
          run_start = -1;
          sum = 0;
        }
        if (run_start < 0) {
          run_start = o;
          run_p0 = p0;
        }
        sum += cnt;
      }
      if (run_start == mine) emit(run_p0, sum);
    }
  }
  if (!WRITE) ngroup[r] = ng;
}

// Gather every SoA array through the sort permutation (src -> dst).
__global__ void permute_kernel(SoA src, SoA dst, const int* __restrict__ idx, int64_t n) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int i = idx[s];
  dst.pos[s] = src.pos[i];
  dst.vm[s] = src.vm[i];
  dst.th[s] = src.th[i];
  dst.fc[s] = src.fc[i];
  dst.tb[s] = src.tb[i];
  dst.dens[s] = src.dens[i];
  dst.rot[s] = src.rot[i];
  dst.grad[s] = src.grad[i];
  dst.acc[s] = src.acc[i];
  dst.hdt[s] = src.hdt[i];
  dst.mintb[s] = src.mintb[i];
  dst.perm[s] = src.perm[i];
}

__global__ void iperm_kernel(const int* __restrict__ perm, int64_t n, int* __restrict__ iperm) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) iperm[perm[s]] = (int)s;
}

// Halo records (swh_space_pack_halo): h, rho, P, c, f, balsara, alpha_visc,
// alpha_diff of the particles with caller indices idx[0..n).
__global__ void halo_pack_kernel(SoA a, const int* __restrict__ idx, int n,
                                 float4* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int s = a.iperm[idx[t]];
  const float4 th = a.th[s];
  out[2 * t] = make_float4((float)a.pos[s].w, th.y, th.z, th.w);
  out[2 * t + 1] = a.fc[s];
}

__global__ void halo_unpack_kernel(SoA a, const int* __restrict__ idx, int n,
                                   const float4* __restrict__ in, int mask,
                                   unsigned int* hmax_bits) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int s = a.iperm[idx[t]];
  const float4 r0 = in[2 * t], r1 = in[2 * t + 1];
  if (mask & SWH_HALO_H) {
    a.pos[s].w = (double)r0.x;
    atomic_max_bits_if(hmax_bits, __float_as_uint(r0.x));
  }
  float4 th = a.th[s];
  if (mask & SWH_HALO_RHO) th.y = r0.y;
  if (mask & SWH_HALO_PC) {
    th.z = r0.z;
    th.w = r0.w;
  }
  a.th[s] = th;
  float4 fc = a.fc[s];
  if (mask & SWH_HALO_F_BALSARA) {
    fc.x = r1.x;
    fc.y = r1.y;
  }
  if (mask & SWH_HALO_ALPHAS) {
    fc.z = r1.z;
    fc.w = r1.w;
  }
  a.fc[s] = fc;
}

__global__ void pcell_kernel(const uint32_t* __restrict__ keys, const int* __restrict__ lin,
                             int64_t n, int ncell, int* __restrict__ pcell) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) pcell[s] = keys[s] < (uint32_t)ncell ? lin[keys[s]] : -1;
}

// xparts (caller order) -> v_full, a_grav (caller order; the drift reads them
// through perm)
__global__ void xunpack_kernel(swh_xpart_layout XL, const char* __restrict__ aos, int64_t n,
                               float4* __restrict__ vfull, float4* __restrict__ agrav) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const char* r = aos + i * XL.stride;
  const float* v = reinterpret_cast<const float*>(r + XL.off_v_full);
  vfull[i] = make_float4(v[0], v[1], v[2], 0.f);
  if (XL.off_a_grav >= 0) {
    const float* g = reinterpret_cast<const float*>(r + XL.off_a_grav);
    agrav[i] = make_float4(g[0], g[1], g[2], 0.f);
  } else {
    agrav[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// approx_expf (src/approx_math.h:35): 4th-order expansion used for |w| < 0.2
__device__ __forceinline__ float approx_expf(float x) {
  return 1.f + x * (1.f + x * (0.5f + x * (1.f / 6.f + 1.f / 24.f * x)));
}

struct DriftParams {
  double dt_drift, dt_kick_hydro, dt_kick_grav, dt_therm;
  float min_u;
};

// drift_part (src/drift.h:143-232) + SPHENIX hydro_predict_extra
// (hydro.h:1012-1066) per particle; float fields in the reference's float
// arithmetic, positions in double. dx_bits / h_bits: running maxima of the
// displacement since the rebuild and of h (float bits, positive).
// max |v_full| over the xparts (float bits; |v| >= 0 orders as its bits)
__global__ __launch_bounds__(256) void vmax_kernel(const float4* __restrict__ vfull, int64_t n,
                                                   unsigned int* vbits) {
  __shared__ float sm[4];
  float v = 0.f;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const float4 q = vfull[s];
    v = fmaxf(v, sqrtf(q.x * q.x + q.y * q.y + q.z * q.z));
  }
  block_max_bits(vbits, v, sm);
}

// xparts / gpart flags (caller order) -> sorted order
__global__ void xsort_kernel(const int* __restrict__ perm, const float4* __restrict__ vfull,
                             const float4* __restrict__ agrav, const int8_t* __restrict__ hasg,
                             int64_t n, float4* __restrict__ vfull_s, float4* __restrict__ agrav_s,
                             int8_t* __restrict__ hasg_s) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const int c = perm[s];
  vfull_s[s] = vfull[c];
  agrav_s[s] = agrav[c];
  hasg_s[s] = hasg[c];
}

__global__ __launch_bounds__(256) void drift_kernel(SoA a, const float4* __restrict__ vfull,
                             const float4* __restrict__ agrav, const int8_t* __restrict__ hasg,
                             float4* __restrict__ xdiff, int64_t n, DriftParams D,
                             unsigned int* dx_bits, unsigned int* h_bits) {
  __shared__ float sm[2][4];
  float dmax = 0.f, hm = 0.f;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    if (a.tb[s] == kTimeBinInhibited) continue;
    const int c = (int)s;  // vfull / agrav / hasg in sorted order (xsort_kernel)
    const float4 vf = vfull[c];
    double4 p = a.pos[s];
    p.x += (double)vf.x * D.dt_drift;
    p.y += (double)vf.y * D.dt_drift;
    p.z += (double)vf.z * D.dt_drift;
    float4 vm = a.vm[s];
    const float4 ac = a.acc[s];
    // float += float * double, as drift_part writes it
    vm.x = (float)((double)vm.x + (double)ac.x * D.dt_kick_hydro);
    vm.y = (float)((double)vm.y + (double)ac.y * D.dt_kick_hydro);
    vm.z = (float)((double)vm.z + (double)ac.z * D.dt_kick_hydro);
    if (hasg[c]) {
      const float4 ag = agrav[c];
      vm.x = (float)((double)vm.x + (double)ag.x * D.dt_kick_grav);
      vm.y = (float)((double)vm.y + (double)ag.y * D.dt_kick_grav);
      vm.z = (float)((double)vm.z + (double)ag.z * D.dt_kick_grav);
    }
    a.vm[s] = vm;
    // hydro_predict_extra
    float4 th = a.th[s];  // u, rho, P, c
    th.x += ac.w * (float)D.dt_therm;
    float h = (float)p.w;
    const float h_inv = 1.f / h;
    const float w1 = a.hdt[s] * h_inv * (float)D.dt_drift;
    h *= fabsf(w1) < 0.2f ? approx_expf(w1) : expf(w1);
    const float w2 = -3.f * w1;
    th.y *= fabsf(w2) < 0.2f ? approx_expf(w2) : expf(w2);
    th.x = fmaxf(th.x, 0.f);  // entropy floor NONE: floor_u = 0
    th.x = fmaxf(th.x, D.min_u);
    // EOS_IDEAL_GAS (equation_of_state.h:121-167)
    const float pressure = kHydroGammaMinusOne * th.x * th.y;
    const float soundspeed = sqrtf(kHydroGamma * pressure / th.y);
    th.z = pressure;
    th.w = soundspeed;
    a.th[s] = th;
    float4 gr = a.grad[s];
    gr.x = fmaxf(gr.x, 2.f * soundspeed);
    a.grad[s] = gr;
    p.w = (double)h;
    a.pos[s] = p;
    // offsets since the last rebuild (xp->x_diff)
    float4 xd = xdiff[s];
    xd.x -= (float)((double)vf.x * D.dt_drift);
    xd.y -= (float)((double)vf.y * D.dt_drift);
    xd.z -= (float)((double)vf.z * D.dt_drift);
    xdiff[s] = xd;
    dmax = fmaxf(dmax, sqrtf(xd.x * xd.x + xd.y * xd.y + xd.z * xd.z));
    hm = fmaxf(hm, h);
  }
  block_max_bits(dx_bits, dmax, sm[0]);
  block_max_bits(h_bits, hm, sm[1]);
}

// cell_start[c] = first sorted index with key >= c (c in [0, ncell]).
__global__ void cell_start_kernel(const uint32_t* __restrict__ keys, int64_t n, int ncell,
                                  int* __restrict__ start) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const int64_t prev = (i == 0) ? -1 : (int64_t)keys[i - 1];
  const int64_t cur = (i == n) ? (int64_t)ncell : (int64_t)keys[i];
  for (int64_t c = prev + 1; c <= cur; c++) start[c] = (int)i;
}

__global__ __launch_bounds__(256) void hmax_kernel(const double4* __restrict__ pos, const int8_t* __restrict__ tb,
                            int64_t n, unsigned int* out_bits) {
  __shared__ float sm[4];
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (tb[i] != kTimeBinInhibited) m = fmaxf(m, (float)pos[i].w);
  block_max_bits(out_bits, m, sm);
}


}  // namespace swh

using namespace swh;

// ---------------------------------------------------------------------------
// SoA views
// ---------------------------------------------------------------------------
namespace swh {

SoA soa_of(swh_space* s) {
  SoA a;
  a.pos = s->pos.as<double4>();
  a.vm = s->vm.as<float4>();
  a.th = s->th.as<float4>();
  a.fc = s->fc.as<float4>();
  a.tb = s->tb.as<int8_t>();
  a.dens = s->dens.as<float4>();
  a.rot = s->rot.as<float4>();
  a.grad = s->grad.as<float4>();
  a.acc = s->acc.as<float4>();
  a.hdt = s->hdt.as<float>();
  a.mintb = s->mintb.as<int8_t>();
  a.perm = s->perm.as<int>();
  a.iperm = s->iperm.as<int>();
  a.n_owned = (int)std::min<int64_t>(s->n_owned, INT32_MAX);
  return a;
}

static size_t soa_bytes_per_part() {
  return sizeof(double4) + 7 * sizeof(float4) + sizeof(float) + 2 * sizeof(int8_t) +
         sizeof(int);
}

// Carve a SoA view out of one contiguous scratch buffer.
static SoA soa_carve(char* base, int64_t n) {
  SoA a;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base + off;
    off += (bytes + 255) & ~size_t(255);
    return p;
  };
  a.pos = reinterpret_cast<double4*>(take(n * sizeof(double4)));
  a.vm = reinterpret_cast<float4*>(take(n * sizeof(float4)));
  a.th = reinterpret_cast<float4*>(take(n * sizeof(float4)));
  a.fc = reinterpret_cast<float4*>(take(n * sizeof(float4)));
  a.dens = reinterpret_cast<float4*>(take(n * sizeof(float4)));
  a.rot = reinterpret_cast<float4*>(take(n * sizeof(float4)));
  a.grad = reinterpret_cast<float4*>(take(n * sizeof(float4)));
  a.acc = reinterpret_cast<float4*>(take(n * sizeof(float4)));
  a.hdt = reinterpret_cast<float*>(take(n * sizeof(float)));
  a.perm = reinterpret_cast<int*>(take(n * sizeof(int)));
  a.iperm = nullptr;
  a.n_owned = INT32_MAX;
  a.tb = reinterpret_cast<int8_t*>(take(n));
  a.mintb = reinterpret_cast<int8_t*>(take(n));
  return a;
}

static swh_status copy_soa(const SoA& src, swh_space* s, hipStream_t st) {
  const int64_t n = s->n;
  SWH_HIP(hipMemcpyAsync(s->pos.ptr, src.pos, n * sizeof(double4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->vm.ptr, src.vm, n * sizeof(float4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->th.ptr, src.th, n * sizeof(float4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->fc.ptr, src.fc, n * sizeof(float4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->tb.ptr, src.tb, n, hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->dens.ptr, src.dens, n * sizeof(float4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->rot.ptr, src.rot, n * sizeof(float4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->grad.ptr, src.grad, n * sizeof(float4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->acc.ptr, src.acc, n * sizeof(float4), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->hdt.ptr, src.hdt, n * sizeof(float), hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->mintb.ptr, src.mintb, n, hipMemcpyDeviceToDevice, st));
  SWH_HIP(hipMemcpyAsync(s->perm.ptr, src.perm, n * sizeof(int), hipMemcpyDeviceToDevice, st));
  return SWH_OK;
}

static swh_status reserve_soa(swh_space* s, int64_t n) {
  SWH_TRY(s->pos.reserve(n * sizeof(double4)));
  SWH_TRY(s->vm.reserve(n * sizeof(float4)));
  SWH_TRY(s->th.reserve(n * sizeof(float4)));
  SWH_TRY(s->fc.reserve(n * sizeof(float4)));
  SWH_TRY(s->tb.reserve(n));
  SWH_TRY(s->dens.reserve(n * sizeof(float4)));
  SWH_TRY(s->rot.reserve(n * sizeof(float4)));
  SWH_TRY(s->grad.reserve(n * sizeof(float4)));
  SWH_TRY(s->acc.reserve(n * sizeof(float4)));
  SWH_TRY(s->hdt.reserve(n * sizeof(float)));
  SWH_TRY(s->mintb.reserve(n));
  SWH_TRY(s->perm.reserve(n * sizeof(int)));
  SWH_TRY(s->iperm.reserve(n * sizeof(int)));
  SWH_TRY(s->ncount.reserve(n * sizeof(int)));
  return SWH_OK;
}

swh_status space_hmax_to_device(swh_space* s) {
  if (!s->counters.ptr) {  // first use: every counter slot starts at zero
    SWH_TRY(s->counters.reserve(128));
    SWH_HIP(hipMemsetAsync(s->counters.ptr, 0, 128, s->stream));
  }
  unsigned int* hb = s->counters.as<unsigned int>() + 2;  // slot 2: hmax bits
  SWH_HIP(hipMemsetAsync(hb, 0, sizeof(unsigned int), s->stream));
  hipLaunchKernelGGL(hmax_kernel, dim3(1024), dim3(256), 0, s->stream, s->pos.as<double4>(),
                     s->tb.as<int8_t>(), s->n, hb);
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

}  // namespace swh

extern "C" {

swh_status swh_space_create(swh_context* ctx, swh_space** out) {
  if (!ctx || !out) return SWH_ERR_ARG;
  SWH_HIP(hipSetDevice(ctx->device));
  auto* s = new swh_space();
  s->ctx = ctx;
  hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete s;
    set_error("hipStreamCreate failed: %s", hipGetErrorString(e));
    return SWH_ERR_HIP;
  }
  *out = s;
  return SWH_OK;
}

swh_status swh_space_destroy(swh_space* s) {
  if (!s) return SWH_OK;
  (void)hipSetDevice(s->ctx->device);
  (void)hipStreamSynchronize(s->stream);
  DevBuf* bufs[] = {&s->aos, &s->pos, &s->vm, &s->th, &s->fc, &s->tb, &s->dens, &s->rot,
                    &s->grad, &s->acc, &s->hdt, &s->mintb, &s->perm, &s->ncount,
                    &s->cell_start, &s->cell_rank, &s->cell_code, &s->cell_span, &s->cell_hreach,
                    &s->vfull_c, &s->agrav_c, &s->hasg_c, &s->xdiff, &s->pcell, &s->cell_lin, &s->groups, &s->seg_groups,
                    &s->seg_off, &s->keys, &s->keys2, &s->idx, &s->idx2, &s->sort_tmp,
                    &s->scan_tmp, &s->counters, &s->tmp_soa, &s->ghost_left,
                    &s->ghost_right, &s->ghost_list, &s->ghost_list2, &s->ghost_search, &s->ghost_seg, &s->grown_q,
                    &s->grown_mark, &s->grown_search,
                    &s->nbr, &s->nbr_cnt, &s->nbr_base, &s->nbr_reach, &s->nbr_ovf, &s->posf, &s->gplan, &s->ctr_stripes,
                    &s->iperm, &s->vfull_s, &s->agrav_s, &s->hasg_s, &s->list_xd0};
  for (DevBuf* b : bufs) b->release();
  s->hstage.release();
  s->ghost_host.release();
  if (s->own_stream && s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
  return SWH_OK;
}

swh_status swh_space_set_stream(swh_space* s, void* stream) {
  if (!s) return SWH_ERR_ARG;
  if (stream) {
    if (s->own_stream && s->stream) {
      (void)hipStreamSynchronize(s->stream);
      (void)hipStreamDestroy(s->stream);
    }
    s->stream = reinterpret_cast<hipStream_t>(stream);
    s->own_stream = false;
  }
  return SWH_OK;
}

swh_status swh_space_set_tuning(swh_space* s, const swh_tuning* t) {
  if (!s || !t || t->cell_factor < 1 || t->cell_factor > 4 ||
      (t->loop_variant != 0 && t->loop_variant != 7) ||
      (t->group_size != 0 && t->group_size != 16) || t->cell_scale < 0.f || t->cell_scale > 4.f ||
      t->diag_mode < 0 || t->diag_mode > 7 || t->diag_mode == 5 ||
      t->diag_mode == 6 || t->list_capacity < 0 || t->list_capacity > 4096 ||
      (t->list_capacity % 4) != 0 || !(t->list_skin >= 0.f) || t->list_skin > 1.f ||
      t->list_keep < 0 || t->list_keep > 1)
    return SWH_ERR_ARG;
  s->tuning = *t;
  s->built = false;
  s->list_valid = false;
  s->list_check = false;
  return SWH_OK;
}

int64_t swh_space_count(const swh_space* s) { return s ? s->n : 0; }

swh_status swh_space_get_info(const swh_space* s, swh_space_info* info) {
  if (!s || !info) return SWH_ERR_ARG;
  std::memset(info, 0, sizeof(*info));
  for (int k = 0; k < 3; k++) {
    info->cdim[k] = s->grid.cdim[k];
    info->cell_width[k] = s->grid.w[k];
  }
  info->ncell = s->grid.ncell;
  info->ngroups = s->ngroups;
  info->h_max = s->grid.hmax;
  for (int k = 0; k < 4; k++) info->loop_stats[k] = s->loop_stats[k];
  info->list_entries = s->list_entries;
  info->list_overflow = s->list_overflow;
  info->list_valid = s->list_valid ? 1 : 0;
  info->dx_max = s->grid.dx;
  if (s->counters.ptr) {  // list builds that ran on the device (u32[26])
    unsigned int nb = 0;
    SWH_HIP(hipMemcpyAsync(&nb, s->counters.as<unsigned int>() + 26, sizeof(nb),
                           hipMemcpyDeviceToHost, s->stream));
    SWH_HIP(hipStreamSynchronize(s->stream));
    info->list_builds = nb;
  }
  return SWH_OK;
}

swh_status swh_space_upload_xparts(swh_space* s, const void* xparts, int64_t count,
                                   const swh_xpart_layout* XL, int on_device) {
  if (!s || !XL || (count > 0 && !xparts) || count != s->n || XL->stride <= 0 ||
      XL->off_v_full < 0 || XL->off_v_full + 12 > XL->stride ||
      (XL->off_a_grav >= 0 && XL->off_a_grav + 12 > XL->stride)) {
    set_error("xparts must match the uploaded parts (count %lld) with v_full in the record",
              (long long)s->n);
    return SWH_ERR_ARG;
  }
  if (count == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  SWH_TRY(s->vfull_c.reserve((size_t)count * sizeof(float4)));
  SWH_TRY(s->agrav_c.reserve((size_t)count * sizeof(float4)));
  SWH_TRY(s->tmp_soa.reserve((size_t)count * XL->stride));
  SWH_HIP(hipMemcpyAsync(s->tmp_soa.ptr, xparts, (size_t)count * XL->stride,
                         on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                         s->stream));
  hipLaunchKernelGGL(xunpack_kernel, dim3((int)((count + 255) / 256)), dim3(256), 0, s->stream,
                     *XL, s->tmp_soa.as<const char>(), count, s->vfull_c.as<float4>(),
                     s->agrav_c.as<float4>());
  SWH_HIP(hipGetLastError());
  // the fastest particle bounds every displacement of the following drifts
  // (v_full is fixed until the next upload), so the drift needs no read-back
  if (!s->counters.ptr) {
    SWH_TRY(s->counters.reserve(128));
    SWH_HIP(hipMemsetAsync(s->counters.ptr, 0, 128, s->stream));
  }
  unsigned int* vbits = s->counters.as<unsigned int>() + 21;
  SWH_HIP(hipMemsetAsync(vbits, 0, sizeof(unsigned int), s->stream));
  hipLaunchKernelGGL(vmax_kernel, dim3((int)std::min<int64_t>((count + 255) / 256, kReduceBlocks)), dim3(256), 0, s->stream,
                     s->vfull_c.as<const float4>(), count, vbits);
  SWH_HIP(hipGetLastError());
  unsigned int vb = 0;
  SWH_HIP(hipMemcpyAsync(&vb, vbits, sizeof(vb), hipMemcpyDeviceToHost, s->stream));
  SWH_HIP(hipStreamSynchronize(s->stream));
  float vmax;
  std::memcpy(&vmax, &vb, sizeof(vmax));
  s->vfull_max = (double)vmax;
  s->xparts_valid = true;
  s->xsorted_valid = false;
  return SWH_OK;
}

swh_status swh_space_drift(swh_space* s, const swh_drift_params* D, const swh_hydro_params* P) {
  if (!s || !D || !P) return SWH_ERR_ARG;
  if (!s->built) {
    set_error("swh_space_rebuild must precede the drift");
    return SWH_ERR_STATE;
  }
  if (s->n == 0) return SWH_OK;
  if (!s->xparts_valid) {
    set_error("swh_space_upload_xparts must precede the drift");
    return SWH_ERR_STATE;
  }
  SWH_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->stream;
  DriftParams dp{D->dt_drift, D->dt_kick_hydro, D->dt_kick_grav, D->dt_therm, D->min_u};
  unsigned int* ctr = s->counters.as<unsigned int>();
  unsigned int* dx_bits = ctr + 19;  // counter slot 19: drift displacement
  SWH_HIP(hipMemsetAsync(dx_bits, 0, sizeof(unsigned int), st));
  if (!s->xsorted_valid) {
    SWH_TRY(s->vfull_s.reserve((size_t)s->n * sizeof(float4)));
    SWH_TRY(s->agrav_s.reserve((size_t)s->n * sizeof(float4)));
    SWH_TRY(s->hasg_s.reserve((size_t)s->n));
    hipLaunchKernelGGL(xsort_kernel, dim3((int)((s->n + 255) / 256)), dim3(256), 0, st,
                       s->perm.as<const int>(), s->vfull_c.as<const float4>(),
                       s->agrav_c.as<const float4>(), s->hasg_c.as<const int8_t>(), s->n,
                       s->vfull_s.as<float4>(), s->agrav_s.as<float4>(), s->hasg_s.as<int8_t>());
    s->xsorted_valid = true;
  }
  hipLaunchKernelGGL(drift_kernel, dim3((int)std::min<int64_t>((s->n + 255) / 256, 4 * kReduceBlocks)), dim3(256), 0, st, soa_of(s),
                     s->vfull_s.as<const float4>(), s->agrav_s.as<const float4>(),
                     s->hasg_s.as<const int8_t>(), s->xdiff.as<float4>(), s->n, dp, dx_bits,
                     ctr + 2);
  SWH_HIP(hipGetLastError());
  // every loop widens its reach by the displacement since the rebuild: bounded
  // by |v_full|_max * dt per drift (the drift kernel keeps the exact per-particle
  // offsets for the next rebuild); no device read-back, the drift stays
  // asynchronous. The periodic reach check (h grown past half the box) runs
  // at the next ghost and rebuild.
  s->grid.dx += s->vfull_max * std::fabs(D->dt_drift) * (1. + 1e-6) + 1e-12;
  // positions moved: kept lists (list_keep) are checked against their skin on
  // the device before the next loop uses them; otherwise they are rebuilt
  if (s->list_valid && (s->tuning.list_keep || s->tuning.diag_mode == 7))
    s->list_check = true;
  else
    s->list_valid = false;
  return SWH_OK;
}

swh_status swh_space_sync(swh_space* s) {
  if (!s) return SWH_ERR_ARG;
  SWH_HIP(hipStreamSynchronize(s->stream));
  return SWH_OK;
}

swh_status swh_space_query(swh_space* s) {
  if (!s) return SWH_ERR_ARG;
  const hipError_t e = hipStreamQuery(s->stream);
  if (e == hipErrorNotReady) return SWH_BUSY;
  SWH_HIP(e);
  return SWH_OK;
}

swh_status swh_space_upload_parts(swh_space* s, const void* parts, int64_t count,
                                  const swh_part_layout* PL, int on_device) {
  if (!s || (count > 0 && !parts) || count < 0 || count > INT32_MAX / 2 || !PL)
    return SWH_ERR_ARG;
  Layout L;
  SWH_TRY(make_layout(PL, &L));
  SWH_HIP(hipSetDevice(s->ctx->device));
  s->layout = L;
  s->n = count;
  s->n_owned = count;
  s->built = false;
  s->list_valid = false;
  if (count == 0) return SWH_OK;
  const size_t bytes = (size_t)count * L.stride;
  SWH_TRY(s->aos.reserve(bytes));
  SWH_TRY(reserve_soa(s, count));
  SWH_HIP(hipMemcpyAsync(s->aos.ptr, parts, bytes,
                         on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                         s->stream));
  const int block = 256;
  const int grid = (int)((count + block - 1) / block);
  SWH_TRY(s->hasg_c.reserve((size_t)count));
  s->xparts_valid = false;
  s->xsorted_valid = false;
  s->grid.dx = 0.;
  hipLaunchKernelGGL(unpack_kernel, dim3(grid), dim3(block), 0, s->stream, L,
                     s->aos.as<const char>(), count, soa_of(s), s->hasg_c.as<int8_t>());
  SWH_HIP(hipGetLastError());
  if (!on_device) SWH_HIP(hipStreamSynchronize(s->stream));  // caller may reuse `parts`
  return SWH_OK;
}

swh_status swh_space_download_parts(swh_space* s, void* parts, const swh_part_layout* PL,
                                    int fields, int on_device) {
  if (!s || (s->n > 0 && !parts) || !PL) return SWH_ERR_ARG;
  Layout L;
  SWH_TRY(make_layout(PL, &L));
  if (L.stride != s->layout.stride) {
    set_error("download layout stride differs from upload");
    return SWH_ERR_ARG;
  }
  if (s->n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  const int block = 256;
  const int grid = (int)((s->n + block - 1) / block);
  hipLaunchKernelGGL(pack_kernel, dim3(grid), dim3(block), 0, s->stream, L,
                     s->aos.as<char>(), s->n, soa_of(s), fields);
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemcpyAsync(parts, s->aos.ptr, (size_t)s->n * L.stride,
                         on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                         s->stream));
  SWH_HIP(hipStreamSynchronize(s->stream));
  return SWH_OK;
}

swh_status swh_space_set_owned(swh_space* s, int64_t n_owned) {
  if (!s || n_owned < 0 || n_owned > s->n) return SWH_ERR_ARG;
  s->n_owned = n_owned;
  s->list_valid = false;  // the lists hold owned (active) particles only
  return SWH_OK;
}

static swh_status halo_check(swh_space* s, const int32_t* idx, int32_t n, const void* buf) {
  if (!s || n < 0 || (n > 0 && (!idx || !buf))) return SWH_ERR_ARG;
  if (n > 0 && !s->built) {
    set_error("swh_space_rebuild must precede the halo exchange");
    return SWH_ERR_STATE;
  }
  return SWH_OK;
}

swh_status swh_space_pack_halo(swh_space* s, const int32_t* idx, int32_t n, float* out) {
  SWH_TRY(halo_check(s, idx, n, out));
  if (n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  hipLaunchKernelGGL(halo_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, s->stream,
                     soa_of(s), idx, n, reinterpret_cast<float4*>(out));
  SWH_HIP(hipGetLastError());
  return SWH_OK;
}

swh_status swh_space_unpack_halo(swh_space* s, const int32_t* idx, int32_t n, const float* in,
                                 int fields) {
  SWH_TRY(halo_check(s, idx, n, in));
  if (fields & ~SWH_HALO_ALL) return SWH_ERR_ARG;
  if (n == 0) return SWH_OK;
  SWH_HIP(hipSetDevice(s->ctx->device));
  hipLaunchKernelGGL(halo_unpack_kernel, dim3((n + 255) / 256), dim3(256), 0, s->stream,
                     soa_of(s), idx, n, reinterpret_cast<const float4*>(in), fields,
                     s->counters.as<unsigned int>() + 2);
  SWH_HIP(hipGetLastError());
  // a halo h that grew can bring new force pairs (r < H_j): relist
  if (fields & SWH_HALO_H) s->list_valid = false;
  return SWH_OK;
}

swh_status swh_space_rebuild(swh_space* s, const swh_hydro_params* P, double min_cell_width) {
  if (!s || !P) return SWH_ERR_ARG;
  const int64_t n = s->n;
  if (n == 0) {
    s->built = true;
    return SWH_OK;
  }
  SWH_HIP(hipSetDevice(s->ctx->device));
  hipStream_t st = s->stream;
  s->list_valid = false;
  s->xsorted_valid = false;  // the sort order changes
  // 1. bounding box + max h
  const int nb = 512;
  SWH_TRY(s->scan_tmp.reserve(nb * 8 * sizeof(double)));
  SWH_TRY(s->hstage.reserve(nb * 8 * sizeof(double)));
  hipLaunchKernelGGL(bbox_kernel, dim3(nb), dim3(256), 0, st, s->pos.as<double4>(),
                     s->tb.as<int8_t>(), n, s->scan_tmp.as<double>());
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemcpyAsync(s->hstage.ptr, s->scan_tmp.ptr, nb * 8 * sizeof(double),
                         hipMemcpyDeviceToHost, st));
  SWH_HIP(hipStreamSynchronize(st));
  const double* hb = static_cast<const double*>(s->hstage.ptr);
  double bb[8] = {1e300, 1e300, 1e300, -1e300, -1e300, -1e300, 0., 0.};
  for (int b = 0; b < nb; b++) {
    for (int k = 0; k < 3; k++) bb[k] = std::min(bb[k], hb[b * 8 + k]);
    for (int k = 3; k < 7; k++) bb[k] = std::max(bb[k], hb[b * 8 + k]);
    bb[7] += hb[b * 8 + 7];
  }
  SwhGrid& g = s->grid;
  g.periodic = P->periodic;
  g.hmax = bb[6] * (double)kGamma;
  const double cells_per_h = s->tuning.cell_scale > 0.f ? (double)s->tuning.cell_scale
                                                       : (double)std::max(1, s->tuning.cell_factor);
  // Cell width: the largest kernel reach H_max when h is near-uniform (a
  // group's neighbourhood is then its 27 cells). When h spans a wide range
  // (clustered boxes) cells sized by H_max would hold whole clumps: size them
  // by the typical H instead (the geometric mean, at least H_max / 6: on the
  // EAGLE stand-in 0.75 x and H_max / 8 enumerated more cells per group and
  // took 1.72 against 1.66 ms per density loop), divided by 1.1 since the
  // build stages two candidates per lane per pass (EAGLE stand-in: cdim 86 ->
  // 94, density loop 1.59 -> 1.45 ms; profiles/r05z5_eagle_cell_sweep.txt);
  // the large-h particles then reach over more cells, and the list build
  // prunes cells by their own maximum H (SWIFT's per-cell h_max in DOPAIR2,
  // runner_doiact_functions_hydro.h:1424-1530).
  const double h_geo = std::exp(bb[7] / (double)n) * (double)kGamma;
  g.adaptive = g.hmax > 1.5 * h_geo;
  const double h_cell = g.adaptive ? std::max(h_geo, g.hmax / 6.) / 1.1 : g.hmax;
  double width = min_cell_width > 0 ? min_cell_width : h_cell / cells_per_h;
  if (!(width > 0)) width = 1.0;
  int64_t total = 1;
  for (int k = 0; k < 3; k++) {
    if (g.periodic) {
      g.origin[k] = 0.;
      g.dim[k] = P->dim[k];
    } else {
      const double ext = std::max(bb[k + 3] - bb[k], 1e-300);
      g.origin[k] = bb[k];
      g.dim[k] = ext * (1. + 1e-12) + 1e-300;
    }
    int c = (int)std::floor(g.dim[k] / width);
    c = std::max(1, std::min(c, 1024));
    g.cdim[k] = c;
    total *= c;
  }
  // keep the cell count bounded (memory and scan cost)
  while (total > std::max<int64_t>(64, 8 * n) && total > 27) {
    total = 1;
    for (int k = 0; k < 3; k++) {
      g.cdim[k] = std::max(1, g.cdim[k] * 3 / 4);
      total *= g.cdim[k];
    }
  }
  for (int k = 0; k < 3; k++) g.w[k] = g.dim[k] / g.cdim[k];
  g.ncell = (int)total;
  if (g.periodic) {
    // the loops take the nearest periodic image only: the kernel reach must
    // stay below half the box (runner_doiact_functions_hydro.h:2283)
    const double dmin = std::min(g.dim[0], std::min(g.dim[1], g.dim[2]));
    if (g.hmax >= 0.5 * dmin) {
      s->built = false;
      swh::set_error("Cell smaller than smoothing length: gamma*h_max=%g, box %g", g.hmax, dmin);
      return SWH_ERR_CELL_SMALL;
    }
  }
  const int block = 256;
  const int64_t nsort = std::max<int64_t>(n, g.ncell);
  SWH_TRY(s->keys.reserve(nsort * sizeof(uint32_t)));
  SWH_TRY(s->keys2.reserve(nsort * sizeof(uint32_t)));
  SWH_TRY(s->idx.reserve(nsort * sizeof(int)));
  SWH_TRY(s->idx2.reserve(nsort * sizeof(int)));
  // 2a. Morton rank of every cell (cached per grid shape)
  if (s->rank_cdim[0] != g.cdim[0] || s->rank_cdim[1] != g.cdim[1] ||
      s->rank_cdim[2] != g.cdim[2]) {
    SWH_TRY(s->cell_rank.reserve((size_t)g.ncell * sizeof(int)));
    const int cg = (g.ncell + block - 1) / block;
    hipLaunchKernelGGL(morton_kernel, dim3(cg), dim3(block), 0, st, g.cdim[0], g.cdim[1],
                       g.ncell, s->keys.as<uint32_t>(), s->idx.as<int>());
    SWH_HIP(hipGetLastError());
    size_t mb = 0;
    SWH_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, mb, s->keys.as<uint32_t>(),
                                               s->keys2.as<uint32_t>(), s->idx.as<int>(),
                                               s->idx2.as<int>(), g.ncell, 0, 30, st));
    SWH_TRY(s->sort_tmp.reserve(mb));
    SWH_HIP(hipcub::DeviceRadixSort::SortPairs(s->sort_tmp.ptr, mb, s->keys.as<uint32_t>(),
                                               s->keys2.as<uint32_t>(), s->idx.as<int>(),
                                               s->idx2.as<int>(), g.ncell, 0, 30, st));
    hipLaunchKernelGGL(rank_scatter_kernel, dim3(cg), dim3(block), 0, st,
                       s->idx2.as<const int>(), g.ncell, s->cell_rank.as<int>());
    SWH_HIP(hipGetLastError());
    SWH_TRY(s->cell_code.reserve((size_t)g.ncell * sizeof(uint32_t)));
    SWH_HIP(hipMemcpyAsync(s->cell_code.ptr, s->keys2.ptr, (size_t)g.ncell * sizeof(uint32_t),
                           hipMemcpyDeviceToDevice, st));
    SWH_TRY(s->cell_lin.reserve((size_t)g.ncell * sizeof(int)));
    SWH_HIP(hipMemcpyAsync(s->cell_lin.ptr, s->idx2.ptr, (size_t)g.ncell * sizeof(int),
                           hipMemcpyDeviceToDevice, st));
    for (int k = 0; k < 3; k++) s->rank_cdim[k] = g.cdim[k];
  }
  SWH_TRY(s->cell_start.reserve(((size_t)g.ncell + 1) * sizeof(int)));
  GridDev gd = grid_dev(s);
  // 2b. keys (Morton rank of the cell) + stable radix sort
  const int grid = (int)((n + block - 1) / block);
  int end_bit = 1;
  while ((1LL << end_bit) <= (int64_t)g.ncell) end_bit++;
  // in-cell Morton bits per dimension (at most 3, within the 32-bit key)
  int sub_bits = std::min(3, (32 - end_bit) / 3);
  if (const char* e = std::getenv("SWH_SUBCELL_BITS")) sub_bits = std::max(0, std::min(sub_bits, std::atoi(e)));
  hipLaunchKernelGGL(key_kernel, dim3(grid), dim3(block), 0, st, gd,
                     s->cell_rank.as<const int>(), s->pos.as<double4>(),
                     s->tb.as<const int8_t>(), n, g.ncell, sub_bits, s->keys.as<uint32_t>(),
                     s->idx.as<int>());
  SWH_HIP(hipGetLastError());
  end_bit += 3 * sub_bits;
  size_t tmp_bytes = 0;
  SWH_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, s->keys.as<uint32_t>(),
                                             s->keys2.as<uint32_t>(), s->idx.as<int>(),
                                             s->idx2.as<int>(), (int)n, 0, end_bit, st));
  SWH_TRY(s->sort_tmp.reserve(tmp_bytes));
  SWH_HIP(hipcub::DeviceRadixSort::SortPairs(s->sort_tmp.ptr, tmp_bytes,
                                             s->keys.as<uint32_t>(), s->keys2.as<uint32_t>(),
                                             s->idx.as<int>(), s->idx2.as<int>(), (int)n, 0,
                                             end_bit, st));
  if (sub_bits > 0) {
    hipLaunchKernelGGL(key_shift_kernel, dim3(grid), dim3(block), 0, st, s->keys2.as<uint32_t>(),
                       n, 3 * sub_bits);
    SWH_HIP(hipGetLastError());
  }
  // 3. permute SoA into cell order
  SWH_TRY(s->tmp_soa.reserve((size_t)n * soa_bytes_per_part() + 16 * 256));
  SoA tmp = soa_carve(s->tmp_soa.as<char>(), n);
  hipLaunchKernelGGL(permute_kernel, dim3(grid), dim3(block), 0, st, soa_of(s), tmp,
                     s->idx2.as<const int>(), n);
  SWH_HIP(hipGetLastError());
  SWH_TRY(copy_soa(tmp, s, st));
  hipLaunchKernelGGL(iperm_kernel, dim3(grid), dim3(block), 0, st, s->perm.as<const int>(), n,
                     s->iperm.as<int>());
  SWH_HIP(hipGetLastError());
  // 4. cell starts
  hipLaunchKernelGGL(cell_start_kernel, dim3((int)((n + 1 + block - 1) / block)), dim3(block),
                     0, st, s->keys2.as<const uint32_t>(), n, g.ncell,
                     s->cell_start.as<int>());
  SWH_HIP(hipGetLastError());
  // 4a. each particle's sorted cell (posf is relative to it; a drift moves
  // particles without re-binning them) and a fresh displacement record
  SWH_TRY(s->pcell.reserve((size_t)n * sizeof(int)));
  SWH_TRY(s->xdiff.reserve((size_t)n * sizeof(float4)));
  hipLaunchKernelGGL(pcell_kernel, dim3(grid), dim3(block), 0, st, s->keys2.as<const uint32_t>(),
                     s->cell_lin.as<const int>(), n, g.ncell, s->pcell.as<int>());
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemsetAsync(s->xdiff.ptr, 0, (size_t)n * sizeof(float4), st));
  g.dx = 0.;
  // 4b. per-linear-cell span table (one load per cell lookup in the loops)
  SWH_TRY(s->cell_span.reserve((size_t)g.ncell * sizeof(int2)));
  hipLaunchKernelGGL(span_kernel, dim3((g.ncell + block - 1) / block), dim3(block), 0, st,
                     s->cell_rank.as<const int>(), s->cell_start.as<const int>(), g.ncell,
                     s->cell_span.as<int2>());
  SWH_HIP(hipGetLastError());
  // 5. i-groups of the tile loops
  const int nc = g.ncell;
  const int gmax = s->tuning.group_size > 0 ? s->tuning.group_size : 16;
  SWH_TRY(s->seg_groups.reserve(((size_t)nc + 1) * sizeof(int)));
  SWH_TRY(s->seg_off.reserve(((size_t)nc + 1) * sizeof(int)));
  const int cgrid = (nc + block - 1) / block;
  hipLaunchKernelGGL(group_kernel<false>, dim3(cgrid), dim3(block), 0, st,
                     s->cell_code.as<const uint32_t>(), s->cell_start.as<const int>(), nc,
                     gmax, s->seg_groups.as<int>(), nullptr, nullptr);
  SWH_HIP(hipGetLastError());
  SWH_HIP(hipMemsetAsync(s->seg_groups.as<int>() + nc, 0, sizeof(int), st));
  size_t sb = 0;
  SWH_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, s->seg_groups.as<int>(),
                                           s->seg_off.as<int>(), nc + 1, st));
  SWH_TRY(s->scan_tmp.reserve(std::max(sb, (size_t)nb * 7 * sizeof(double))));
  SWH_HIP(hipcub::DeviceScan::ExclusiveSum(s->scan_tmp.ptr, sb, s->seg_groups.as<int>(),
                                           s->seg_off.as<int>(), nc + 1, st));
  int ng = 0;
  SWH_HIP(hipMemcpyAsync(&ng, s->seg_off.as<int>() + nc, sizeof(int), hipMemcpyDeviceToHost,
                         st));
  SWH_HIP(hipStreamSynchronize(st));
  s->ngroups = ng;
  SWH_TRY(s->groups.reserve(((size_t)ng + 1) * sizeof(int2)));
  hipLaunchKernelGGL(group_kernel<true>, dim3(cgrid), dim3(block), 0, st,
                     s->cell_code.as<const uint32_t>(), s->cell_start.as<const int>(), nc,
                     gmax, nullptr, s->seg_off.as<const int>(), s->groups.as<int2>());
  SWH_HIP(hipGetLastError());
  SWH_TRY(space_hmax_to_device(s));
  s->built = true;
  return SWH_OK;
}

}  // extern "C"
