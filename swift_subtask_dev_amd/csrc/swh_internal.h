// swh_internal.h — host/device shared internals of libswifthip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "swifthip.h"

namespace swh {

// ---------------------------------------------------------------------------
// Errors: thread-local message + status codes, no aborts.
// ---------------------------------------------------------------------------
void set_error(const char* fmt, ...);

#define SWH_HIP(call)                                                           \
  do {                                                                          \
    hipError_t _e = (call);                                                     \
    if (_e != hipSuccess) {                                                     \
      ::swh::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(_e),   \
                       __FILE__, __LINE__);                                     \
      return (_e == hipErrorOutOfMemory) ? SWH_ERR_OOM : SWH_ERR_HIP;           \
    }                                                                           \
  } while (0)

#define SWH_TRY(expr)                      \
  do {                                     \
    swh_status _s = (expr);                \
    if (_s != SWH_OK) return _s;           \
  } while (0)

// Growable device buffer (never shrinks; reused across calls so the loops do
// no allocation once warm).
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  swh_status reserve(size_t b) {
    if (b <= bytes) return SWH_OK;
    if (ptr) {
      hipError_t e = hipFree(ptr);
      (void)e;
      ptr = nullptr;
      bytes = 0;
    }
    size_t nb = b < 256 ? 256 : b;
    hipError_t e = hipMalloc(&ptr, nb);
    if (e != hipSuccess) {
      set_error("hipMalloc(%zu) failed: %s", nb, hipGetErrorString(e));
      return SWH_ERR_OOM;
    }
    bytes = nb;
    return SWH_OK;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  template <typename T>
  T* as() const { return reinterpret_cast<T*>(ptr); }
};

// Pinned host staging buffer.
struct HostBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  swh_status reserve(size_t b) {
    if (b <= bytes) return SWH_OK;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    size_t nb = b < 4096 ? 4096 : b;
    hipError_t e = hipHostMalloc(&ptr, nb, hipHostMallocDefault);
    if (e != hipSuccess) {
      set_error("hipHostMalloc(%zu) failed: %s", nb, hipGetErrorString(e));
      bytes = 0;
      return SWH_ERR_OOM;
    }
    bytes = nb;
    return SWH_OK;
  }
  void release() {
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
};

// Device copy of the AoS layout (offsets), passed by value to kernels.
struct Layout {
  int stride;
  int id, x, v, a_hydro, mass, h, u, u_dt, rho;
  int div_v, div_v_dt, div_v_prev, visc_alpha, v_sig;
  int laplace_u, diff_alpha;
  int wcount, wcount_dh, rho_dh, rot_v;
  int f, pressure, soundspeed, h_dt, balsara, avmn;
  int time_bin, min_tb;
  int gpart;  // struct gpart* (-1: none)
};
swh_status make_layout(const swh_part_layout* L, Layout* out);

struct GLayout {
  int stride, x, a_grav, potential, mass, epsilon, time_bin;
  int old_a_grav_norm;  // -1: not in the record (the adaptive MAC then sees 0)
};
swh_status make_glayout(const swh_gpart_layout* L, GLayout* out);

// Per-task worker: one stream + staging buffers, leased per host thread.
struct TaskWorker {
  hipStream_t stream = nullptr;
  DevBuf dparts, dparts2, dind, dself, dcount;
  HostBuf hstage, hstage2;
  std::mutex busy;
};

}  // namespace swh

struct swh_context {
  int device = 0;
  swh_precision precision = SWH_PRECISION_F64;
  int num_cus = 256;
  std::mutex lease_mutex;
  std::vector<swh::TaskWorker*> workers;
  swh::TaskWorker* lease();
  void unlease(swh::TaskWorker* w);
};

// Neighbour grid of the batch path.
struct SwhGrid {
  int cdim[3] = {0, 0, 0};
  double w[3] = {0, 0, 0};       // cell widths
  double origin[3] = {0, 0, 0};  // lower corner of the gridded domain
  double dim[3] = {0, 0, 0};     // box (periodic) or domain extent
  int periodic = 0;
  int ncell = 0;
  double hmax = 0;  // max H = gamma*h over all particles at rebuild
  bool adaptive = false;  // cells sized by the typical H (h spans a wide range)
  double dx = 0;    // largest displacement since the rebuild (drift): loops widen their reach
};

// swh_tuning.list_skin of a new space (swifthip.h SWH_DEFAULT_LIST_SKIN)
constexpr float kDefaultListSkin = SWH_DEFAULT_LIST_SKIN;

// Device-resident particle set, sorted by grid cell in Morton order of the
// cells (cell_rank maps a linear x-fastest cell index to its Morton rank).
struct swh_space {
  swh_context* ctx = nullptr;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  int64_t n = 0;
  bool built = false;
  SwhGrid grid;
  swh_tuning tuning{1, 0, 0, 0.f, 0, 0, kDefaultListSkin, 0};

  // AoS image of the caller's records (for write-back of untouched fields)
  swh::DevBuf aos;
  swh::Layout layout{};

  // sorted SoA (j-records packed for gathers)
  swh::DevBuf pos;   // double4 x,y,z,h
  swh::DevBuf vm;    // float4 vx,vy,vz,m
  swh::DevBuf th;    // float4 u,rho,P,c
  swh::DevBuf fc;    // float4 f,balsara,alpha_visc,alpha_diff
  swh::DevBuf tb;    // int8 time_bin
  // i-side state/outputs (sorted order), float unless noted
  swh::DevBuf dens;  // float4 rho_dh, wcount, wcount_dh, div_v
  swh::DevBuf rot;   // float4 rot_x, rot_y, rot_z, laplace_u
  swh::DevBuf grad;  // float4 v_sig, alpha_visc_max_ngb, div_v_prev, div_v_dt
  swh::DevBuf acc;   // float4 ax, ay, az, u_dt
  swh::DevBuf hdt;   // float h_dt
  swh::DevBuf mintb; // int8 min_ngb_time_bin
  swh::DevBuf perm;  // int32 sorted index -> caller index
  swh::DevBuf iperm; // int32 caller index -> sorted index
  int64_t n_owned = 0;  // caller indices >= n_owned: foreign halo (swh_space_set_owned)
  swh::DevBuf ncount;  // int32 per-particle interaction count (diagnostic)
  // drift (swh_space_drift): caller-order xpart data and the gpart flag,
  // sorted-order displacement since the rebuild and the sorted cell of each
  // particle (positions relative to it in posf stay valid when it drifts out)
  swh::DevBuf vfull_c, agrav_c, hasg_c, xdiff, pcell, cell_lin;
  // the xparts and gpart flags in sorted order (gathered once per rebuild /
  // upload, so every drift streams them)
  swh::DevBuf vfull_s, agrav_s, hasg_s;
  bool xsorted_valid = false;
  bool xparts_valid = false;
  double vfull_max = 0.;  // max |v_full| of the uploaded xparts (drift displacement bound)
  // grid
  swh::DevBuf cell_start;  // int32[ncell+1], indexed by Morton rank
  swh::DevBuf cell_rank;   // int32[ncell]: linear cell -> Morton rank
  swh::DevBuf cell_code;   // uint32[ncell]: Morton code of each rank (ascending)
  swh::DevBuf cell_span;   // int2[ncell]: linear cell -> sorted range
  swh::DevBuf cell_hreach; // float[ncell]: max R = gamma h (1 + skin) of the cell (list build)
  int rank_cdim[3] = {0, 0, 0};  // grid the rank table was built for
  swh::DevBuf groups;      // int2[ngroups]: i-groups (start, count) of the tile loops
  swh::DevBuf seg_groups, seg_off;
  int32_t ngroups = 0;
  int64_t loop_stats[4] = {0, 0, 0, 0};  // work counters of the last counted tile loop
  // the step's pair lists (swh_list.h): valid from a density loop until the
  // next upload / rebuild / tuning change, or a ghost that grows an H past its R
  swh::DevBuf nbr, nbr_cnt, nbr_base, nbr_reach, nbr_ovf;
  swh::DevBuf posf;  // float4: position relative to its grid cell's corner, h
  swh::DevBuf gplan;  // BuildPlan per i-group: the list build's wave-uniform setup
  swh::DevBuf list_xd0;  // float4: the displacement record (xdiff) at the list build
  bool list_valid = false;
  bool xd0_zero = false;  // list_xd0 is logically zero (built with no drift since the re-bin)
  bool list_check = false;  // kept lists after a drift: the device checks them first
  // particles the ghost converged with H past their list reach (queue
  // grown_q, u32[17]): the gradient / force loops search them (and, force,
  // their neighbours within H) instead of rebuilding every list
  int32_t grown_n = 0;
  swh::DevBuf grown_q, grown_mark, grown_search;
  int32_t list_mab = 0, list_K = 0;
  float list_skin_cur = 0.f;  // skin of the lists in use (tuning, or the ghost's rebuild)
  int64_t list_entries = 0;   // last counted build: total entries
  int32_t list_overflow = 0;  // last counted build: particles over capacity
  // scratch
  swh::DevBuf keys, keys2, idx, idx2, sort_tmp, scan_tmp, counters;
  swh::DevBuf ctr_stripes;  // counted launches' per-block counter stripes (swh_hydro.hip)
  swh::DevBuf tmp_soa;     // staging for permutation gathers
  swh::DevBuf ghost_left, ghost_right, ghost_list, ghost_list2, ghost_search;
  swh::DevBuf ghost_seg;  // 2 x (kSegs + 1) counts of the ghost's rerun lists
  swh::HostBuf ghost_host;  // pinned: the passes' counts read back
  unsigned int* ghost_zero_next = nullptr;  // cleared by the rerun launch (swh_ghost)
  swh::HostBuf hstage;
};

struct swh_gspace {
  swh_context* ctx = nullptr;
  hipStream_t stream = nullptr;
  int64_t n = 0;
  swh::DevBuf aos;
  swh::GLayout layout{};
  swh::DevBuf pos;     // double4 x,y,z,eps
  swh::DevBuf hinv;    // double 1/eps
  swh::DevBuf mass;    // float  mass (0 for inhibited)
  swh::DevBuf active;  // int8
  swh::DevBuf accel;   // double4 ax, ay, az, pot (accumulated this call)
  swh::DevBuf oagn;    // float old_a_grav_norm (the adaptive MAC's estimate)
  swh::DevBuf mpoles;  // swh_multipole[nleaves] (swh_gspace_make_multipoles)
  bool mpoles_valid = false;
  bool mpoles_given = false;  // swh_gspace_set_multipoles: the tree uses the caller's
  bool any_mpole = false;  // some pair has allow_mpole
  swh::DevBuf leaves, pair_off, pairs;
  int32_t nleaves = 0, npairs = 0;
  int32_t max_leaf = 0;
  swh::DevBuf counter;
  swh::DevBuf m2p_bits;  // u64 per pair: the lanes whose i took the entry's multipole (launch_pp)
  // tree gravity (swh_gspace_set_tree / swh_grav_tree)
  std::vector<swh_gcell> tree;   // host copy of the cell table
  swh::DevBuf cell_act;          // int8 per cell: any active gpart
  swh::DevBuf ftens;             // double[35] per cell: field tensors
  swh::DevBuf m2l_off, m2l_src;  // CSR per target cell: int2 {source, symmetric}
  swh::DevBuf l2l_list;          // int2 {cell, parent}, grouped by depth
  std::vector<int32_t> l2l_depth_off;  // l2l_list range of each depth
  swh::DevBuf m2m_list;          // int: split cells, deepest first (the upward M2M pass)
  std::vector<int32_t> m2m_depth_off;  // m2m_list range of each depth
  swh::DevBuf leaf_ids;          // int: the unsplit cells
  swh::DevBuf leaf_of;           // int per gpart: its unsplit cell (-1: none)
  int32_t nleaf_cells = 0;
  int32_t tree_max_leaf = 0;     // largest unsplit cell
  std::vector<int32_t> tree_parent;  // -1 for a root
  // ownership (swh_gspace_set_owned_cells): the walk emits P-P / M-M entries
  // only for owned target cells (empty: every cell is owned)
  std::vector<uint8_t> owned;
  swh::DevBuf owned_d;
  // device walk (swh_grav_tree): the cell table, two frontiers of tasks, the
  // emitted P-P / M-M entries (keys cell << 32 | other, flags) and their
  // sorted copies, per-cell counts
  swh::DevBuf tree_d, wf0, wf1, pp_key, pp_val, pp_key2, pp_val2;
  swh::DevBuf mm_key, mm_val, mm_key2, mm_val2, wsort_tmp, wrec, wcnt, wbase;
  // PM mesh (swh_gspace_pm_mesh): density / potential mesh, its r2c
  // transform and the cached hipFFT plans of side mesh_N
  swh::DevBuf mesh_rho, mesh_frho;
  int32_t mesh_N = 0;
  bool mesh_plans_valid = false;
  void* mesh_fwd = nullptr;
  void* mesh_inv = nullptr;
};

namespace swh {
void mesh_release(swh_gspace* g);  // swh_mesh.hip: mesh buffers and hipFFT plans
}
