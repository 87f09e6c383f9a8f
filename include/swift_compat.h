/*
 * swift_compat.h — repo-owned, field-name-compatible mirrors of the SWIFT
 * structures that the hydro/gravity hot path reads, for SWIFT's DEFAULT
 * configure (SPHENIX SPH, cubic-spline kernel, 3D, gamma=5/3, all subgrid
 * modules *_NONE, multi-softening gravity).
 *
 * Why this file exists: the C adapter (swift_subtask_dev_amd/csrc/swh_swift_adapter.c)
 * implements SWIFT's per-task entry points (runner_doself1_branch_density, ...)
 * with SWIFT's exact signatures. Inside a real SWIFT build that adapter is
 * compiled against SWIFT's own headers ("swift.h"); in this repo (no SWIFT
 * build, no configure) it is compiled against these mirrors, which use the
 * SAME field names, so the adapter source is identical in both settings.
 * The HIP library itself (swifthip.h) never sees any of these types.
 *
 * Only `struct part` and `struct gpart` are byte-for-byte layout mirrors
 * (they are the arrays the GPU reads); `struct cell`, `struct engine`, ...
 * only mirror the field NAMES the hot path uses.
 *
 * Layout sources (reference, /root/reference):
 *   struct part   src/hydro/SPHENIX/hydro_part.h:99-309   (160 B, SWIFT_STRUCT_ALIGN 32)
 *   struct gpart  src/gravity/MultiSoftening/gravity_part.h  (96 B)
 *   sort_entry    src/sort_part.h:32-39
 *   struct cell   src/cell.h:354-500, src/cell_hydro.h:34-174, src/cell_grav.h
 *   struct engine src/engine.h (fields listed in SURVEY.md §8b "Preconditions")
 */
#ifndef SWH_SWIFT_COMPAT_H
#define SWH_SWIFT_COMPAT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef long long integertime_t; /* src/timeline.h:32 */
typedef int8_t timebin_t;        /* src/timeline.h:33 */

#define num_time_bins 56                        /* src/timeline.h:36 */
#define time_bin_inhibited (num_time_bins + 2)  /* src/timeline.h:42 */
#define time_bin_not_created (num_time_bins + 3)

/* ---------------------------------------------------------------------- */
/* struct part: SPHENIX layout, 160 bytes (src/hydro/SPHENIX/hydro_part.h)  */
/* ---------------------------------------------------------------------- */
struct part {
  long long id;        /* @0   */
  void *gpart;         /* @8   */
  double x[3];         /* @16  */
  float v[3];          /* @40  */
  float a_hydro[3];    /* @52  */
  float mass;          /* @64  */
  float h;             /* @68  */
  float u;             /* @72  */
  float u_dt;          /* @76  */
  float rho;           /* @80  */
  struct {
    float div_v;               /* @84  */
    float div_v_dt;            /* @88  */
    float div_v_previous_step; /* @92  */
    float alpha;               /* @96  */
    float v_sig;               /* @100 */
  } viscosity;
  struct {
    float laplace_u; /* @104 */
    float alpha;     /* @108 */
  } diffusion;
  union {
    struct {
      float wcount;    /* @112 */
      float wcount_dh; /* @116 */
      float rho_dh;    /* @120 */
      float rot_v[3];  /* @124 */
    } density;
    struct {
      float f;                  /* @112 */
      float pressure;           /* @116 */
      float soundspeed;         /* @120 */
      float h_dt;               /* @124 */
      float balsara;            /* @128 */
      float alpha_visc_max_ngb; /* @132 */
    } force;
  };
  /* mhd/chemistry/cooling/feedback/BH/sink/pressure-floor/rt part data are
   * empty structs in the default configure; rt_timestepping_data is one
   * timebin_t (src/rt_struct.h:53-61). */
  timebin_t rt_time_bin; /* @136 */
  timebin_t time_bin;    /* @137 */
  struct {
    timebin_t wakeup;           /* @138 */
    timebin_t min_ngb_time_bin; /* @139 */
    char to_be_synchronized;    /* @140 */
  } limiter_data;              /* src/timestep_limiter_struct.h:36-46 */
} __attribute__((aligned(32)));

/* ---------------------------------------------------------------------- */
/* struct gpart: multi-softening layout, 96 bytes                          */
/* ---------------------------------------------------------------------- */
struct gpart {
  long long id_or_neg_offset; /* @0  */
  double x[3];                /* @8  */
  float v_full[3];            /* @32 */
  float a_grav[3];            /* @44 */
  float a_grav_mesh[3];       /* @56 */
  float potential;            /* @68 */
  float potential_mesh;       /* @72 */
  float mass;                 /* @76 */
  float old_a_grav_norm;      /* @80 */
  float epsilon;              /* @84 */
  timebin_t time_bin;         /* @88 */
  int8_t type;                /* @89  enum part_type is __attribute__((packed)) */
} __attribute__((aligned(32)));

/* struct xpart (src/hydro/SPHENIX/hydro_part.h:50-90): the fields the drift
 * reads (v_full, a_grav) and keeps (x_diff, x_diff_sort); the splitting /
 * cooling / tracer / star-formation / feedback / MHD members that follow are
 * not read (padding here; compiled against SWIFT the adapter takes
 * offsetof of the real struct). 96 B as SURVEY's probe. */
struct xpart {
  float x_diff[3];      /* @0  */
  float x_diff_sort[3]; /* @12 */
  float v_full[3];      /* @24 */
  float a_grav[3];      /* @36 */
  float u_full;         /* @48 */
  char other_xpart_data_[44];
} __attribute__((aligned(32)));

/* src/sort_part.h:32-39 */
struct sort_entry {
  float d;
  int i;
};

/* ---------------------------------------------------------------------- */
/* Engine-side scalars read by the hot path                                */
/* ---------------------------------------------------------------------- */
struct cosmology {
  double a, H, a2_inv;
  double a_factor_sound_speed;
  double a_factor_Balsara_eps;
};

struct viscosity_global_data {
  float alpha, alpha_max, alpha_min, length;
};
struct diffusion_global_data {
  float alpha, beta, alpha_max, alpha_min;
};

struct hydro_props {
  float eta_neighbours;
  float h_tolerance;
  float h_max;
  float h_min;
  int max_smoothing_iterations;
  int use_mass_weighted_num_ngb;
  struct viscosity_global_data viscosity;
  struct diffusion_global_data diffusion;
};

struct cell;
struct space {
  int periodic;
  double dim[3];
  /* the top-level grid (src/space.h): runner_do_grav_long_range's loop */
  struct cell *cells_top;
  int *cells_with_particles_top;
  int nr_cells_with_particles;
};

struct pm_mesh {
  int periodic;
  double dim[3];
  float r_s_inv;
  double r_cut_min;
  double r_cut_max;
};

/* src/multipole_struct.h:36-220 at SELF_GRAVITY_MULTIPOLE_ORDER 4 (the
 * adapter reads the fields by name; compiled against SWIFT's headers it
 * uses SWIFT's own layout) */
struct grav_tensor {
  float F_000;
  float F_100, F_010, F_001;
  float F_200, F_020, F_002, F_110, F_101, F_011;
  float F_300, F_030, F_003, F_210, F_201, F_120, F_021, F_102, F_012, F_111;
  float F_400, F_040, F_004, F_310, F_301, F_130, F_031, F_103, F_013, F_220, F_202, F_022,
      F_211, F_121, F_112;
  int interacted;
};

struct multipole {
  float vel[3];
  float max_delta_vel[3];
  float min_delta_vel[3];
  float max_softening;
  float min_old_a_grav_norm;
  float power[5];
  float M_000;
  float M_200, M_020, M_002, M_110, M_101, M_011;
  float M_300, M_030, M_003, M_210, M_201, M_120, M_021, M_102, M_012, M_111;
  float M_400, M_040, M_004, M_310, M_301, M_130, M_031, M_103, M_013, M_220, M_202, M_022,
      M_211, M_121, M_112;
};

struct gravity_tensors {
  struct grav_tensor pot;
  struct multipole m_pole;
  double CoM[3];
  double CoM_rebuild[3];
  double r_max;
  double r_max_rebuild;
};

/* src/gravity_properties.h: the M2P acceptance fields */
struct gravity_props {
  int use_advanced_MAC;
  int use_adaptive_tolerance;
  int use_gadget_tolerance;
  float adaptive_tolerance;
  double theta_crit;
  int use_tree_below_softening;
  int consider_truncation_in_MAC;
};

struct engine {
  struct space *s;
  const struct cosmology *cosmology;
  const struct hydro_props *hydro_properties;
  struct pm_mesh *mesh;
  const struct gravity_props *gravity_properties;
  timebin_t max_active_bin;
  integertime_t ti_current;
  double time_base;
  int policy;
  int nodeID;
};

struct runner {
  struct engine *e;
  int id;
};

/* ---------------------------------------------------------------------- */
/* struct cell: the fields of struct cell / cell_hydro / cell_grav used by  */
/* the loops (names as in src/cell.h, src/cell_hydro.h, src/cell_grav.h)    */
/* ---------------------------------------------------------------------- */
struct cell {
  double loc[3];
  double width[3];
  float dmin;
  int split;
  int nodeID;
  struct cell *progeny[8];
  struct cell *parent;
  struct {
    struct part *parts;
    struct xpart *xparts;
    struct sort_entry *sort[13]; /* one list per sid, count+1 entries */
    int count;
    float h_max, h_max_old, h_max_active;
    float dx_max_part, dx_max_sort, dx_max_sort_old, dx_max_part_old;
    uint16_t sorted;
    integertime_t ti_end_min;
    integertime_t ti_old_part;
  } hydro;
  struct {
    struct gpart *parts;
    int count;
    struct gravity_tensors *multipole;
    integertime_t ti_end_min;
    integertime_t ti_old_part;
    integertime_t ti_old_multipole;
  } grav;
};

/* src/cell.h:1176 (storage differs: SWIFT packs the 13 lists in one
 * meta-array; the accessor contract is the same). */
static inline struct sort_entry *cell_get_hydro_sorts(const struct cell *c,
                                                      const int sid) {
  return c->hydro.sort[sid];
}

#ifdef __cplusplus
}
#endif

#endif /* SWH_SWIFT_COMPAT_H */
