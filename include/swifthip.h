/*
 * swifthip.h — C ABI of libswifthip: an MI355X (gfx950, CDNA4) HIP
 * implementation of SWIFT's SPH neighbour loops (density, gradient, force,
 * ghost h-iteration) and leaf-leaf P2P gravity.
 *
 * Plain C: pointers, sizes and POD structs only; no SWIFT, HIP or torch types
 * in any signature. The SWIFT-signature entry points (runner_doself1_branch_
 * density(struct runner*, struct cell*) ...) live in the thin C adapter
 * (swifthip_swift.h) that marshals SWIFT cells into the views below.
 *
 * Two families of entry points:
 *
 *  (1) Per-task (drop-in, synchronous): one call = one SWIFT task on host
 *      struct part / struct gpart arrays, results written back in place
 *      before return. Replaces the bodies of
 *        DOSELF1_BRANCH / DOPAIR1_BRANCH  src/runner_doiact_functions_hydro.h:2271,1331
 *        DOSELF2_BRANCH / DOPAIR2_BRANCH  src/runner_doiact_functions_hydro.h:2486,1972
 *        DOSELF_SUBSET_BRANCH / DOPAIR_SUBSET_BRANCH  :1048, :884
 *        runner_doself_grav_pp / runner_dopair_grav_pp  src/runner_doiact_grav.c:1788,1202
 *
 *  (2) Batch (performance): a device-resident particle set (swh_space) on
 *      which whole loops run as one launch each, replacing every density /
 *      gradient / force task of a step plus the ghost and extra ghost
 *      (src/runner_ghost.c:1085, :992) and runner_do_end_hydro_force
 *      (src/runner_others.c:618). The interaction set is exactly that of the
 *      task graph: every active i meets every j with r < H_i (density,
 *      gradient) or r < max(H_i, H_j) (force), nearest periodic image.
 *
 * Errors: every function returns swh_status; nothing aborts. The SWIFT
 * adapter maps non-zero codes to SWIFT's error() exactly where the reference
 * calls error() ("Interacting unsorted cells.", ...).
 *
 * Precision: interactions and per-particle updates evaluated in fp64 (the
 * default) or fp32 (SWH_PRECISION_F32, the reference's own precision);
 * storage stays at struct part precision (float fields, double positions).
 */
#ifndef SWIFTHIP_H
#define SWIFTHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWH_ABI_VERSION 11

#if defined(__GNUC__)
#define SWH_API __attribute__((visibility("default")))
#else
#define SWH_API
#endif

typedef enum swh_status {
  SWH_OK = 0,
  SWH_ERR_ARG = 1,           /* invalid argument / shape */
  SWH_ERR_HIP = 2,           /* HIP runtime error (see swh_last_error) */
  SWH_ERR_UNSORTED = 3,      /* "Interacting unsorted cells." */
  SWH_ERR_CELL_SMALL = 4,    /* "Cell smaller than smoothing length" */
  SWH_ERR_NOT_CONVERGED = 5, /* "Smoothing length failed to converge" */
  SWH_ERR_NO_DEVICE = 6,     /* no usable gfx950 device */
  SWH_ERR_OOM = 7,           /* device allocation failed */
  SWH_ERR_STATE = 8,         /* call out of order (e.g. loop before rebuild) */
  SWH_BUSY = 9               /* swh_*_query: queued work still running (not an error) */
} swh_status;

typedef enum swh_precision { SWH_PRECISION_F64 = 0, SWH_PRECISION_F32 = 1 } swh_precision;

/* ------------------------------------------------------------------ */
/* Particle layout descriptors: byte offsets inside the caller's AoS   */
/* record, so the library never hard-codes struct part (its layout is  */
/* configure-dependent in SWIFT). -1 = field absent.                   */
/* ------------------------------------------------------------------ */
typedef struct swh_part_layout {
  int32_t stride; /* sizeof(struct part) */
  int32_t off_id;                                   /* long long */
  int32_t off_x;                                    /* double[3] */
  int32_t off_v, off_a_hydro;                       /* float[3]  */
  int32_t off_mass, off_h, off_u, off_u_dt, off_rho;
  int32_t off_div_v, off_div_v_dt, off_div_v_previous_step, off_visc_alpha, off_v_sig;
  int32_t off_laplace_u, off_diff_alpha;
  /* density union member */
  int32_t off_wcount, off_wcount_dh, off_rho_dh, off_rot_v; /* rot_v float[3] */
  /* force union member */
  int32_t off_f, off_pressure, off_soundspeed, off_h_dt, off_balsara, off_alpha_visc_max_ngb;
  int32_t off_time_bin;         /* int8 */
  int32_t off_min_ngb_time_bin; /* int8 */
  int32_t off_gpart;            /* struct gpart* (drift: gravity kick if non-NULL), -1: none */
} swh_part_layout;

/* struct xpart fields the drift reads (src/hydro/SPHENIX/hydro_part.h:50-90). */
typedef struct swh_xpart_layout {
  int32_t stride;     /* sizeof(struct xpart) */
  int32_t off_v_full; /* float[3] */
  int32_t off_a_grav; /* float[3] */
} swh_xpart_layout;

typedef struct swh_gpart_layout {
  int32_t stride; /* sizeof(struct gpart) */
  int32_t off_x;          /* double[3] */
  int32_t off_a_grav;     /* float[3]  */
  int32_t off_potential;  /* float     */
  int32_t off_mass;       /* float     */
  int32_t off_epsilon;    /* float     */
  int32_t off_time_bin;   /* int8      */
  int32_t off_old_a_grav_norm; /* float (the adaptive MAC's acceleration estimate) */
} swh_gpart_layout;

/* Layouts of SWIFT's default configure (SPHENIX part: 160 B; multi-softening
 * gpart: 96 B). See include/swift_compat.h for the field map. */
SWH_API void swh_part_layout_sphenix(swh_part_layout *out);
SWH_API void swh_gpart_layout_multisoftening(swh_gpart_layout *out);

/* ------------------------------------------------------------------ */
/* Engine scalars the hydro path reads (struct engine / cosmology /    */
/* hydro_props fields, SURVEY.md 8b "Preconditions").                  */
/* ------------------------------------------------------------------ */
typedef struct swh_hydro_params {
  double a, H, a2_inv, a_factor_sound_speed, a_factor_Balsara_eps; /* cosmology */
  double time_base;                                                /* engine    */
  float eta_neighbours, h_tolerance, h_max, h_min;                 /* hydro_props */
  int32_t max_smoothing_iterations;
  int32_t use_mass_weighted_num_ngb;
  float visc_alpha, visc_alpha_max, visc_alpha_min, visc_length;
  float diff_alpha, diff_beta, diff_alpha_max, diff_alpha_min;
  int32_t max_active_bin; /* e->max_active_bin */
  int32_t periodic;       /* e->s->periodic    */
  double dim[3];          /* e->s->dim         */
  /* dt_alpha of the extra ghost per time bin (SWH_NUM_TIME_BINS + 1 entries,
   * nullable). NULL: the non-cosmological get_timestep(bin, time_base). With
   * cosmology the engine passes, for every bin b, the physical time of the
   * bin's current step, cosmology_get_delta_time(cosmo, ti_begin,
   * ti_begin + get_integer_timestep(b)) with ti_begin =
   * get_integer_time_begin(ti_current - 1, b) (src/runner_ghost.c:1038-1046). */
  const double *dt_alpha_bins;
} swh_hydro_params;
#define SWH_NUM_TIME_BINS 56

typedef struct swh_grav_params {
  int32_t periodic;  /* e->mesh->periodic  */
  float dim[3];      /* e->mesh->dim       */
  float r_s_inv;     /* e->mesh->r_s_inv   */
  double r_cut_min;  /* e->mesh->r_cut_min */
  int32_t max_active_bin;
  /* M2P acceptance (gravity_M2P_accept, src/multipole_accept.h:290-373):
   * e->gravity_properties fields */
  float theta_crit;
  float adaptive_tolerance;
  int32_t use_advanced_MAC;
  int32_t use_gadget_tolerance;
  int32_t use_tree_below_softening;
  int32_t consider_truncation_in_MAC;
  double r_cut_max;  /* e->mesh->r_cut_max: the tree walk skips pairs beyond it */
} swh_grav_params;

/* A cell's multipole expansion about its centre of mass, order 4 (SWIFT's
 * default SELF_GRAVITY_MULTIPOLE_ORDER): the fields of struct gravity_tensors
 * / struct multipole (src/multipole_struct.h:110-220) that M2P reads.
 * M[] holds the 35 terms M_abc, a+b+c <= 4, in struct multipole's member
 * order with the (zero) dipole at 1..3:
 *   0 M_000 | 1 M_100 2 M_010 3 M_001 |
 *   4 M_200 5 M_020 6 M_002 7 M_110 8 M_101 9 M_011 |
 *   10 M_300 11 M_030 12 M_003 13 M_210 14 M_201 15 M_120 16 M_021 17 M_102
 *   18 M_012 19 M_111 |
 *   20 M_400 21 M_040 22 M_004 23 M_310 24 M_301 25 M_130 26 M_031 27 M_103
 *   28 M_013 29 M_220 30 M_202 31 M_022 32 M_211 33 M_121 34 M_112 */
#define SWH_MPOLE_TERMS 35
typedef struct swh_multipole {
  double CoM[3];
  double r_max;
  float M[SWH_MPOLE_TERMS];
  float power[5];           /* multipole power per order */
  float max_softening;
  float min_old_a_grav_norm;
} swh_multipole;

/* ------------------------------------------------------------------ */
/* Context: one per (process, device). Thread-safe: per-task calls     */
/* from different host threads use different internal streams.        */
/* ------------------------------------------------------------------ */
typedef struct swh_context swh_context;

SWH_API swh_status swh_init(swh_context **ctx, int device);
SWH_API swh_status swh_finalize(swh_context *ctx);
SWH_API swh_status swh_set_precision(swh_context *ctx, swh_precision p);
SWH_API const char *swh_status_string(swh_status s);
/* Last error text of the calling thread (empty string if none). */
SWH_API const char *swh_last_error(void);
SWH_API int swh_abi_version(void);
/* The SPH kernel this library was built for ("cubic-spline" or
 * "wendland-c2"): SWIFT selects it at configure time (--with-kernel,
 * configure.ac:2107-2137, kernel_hydro.h:45-147); one library per kernel
 * (libswifthip.so / libswifthip_wc2.so), the same ABI. (ABI v9) */
SWH_API const char *swh_kernel_name(void);

/* ================================================================== */
/* (1) Per-task entry points                                          */
/* ================================================================== */
typedef struct swh_cell_view {
  void *parts;     /* host pointer to `count` AoS records (struct part) */
  int32_t count;
  int32_t active;  /* cell_is_active_hydro(c, e) */
  double loc[3];
  double width[3];
} swh_cell_view;

/* Density / gradient loops (r < H_i): DOSELF1 / DOPAIR1 semantics. In a pair,
 * active particles of BOTH cells are updated. `shift` is SWIFT's periodic
 * shift: particle i of ci interacts as x_i - shift (space_getsid.h:46-82). */
SWH_API swh_status swh_doself_density(swh_context *ctx, const swh_cell_view *c,
                              const swh_part_layout *L, const swh_hydro_params *P);
SWH_API swh_status swh_dopair_density(swh_context *ctx, const swh_cell_view *ci,
                              const swh_cell_view *cj, const double shift[3],
                              const swh_part_layout *L, const swh_hydro_params *P);
SWH_API swh_status swh_doself_gradient(swh_context *ctx, const swh_cell_view *c,
                               const swh_part_layout *L, const swh_hydro_params *P);
SWH_API swh_status swh_dopair_gradient(swh_context *ctx, const swh_cell_view *ci,
                               const swh_cell_view *cj, const double shift[3],
                               const swh_part_layout *L, const swh_hydro_params *P);
/* Force loop (r < max(H_i, H_j), + time-bin limiter): DOSELF2 / DOPAIR2. */
SWH_API swh_status swh_doself_force(swh_context *ctx, const swh_cell_view *c,
                            const swh_part_layout *L, const swh_hydro_params *P);
SWH_API swh_status swh_dopair_force(swh_context *ctx, const swh_cell_view *ci,
                            const swh_cell_view *cj, const double shift[3],
                            const swh_part_layout *L, const swh_hydro_params *P);
/* Subset density (ghost reruns): only parts_i[ind[0..count)] of ci are
 * updated, against all of ci (self) or cj (pair). DOSELF_SUBSET /
 * DOPAIR_SUBSET semantics. `parts_i` may differ from ci->parts (SWIFT passes
 * the ghost's leaf array). */
SWH_API swh_status swh_doself_subset_density(swh_context *ctx, const swh_cell_view *ci,
                                     void *parts_i, const int32_t *ind, int32_t count,
                                     const swh_part_layout *L, const swh_hydro_params *P);
SWH_API swh_status swh_dopair_subset_density(swh_context *ctx, const swh_cell_view *ci,
                                     void *parts_i, const int32_t *ind, int32_t count,
                                     const swh_cell_view *cj, const double shift[3],
                                     const swh_part_layout *L, const swh_hydro_params *P);

/* P2P gravity on host gpart arrays. */
typedef struct swh_gcell_view {
  void *gparts;
  int32_t count;
  int32_t active;
  double loc[3];
  double width[3];
  double CoM[3];   /* multipole->CoM   */
  double r_max;    /* multipole->r_max */
  const swh_multipole *multipole; /* the cell's expansion (needed with allow_mpole) */
} swh_gcell_view;

SWH_API swh_status swh_grav_self_pp(swh_context *ctx, const swh_gcell_view *c,
                            const swh_gpart_layout *L, const swh_grav_params *G);
/* runner_dopair_grav_pp: with allow_mpole, every active particle of one
 * cell that passes gravity_M2P_accept against the other cell's multipole
 * (evaluated in float exactly as gravity_cache_populate does) takes the M2P
 * route (runner_dopair_grav_pm_full / _truncated) instead of P2P. */
SWH_API swh_status swh_grav_pair_pp(swh_context *ctx, const swh_gcell_view *ci,
                            const swh_gcell_view *cj, int symmetric, int allow_mpole,
                            const swh_gpart_layout *L, const swh_grav_params *G);

/* ================================================================== */
/* (2) Batch, device-resident                                         */
/* ================================================================== */
typedef struct swh_space swh_space;

SWH_API swh_status swh_space_create(swh_context *ctx, swh_space **s);
SWH_API swh_status swh_space_destroy(swh_space *s);
/* Bind a HIP stream (hipStream_t passed as void*; NULL = the space's own). */
SWH_API swh_status swh_space_set_stream(swh_space *s, void *stream);
/* Upload from a host AoS array (struct part records) or from a DEVICE AoS
 * array (`parts` already in HBM, e.g. a torch uint8 tensor). */
SWH_API swh_status swh_space_upload_parts(swh_space *s, const void *parts, int64_t count,
                                  const swh_part_layout *L, int on_device);
/* Fields written back: SWH_FIELDS_DENSITY after density+ghost, SWH_FIELDS_FORCE
 * after force (the union member of struct part that is live), SWH_FIELDS_DRIFT
 * after a drift (x, v, u, h, rho, pressure, soundspeed, v_sig), or ALL. */
#define SWH_FIELDS_DENSITY 1
#define SWH_FIELDS_GRADIENT 2
#define SWH_FIELDS_FORCE 4
#define SWH_FIELDS_DRIFT 8
#define SWH_FIELDS_ALL 15
SWH_API swh_status swh_space_download_parts(swh_space *s, void *parts, const swh_part_layout *L,
                                    int fields, int on_device);
SWH_API int64_t swh_space_count(const swh_space *s);

/* Bin the particles into the device neighbour grid (cell width >=
 * `min_cell_width`, or derived from max H when <= 0). Equivalent of
 * space_rebuild + runner_do_hydro_sort for this path. */
SWH_API swh_status swh_space_rebuild(swh_space *s, const swh_hydro_params *P,
                             double min_cell_width);

/* Loops over all active particles. n_interactions (optional) receives the
 * number of directed interactions evaluated (r < H_i, resp. max(H_i,H_j)). */
SWH_API swh_status swh_space_init_parts(swh_space *s, const swh_hydro_params *P);
/* hydro_reset_acceleration + timestep_limiter_prepare_force on active parts
 * (what the extra ghost does before the force loop). */
SWH_API swh_status swh_space_reset_acceleration(swh_space *s, const swh_hydro_params *P);
SWH_API swh_status swh_density_loop(swh_space *s, const swh_hydro_params *P, int64_t *n_interactions);
SWH_API swh_status swh_ghost(swh_space *s, const swh_hydro_params *P, int32_t *iterations,
                     int64_t *n_unconverged);
SWH_API swh_status swh_gradient_loop(swh_space *s, const swh_hydro_params *P, int64_t *n_interactions);
SWH_API swh_status swh_extra_ghost(swh_space *s, const swh_hydro_params *P);
SWH_API swh_status swh_force_loop(swh_space *s, const swh_hydro_params *P, int64_t *n_interactions);
SWH_API swh_status swh_end_force(swh_space *s, const swh_hydro_params *P);
/* Multi-GPU (one process per GPU). Caller indices >= n_owned are
 * foreign: read-only halo copies of particles another rank owns (SWIFT's
 * foreign cells). They are neighbours of every loop and are never updated.
 * Default after an upload: every particle owned. */
SWH_API swh_status swh_space_set_owned(swh_space *s, int64_t n_owned);
/* Halo refresh between loop phases. A halo record is 8 floats: h, rho,
 * pressure, soundspeed, f (grad-h term), balsara, alpha_visc, alpha_diff.
 * pack writes the records of the particles with caller indices idx[0..n)
 * (DEVICE arrays) to out (device, n * 8 floats); unpack writes the `fields`
 * groups of the records in `in` to the particles idx[0..n). Both are ordered
 * on the space's stream. */
#define SWH_HALO_RECORD_FLOATS 8
#define SWH_HALO_H 1
#define SWH_HALO_RHO 2
#define SWH_HALO_PC 4         /* pressure, soundspeed */
#define SWH_HALO_F_BALSARA 8  /* f, balsara */
#define SWH_HALO_ALPHAS 16    /* alpha_visc, alpha_diff */
#define SWH_HALO_ALL 31
SWH_API swh_status swh_space_pack_halo(swh_space *s, const int32_t *idx, int32_t n, float *out);
SWH_API swh_status swh_space_unpack_halo(swh_space *s, const int32_t *idx, int32_t n,
                                         const float *in, int fields);
/* Drift (runner_do_drift_part over every cell, src/runner_drift.c:41 ->
 * drift_part, src/drift.h:143-232, with SPHENIX hydro_predict_extra,
 * src/hydro/SPHENIX/hydro.h:1012-1066; entropy and pressure floors NONE):
 * x += v_full dt_drift; v += a_hydro dt_kick_hydro (+ a_grav dt_kick_grav for
 * particles with a gpart); u += u_dt dt_therm; h, rho by exp(+-w1); u floored
 * at min_u; P, c from the EOS; v_sig >= 2c. Every non-inhibited particle,
 * owned or foreign, is drifted. The particles stay in their cells: the loops
 * widen their reach by the largest displacement since the last rebuild
 * (swh_space_info.dx_max, SWIFT's dx_max_part), so they stay exact; rebuild
 * when it grows too large (SWIFT: space_maxreldx of the cell size). The
 * xparts (v_full, a_grav) are uploaded in caller order, once per step. */
typedef struct swh_drift_params {
  double dt_drift, dt_kick_hydro, dt_kick_grav, dt_therm;
  float min_u; /* hydro_props->minimal_internal_energy / cosmo->a_factor_internal_energy */
} swh_drift_params;
SWH_API swh_status swh_space_upload_xparts(swh_space *s, const void *xparts, int64_t count,
                                           const swh_xpart_layout *XL, int on_device);
SWH_API swh_status swh_space_drift(swh_space *s, const swh_drift_params *D,
                                   const swh_hydro_params *P);

/* Wait for all queued work on the space's stream. */
SWH_API swh_status swh_space_sync(swh_space *s);
/* Without waiting: SWH_OK when all queued work on the space's stream has
 * finished, SWH_BUSY while it runs. The batch calls only enqueue (with NULL
 * counters nothing waits), so a scheduler can start a phase as one task and
 * let its CPU runners take other tasks, polling this where SWIFT's dependent
 * task (e.g. the ghost after the density loop, engine_maketasks.c:2313-2316
 * ghost_in/ghost_out) would become ready. */
SWH_API swh_status swh_space_query(swh_space *s);

/* Kernel-tuning knobs of the batch loops (bench/diagnostics). */
#define SWH_DEFAULT_LIST_SKIN 0.01f
typedef struct swh_tuning {
  int32_t cell_factor;  /* neighbour-grid cells per H_max (1..4) */
  int32_t loop_variant; /* 0 or 7: pair lists -- the density loop builds the step's lists
                           (r < max(R_i, R_j), R = gamma h (1 + list_skin)), the density /
                           gradient / force loops walk them */
  int32_t group_size;   /* list-build i-group size: 0 (default) or 16 */
  float cell_scale;     /* if > 0: cells per H_max as a real number (overrides cell_factor) */
  int32_t diag_mode;    /* 0; profiling only (results invalid): 1 = list build stages
                           candidates only, 2 = build without list writes, 4 = fixed-j
                           gathers; 7 (results valid) = as list_keep */
  int32_t list_capacity; /* list entries per particle (0 = 128); more hits: a wave-per-
                            particle search */
  float list_skin;       /* relative slack of the list reach over gamma h (SWH_DEFAULT_LIST_SKIN
                            = 0.01 when the space is created: nearly all of the ghost's h
                            iterations stay within the lists' reach, so the ghost does not
                            rebuild them, and the gradient / force loops search the few
                            particles that grew past it; 0: exact lists, rebuilt by the
                            ghost whenever many H outgrow their reach) */
  int32_t list_keep;     /* 1: keep the lists across loops and drifts while they cover every
                            pair, as SWIFT keeps its sorts until dx_max_sort exceeds
                            space_maxreldx (space.h:66): after a drift the device compares
                            each H + 2 D (D = largest displacement since the build) with
                            the build reach gamma h (1 + list_skin) and rebuilds only when
                            some particle exceeds it, without a host round trip.
                            0 (default): every density loop builds the lists. */
} swh_tuning;
SWH_API swh_status swh_space_set_tuning(swh_space *s, const swh_tuning *t);

/* Neighbour-grid diagnostics of the last rebuild. */
typedef struct swh_space_info {
  int32_t cdim[3];  /* grid cells per dimension */
  int32_t ncell;
  int32_t ngroups;  /* i-groups of the tile loops (octree leaves, <= 64 parts) */
  int32_t reserved;
  double cell_width[3];
  double h_max;     /* max gamma*h at rebuild */
  int64_t loop_stats[4]; /* last counted search (tile loop or list build): candidates loaded,
                            staged, test wave steps, list-flush lane steps */
  int64_t list_entries;  /* last counted list build: total entries */
  int32_t list_overflow; /* last counted list build: particles over list_capacity */
  int32_t list_valid;    /* the step's pair lists are current */
  double dx_max;         /* largest displacement since the last rebuild (drift) */
  int64_t list_builds;   /* pair-list builds run on the device since the space was created */
} swh_space_info;
/* Note: get_info WAITS for the space's stream (it reads the device's
 * list-build counter, info->list_builds); in the enqueue-then-poll model
 * (swh_space_query) call it only after the queued phases are done. */
SWH_API swh_status swh_space_get_info(const swh_space *s, swh_space_info *info);

/* Batch P2P gravity over leaf cells of a device-resident gpart set. Leaves
 * are contiguous [start, start+count) ranges; for each i-leaf, the CSR list
 * pairs[pair_offset[i] .. pair_offset[i+1]) names the source leaves
 * (including i itself for the self term) with a per-pair truncation flag
 * (runner_doself/dopair_grav_pp's full-vs-truncated choice). */
typedef struct swh_gspace swh_gspace;
typedef struct swh_leaf {
  int32_t start;
  int32_t count;
} swh_leaf;
typedef struct swh_leaf_pair {
  int32_t j;           /* source leaf index */
  int32_t truncated;   /* 1: long-range truncated kernel */
  int32_t allow_mpole; /* 1: i-particles passing the MAC take leaf j's multipole (M2P) */
} swh_leaf_pair;
SWH_API swh_status swh_gspace_create(swh_context *ctx, swh_gspace **g);
SWH_API swh_status swh_gspace_destroy(swh_gspace *g);
SWH_API swh_status swh_gspace_upload(swh_gspace *g, const void *gparts, int64_t count,
                             const swh_gpart_layout *L, int on_device);
SWH_API swh_status swh_gspace_set_leaves(swh_gspace *g, const swh_leaf *leaves, int32_t nleaves,
                                 const int32_t *pair_offset, const swh_leaf_pair *pairs,
                                 int32_t npairs);
/* Leaf multipoles (gravity_P2M + gravity_multipole_compute_power,
 * src/multipole.h:878-1266) of every leaf, on the device; needed before a
 * batch with allow_mpole pairs. `out` (nullable): a host copy. */
SWH_API swh_status swh_gspace_make_multipoles(swh_gspace *g, swh_multipole *out);
/* P2P (+ M2P on allow_mpole pairs) of every leaf's active particles.
 * n_interactions: P2P pair interactions; n_m2p (nullable): M2P evaluations. */
SWH_API swh_status swh_grav_pp_batch(swh_gspace *g, const swh_grav_params *G,
                                     int64_t *n_interactions, int64_t *n_m2p);
SWH_API swh_status swh_gspace_download(swh_gspace *g, void *gparts, const swh_gpart_layout *L,
                               int on_device);

/* Tree gravity (SURVEY 8 a15 recursion, 8f row 3 M2L): the cell tree of the
 * uploaded gparts, cells[c] = {start, count} ranges nested as SWIFT's
 * (a split cell's progeny partition its range). swh_grav_tree then runs a
 * step's gravity tasks on it:
 *   runner_doself_recursive_grav on every cell of self_cells and
 *   runner_dopair_recursive_grav on every pair of pair_cells (2 per pair)
 *   (src/runner_doiact_grav.c:2208-2431: the r_cut_max skip, P-P of cells of
 *   <= 1 particle (runner_dopair_grav_pp_no_cache), M-M when
 *   gravity_M2L_accept_symmetric passes, leaf-leaf P-P with M2P
 *   (runner_dopair_grav_pp, allow_mpole), else split the larger cell),
 * then the down pass (runner_do_grav_down, 65-164: L2L from each cell's
 * parent, L2P at the leaves). Multipoles as space_split builds them
 * (src/space_split.c:340-440): gravity_P2M at the leaves, then up the tree
 * the mass-weighted CoM of the progeny, gravity_M2M of every child to it
 * (multipole.h:1278), r_max = min(max_k (r_max_k + |CoM - CoM_k|), the
 * CoM's distance to the farthest cell corner), max softening / min old |a|
 * over the progeny, gravity_multipole_compute_power. Everything runs on the
 * device (SWH_HOST_WALK=1: the walk on the host, SWH_HOST_THREADS threads).
 * Results accumulate like swh_grav_pp_batch's (swh_gspace_download adds
 * them). */
typedef struct swh_gcell {
  int32_t start, count; /* gpart range */
  int32_t split;        /* 1: progeny[] partition the range */
  int32_t progeny[8];   /* child cell indices (-1: none) */
  int32_t reserved;
  double loc[3];        /* c->loc: lower corner */
  double width[3];      /* c->width */
} swh_gcell;
typedef struct swh_grav_tree_stats {
  int64_t n_pp;         /* P2P pair interactions */
  int64_t n_m2p;        /* M2P evaluations */
  int64_t n_m2l;        /* M2L applications (a symmetric M-M counts 2) */
  int64_t n_pp_tasks;   /* leaf <- cell P-P entries of the walk */
  int64_t n_skipped;    /* cell pairs beyond r_cut_max */
  /* device time of the phases of this call (ms, HIP events on the gspace's
   * stream): multipoles (P2M + M2M), walk, P2P, M2P, M2L + L2L + L2P */
  float ms_multipoles, ms_walk, ms_p2p, ms_m2p, ms_down;
  int32_t reserved;
  int64_t n_pp_truncated; /* of n_pp: pairs of truncated entries (periodic, beyond r_cut_min:
                             runner_dopair/doself_grav_pp_truncated) -- ABI v10 */
} swh_grav_tree_stats;
SWH_API swh_status swh_gspace_set_tree(swh_gspace *g, const swh_gcell *cells, int32_t ncells);
/* Ownership for a step sharded over ranks (i-cells owned per GPU,
 * every gpart and multipole replicated read-only): owned[c] != 0 for the
 * cells whose gparts this rank computes. swh_grav_tree then runs only the
 * tasks that can reach an owned cell and emits P-P / M-M entries only for
 * owned targets; M-M symmetry and every acceptance decision still use the
 * whole tree, so an owned gpart's result equals the single-domain one
 * bit for bit, and the other gparts receive nothing from the tree (their
 * accumulators are not meaningful on this rank). Ownership is whole
 * subtrees: a cell must be owned exactly when its parent is (root cells
 * choose). owned = NULL: every cell (the default, and after set_tree). */
SWH_API swh_status swh_gspace_set_owned_cells(swh_gspace *g, const uint8_t *owned,
                                              int32_t ncells);
SWH_API swh_status swh_grav_tree(swh_gspace *g, const swh_grav_params *G,
                                 const int32_t *self_cells, int32_t nself,
                                 const int32_t *pair_cells, int32_t npair,
                                 swh_grav_tree_stats *stats);
/* The same tasks with flags: SWH_TREE_NO_DOWN leaves out the down pass, so
 * the field tensors hold each cell's M2L sums (runner_doself/dopair_
 * recursive_grav only accumulate into c->grav.multipole->pot; SWIFT's
 * runner_do_grav_down task pushes them down later: swh_gspace_grav_down). */
#define SWH_TREE_NO_DOWN 1
SWH_API swh_status swh_grav_tree_tasks(swh_gspace *g, const swh_grav_params *G,
                                       const int32_t *self_cells, int32_t nself,
                                       const int32_t *pair_cells, int32_t npair, int32_t flags,
                                       swh_grav_tree_stats *stats);
/* Field tensors of the last swh_grav_tree (35 floats per cell, struct
 * grav_tensor's F order = swh_multipole::M's), after the down pass. */
SWH_API swh_status swh_gspace_field_tensors(swh_gspace *g, float *out);
/* The tree cells' multipoles (after swh_grav_tree, or as given). */
SWH_API swh_status swh_gspace_multipoles(swh_gspace *g, swh_multipole *out);
/* Use the caller's multipoles for the cells of the current tree (SWIFT's
 * c->grav.multipole, drifted by its own tasks) instead of building them from
 * the gparts; valid until the next swh_gspace_set_tree. */
SWH_API swh_status swh_gspace_set_multipoles(swh_gspace *g, const swh_multipole *in);
/* runner_do_grav_down (runner_doiact_grav.c:65-164) over the current tree:
 * fields = each cell's field tensor (35 floats per cell, as
 * swh_gspace_field_tensors); L2L into the progeny depth by depth, L2P into the
 * active gparts of the leaves; swh_gspace_download adds the accelerations and
 * potentials, swh_gspace_field_tensors returns the pushed-down tensors. */
SWH_API swh_status swh_gspace_grav_down(swh_gspace *g, const swh_grav_params *G,
                                        const float *fields);
/* M-M interactions of explicit pairs of the caller's multipoles (ABI v11):
 * SWIFT's M-M tasks outside the recursive walk -- runner_dopair_grav_mm_progenies
 * (src/runner_doiact_grav.c:2067-2093) and runner_do_grav_long_range
 * (2441-2530). pairs[3k], pairs[3k+1], pairs[3k+2] = target, source,
 * symmetric: the target's field tensor (at its CoM) receives the source's
 * M2L, with gravity_M2L_symmetric's softening (the larger max_softening of
 * the two) when symmetric != 0, else gravity_M2L_nonsym's (the source's);
 * a symmetric M-M pair is given as two entries. fields: nmp x 35 floats
 * (struct grav_tensor's F order), overwritten: each target's sums, zero for
 * the multipoles that receive nothing. Thread-safe like the per-task calls. */
SWH_API swh_status swh_grav_m2l_pairs(swh_context *ctx, const swh_grav_params *G,
                                      const swh_multipole *mp, int32_t nmp,
                                      const int32_t *pairs, int32_t npairs, float *fields);
/* gravity_M2L_accept_symmetric (src/multipole_accept.h:78-205) of A and B at
 * squared CoM distance r2, in the reference's float arithmetic -- the MAC the
 * tree walk uses. For cell_can_use_pair_mm's rebuild-time decision
 * (src/cell.c:1420-1460) pass CoM_rebuild / r_max_rebuild. Returns 1 / 0. */
SWH_API int swh_grav_m2l_accept(const swh_grav_params *G, const swh_multipole *A,
                                const swh_multipole *B, double r2);
SWH_API swh_status swh_gspace_sync(swh_gspace *g);
/* Without waiting: SWH_OK when the gspace's stream is idle, SWH_BUSY otherwise. */
SWH_API swh_status swh_gspace_query(swh_gspace *g);

/* PM mesh gravity: pm_mesh_compute_potential's
 * non-distributed path, compute_potential_global (src/mesh_gravity.c:844-1041)
 * without neutrinos, over the uploaded gparts: CIC assignment of the masses
 * (inhibited gparts skipped), r2c FFT, the Green function with the
 * long-range truncation and CIC deconvolution (mesh_apply_Green_function),
 * c2r FFT, then per gpart the CIC potential and the 5-point-stencil
 * accelerations times const_G (mesh_to_gpart_CIC), written into the records'
 * a_grav_mesh[3] / potential_mesh floats (overwritten, as the reference zeroes
 * them first); swh_gspace_download returns them. potential_out (nullable): the
 * N^3 potential mesh (row-major, z fastest), as mesh->potential_global. */
typedef struct swh_pm_params {
  int32_t N;                  /* gravity_props.mesh_size (even, 2 to 1290; odd N refused, see swh_mesh.hip) */
  int32_t off_a_grav_mesh;    /* byte offsets in the gpart record: float[3] */
  int32_t off_potential_mesh; /* float */
  int32_t reserved;
  double box_size;            /* s->dim[0] (cubic periodic box) */
  double r_s;                 /* mesh->r_s = a_smooth * box_size / N */
  double const_G;             /* physical_constants->const_newton_G (used as float) */
} swh_pm_params;
SWH_API swh_status swh_gspace_pm_mesh(swh_gspace *g, const swh_pm_params *M,
                                      double *potential_out);

#ifdef __cplusplus
}
#endif

#endif /* SWIFTHIP_H */
