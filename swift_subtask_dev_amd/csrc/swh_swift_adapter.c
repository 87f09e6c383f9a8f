/*
 * swh_swift_adapter.c — SWIFT-signature per-task entry points on top of
 * libswifthip (see include/swifthip_swift.h).
 *
 * Each function reproduces the control logic of the *_BRANCH function it
 * replaces (early returns, precondition errors, space_getsid's periodic shift
 * and ci/cj swap) and hands the interaction work to the GPU via the
 * layout-independent C ABI (swifthip.h). Plain C, compiled against SWIFT's
 * headers inside SWIFT, against include/swift_compat.h here.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "swifthip.h"
#include "swifthip_swift.h"

#ifndef SWH_ADAPTER_ERROR
static __thread char swhs_err[256];
#define SWH_ADAPTER_ERROR(msg)                         \
  do {                                                 \
    snprintf(swhs_err, sizeof(swhs_err), "%s", (msg)); \
    return;                                            \
  } while (0)
#endif

static swh_context *swhs_ctx = NULL;
static swh_part_layout swhs_layout;
static swh_gpart_layout swhs_glayout;

#if defined(SWH_KERNEL_WENDLAND_C2)
#define kernel_gamma ((float)(1.936492)) /* src/kernel_hydro.h:137 */
#else
#define kernel_gamma ((float)(1.825742)) /* src/kernel_hydro.h:51 */
#endif
#define space_maxreldx 0.1f              /* src/space.h:66 */

/* src/sort_part.h:59-92 */
static const int swhs_runner_flip[27] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0,
                                         0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static const int swhs_sortlistID[27] = {0, 1, 2, 3, 4,  5,  6,  7,  8,  9,  10, 11, 12, 0,
                                        12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};

/* The record layouts as THIS translation unit sees them: compiled against
 * SWIFT's headers inside SWIFT, the offsets follow whatever configure built
 * struct part / struct gpart (debug checks, subgrid fields, ...); the library
 * never assumes a layout of its own. */
void swifthip_swift_part_layout(swh_part_layout *o) {
  o->stride = (int32_t)sizeof(struct part);
  o->off_id = (int32_t)offsetof(struct part, id);
  o->off_x = (int32_t)offsetof(struct part, x);
  o->off_v = (int32_t)offsetof(struct part, v);
  o->off_a_hydro = (int32_t)offsetof(struct part, a_hydro);
  o->off_mass = (int32_t)offsetof(struct part, mass);
  o->off_h = (int32_t)offsetof(struct part, h);
  o->off_u = (int32_t)offsetof(struct part, u);
  o->off_u_dt = (int32_t)offsetof(struct part, u_dt);
  o->off_rho = (int32_t)offsetof(struct part, rho);
  o->off_div_v = (int32_t)offsetof(struct part, viscosity.div_v);
  o->off_div_v_dt = (int32_t)offsetof(struct part, viscosity.div_v_dt);
  o->off_div_v_previous_step = (int32_t)offsetof(struct part, viscosity.div_v_previous_step);
  o->off_visc_alpha = (int32_t)offsetof(struct part, viscosity.alpha);
  o->off_v_sig = (int32_t)offsetof(struct part, viscosity.v_sig);
  o->off_laplace_u = (int32_t)offsetof(struct part, diffusion.laplace_u);
  o->off_diff_alpha = (int32_t)offsetof(struct part, diffusion.alpha);
  o->off_wcount = (int32_t)offsetof(struct part, density.wcount);
  o->off_wcount_dh = (int32_t)offsetof(struct part, density.wcount_dh);
  o->off_rho_dh = (int32_t)offsetof(struct part, density.rho_dh);
  o->off_rot_v = (int32_t)offsetof(struct part, density.rot_v);
  o->off_f = (int32_t)offsetof(struct part, force.f);
  o->off_pressure = (int32_t)offsetof(struct part, force.pressure);
  o->off_soundspeed = (int32_t)offsetof(struct part, force.soundspeed);
  o->off_h_dt = (int32_t)offsetof(struct part, force.h_dt);
  o->off_balsara = (int32_t)offsetof(struct part, force.balsara);
  o->off_alpha_visc_max_ngb = (int32_t)offsetof(struct part, force.alpha_visc_max_ngb);
  o->off_time_bin = (int32_t)offsetof(struct part, time_bin);
  o->off_min_ngb_time_bin = (int32_t)offsetof(struct part, limiter_data.min_ngb_time_bin);
  o->off_gpart = (int32_t)offsetof(struct part, gpart);
}

void swifthip_swift_gpart_layout(swh_gpart_layout *o) {
  o->stride = (int32_t)sizeof(struct gpart);
  o->off_x = (int32_t)offsetof(struct gpart, x);
  o->off_a_grav = (int32_t)offsetof(struct gpart, a_grav);
  o->off_potential = (int32_t)offsetof(struct gpart, potential);
  o->off_mass = (int32_t)offsetof(struct gpart, mass);
  o->off_epsilon = (int32_t)offsetof(struct gpart, epsilon);
  o->off_time_bin = (int32_t)offsetof(struct gpart, time_bin);
  o->off_old_a_grav_norm = (int32_t)offsetof(struct gpart, old_a_grav_norm);
}

static void split_pairs_init(void);

int swifthip_swift_init(int device, int precision) {
  if (swhs_ctx) return 0;
  if (swh_init(&swhs_ctx, device) != SWH_OK) return -1;
  swh_set_precision(swhs_ctx, precision ? SWH_PRECISION_F32 : SWH_PRECISION_F64);
  swifthip_swift_part_layout(&swhs_layout);
  swifthip_swift_gpart_layout(&swhs_glayout);
  split_pairs_init();
  return 0;
}

int swifthip_swift_set_precision(int precision) {
  if (!swhs_ctx) return -1;
  return swh_set_precision(swhs_ctx, precision ? SWH_PRECISION_F32 : SWH_PRECISION_F64) ==
                 SWH_OK
             ? 0
             : -1;
}

/* One persistent gspace and staging buffer per runner thread: the recursive
 * gravity tasks (runner_do{self,pair}_recursive_grav, runner_do_grav_down)
 * reuse its device buffers and stream instead of creating and destroying a
 * gspace per task -- SWIFT runs thousands of these tasks per step. The
 * registry lets swifthip_swift_finalize destroy them all; a thread whose
 * gspace belongs to a finalized context (older generation) makes a new one.
 * Past SWHS_MAX_GSPACES threads a task falls back to a gspace of its own. */
#define SWHS_MAX_GSPACES 1024
static __thread swh_gspace *swhs_tls_gs = NULL;
static __thread unsigned swhs_tls_gen = 0;
static __thread char *swhs_tls_stage = NULL;
static __thread size_t swhs_tls_stage_cap = 0;
static unsigned swhs_ctx_gen = 1;
static pthread_mutex_t swhs_reg_lock = PTHREAD_MUTEX_INITIALIZER;
static swh_gspace *swhs_reg[SWHS_MAX_GSPACES];
static int swhs_nreg = 0;

void swifthip_swift_finalize(void) {
  pthread_mutex_lock(&swhs_reg_lock);
  for (int k = 0; k < swhs_nreg; k++) swh_gspace_destroy(swhs_reg[k]);
  swhs_nreg = 0;
  swhs_ctx_gen++;
  pthread_mutex_unlock(&swhs_reg_lock);
  if (swhs_ctx) swh_finalize(swhs_ctx);
  swhs_ctx = NULL;
}

#ifndef SWH_ADAPTER_ERROR_EXTERNAL
const char *swifthip_swift_last_error(void) { return swhs_err; }
void swifthip_swift_clear_error(void) { swhs_err[0] = 0; }
#endif

static int cell_is_active_hydro(const struct cell *c, const struct engine *e) {
  return c->hydro.ti_end_min == e->ti_current; /* src/active.h:176-190 */
}
static int cell_are_part_drifted(const struct cell *c, const struct engine *e) {
  return c->hydro.ti_old_part == e->ti_current; /* src/active.h */
}
static int cell_is_active_gravity(const struct cell *c, const struct engine *e) {
  return c->grav.ti_end_min == e->ti_current; /* src/active.h:236 */
}

static void params_of(const struct engine *e, swh_hydro_params *P) {
  const struct cosmology *c = e->cosmology;
  const struct hydro_props *hp = e->hydro_properties;
  memset(P, 0, sizeof(*P));
  P->a = c->a;
  P->H = c->H;
  P->a2_inv = c->a2_inv;
  P->a_factor_sound_speed = c->a_factor_sound_speed;
  P->a_factor_Balsara_eps = c->a_factor_Balsara_eps;
  P->time_base = e->time_base;
  if (hp) {
    P->eta_neighbours = hp->eta_neighbours;
    P->h_tolerance = hp->h_tolerance;
    P->h_max = hp->h_max;
    P->h_min = hp->h_min;
    P->max_smoothing_iterations = hp->max_smoothing_iterations;
    P->use_mass_weighted_num_ngb = hp->use_mass_weighted_num_ngb;
    P->visc_alpha = hp->viscosity.alpha;
    P->visc_alpha_max = hp->viscosity.alpha_max;
    P->visc_alpha_min = hp->viscosity.alpha_min;
    P->visc_length = hp->viscosity.length;
    P->diff_alpha = hp->diffusion.alpha;
    P->diff_beta = hp->diffusion.beta;
    P->diff_alpha_max = hp->diffusion.alpha_max;
    P->diff_alpha_min = hp->diffusion.alpha_min;
  }
  P->max_active_bin = e->max_active_bin;
  P->periodic = e->s->periodic;
  for (int k = 0; k < 3; k++) P->dim[k] = e->s->dim[k];
}

static void view_of(const struct cell *c, const struct engine *e, swh_cell_view *v) {
  v->parts = c->hydro.parts;
  v->count = c->hydro.count;
  v->active = cell_is_active_hydro(c, e);
  for (int k = 0; k < 3; k++) {
    v->loc[k] = c->loc[k];
    v->width[k] = c->width[k];
  }
}

/* src/space_getsid.h:46-82 */
static int space_getsid(const struct space *s, struct cell **ci, struct cell **cj,
                        double shift[3]) {
  double dx[3];
  for (int k = 0; k < 3; k++) {
    dx[k] = (*cj)->loc[k] - (*ci)->loc[k];
    if (s->periodic && dx[k] < -s->dim[k] / 2)
      shift[k] = s->dim[k];
    else if (s->periodic && dx[k] > s->dim[k] / 2)
      shift[k] = -s->dim[k];
    else
      shift[k] = 0.0;
    dx[k] += shift[k];
  }
  int sid = 0;
  for (int k = 0; k < 3; k++) sid = 3 * sid + ((dx[k] < 0.0) ? 0 : ((dx[k] > 0.0) ? 2 : 1));
  if (swhs_runner_flip[sid]) {
    struct cell *t = *ci;
    *ci = *cj;
    *cj = t;
    for (int k = 0; k < 3; k++) shift[k] = -shift[k];
  }
  return swhs_sortlistID[sid];
}

static void report(swh_status s) {
  static __thread char buf[512];
  if (s == SWH_OK) return;
  snprintf(buf, sizeof(buf), "%s: %s", swh_status_string(s), swh_last_error());
  SWH_ADAPTER_ERROR(buf);
}

/* DOPAIR1_BRANCH / DOPAIR2_BRANCH control logic
 * (runner_doiact_functions_hydro.h:1331-1413, 1972-2054). */
static void pair_branch(struct runner *r, struct cell *ci, struct cell *cj, int loop) {
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (ci->hydro.count == 0 || cj->hydro.count == 0) return;
  if (!cell_is_active_hydro(ci, e) && !cell_is_active_hydro(cj, e)) return;
  if (!cell_are_part_drifted(ci, e) || !cell_are_part_drifted(cj, e))
    SWH_ADAPTER_ERROR("Interacting undrifted cells.");
  double shift[3] = {0.0, 0.0, 0.0};
  const int sid = space_getsid(e->s, &ci, &cj, shift);
  if (!(ci->hydro.sorted & (1 << sid)) ||
      ci->hydro.dx_max_sort_old > space_maxreldx * ci->dmin)
    SWH_ADAPTER_ERROR("Interacting unsorted cells.");
  if (!(cj->hydro.sorted & (1 << sid)) ||
      cj->hydro.dx_max_sort_old > space_maxreldx * cj->dmin)
    SWH_ADAPTER_ERROR("Interacting unsorted cells.");
  swh_hydro_params P;
  params_of(e, &P);
  swh_cell_view vi, vj;
  view_of(ci, e, &vi);
  view_of(cj, e, &vj);
  swh_status s;
  if (loop == 0)
    s = swh_dopair_density(swhs_ctx, &vi, &vj, shift, &swhs_layout, &P);
  else if (loop == 1)
    s = swh_dopair_gradient(swhs_ctx, &vi, &vj, shift, &swhs_layout, &P);
  else
    s = swh_dopair_force(swhs_ctx, &vi, &vj, shift, &swhs_layout, &P);
  report(s);
}

/* DOSELF1_BRANCH / DOSELF2_BRANCH (runner_doiact_functions_hydro.h:2271, 2486) */
static void self_branch(struct runner *r, struct cell *c, int loop) {
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (c->hydro.count == 0) return;
  if (!cell_is_active_hydro(c, e)) return;
  if (c->hydro.h_max_old * kernel_gamma > c->dmin)
    SWH_ADAPTER_ERROR("Cell smaller than smoothing length");
  if (!cell_are_part_drifted(c, e)) SWH_ADAPTER_ERROR("Interacting undrifted cell.");
  swh_hydro_params P;
  params_of(e, &P);
  swh_cell_view v;
  view_of(c, e, &v);
  swh_status s;
  if (loop == 0)
    s = swh_doself_density(swhs_ctx, &v, &swhs_layout, &P);
  else if (loop == 1)
    s = swh_doself_gradient(swhs_ctx, &v, &swhs_layout, &P);
  else
    s = swh_doself_force(swhs_ctx, &v, &swhs_layout, &P);
  report(s);
}

void runner_doself1_branch_density(struct runner *r, struct cell *c) { self_branch(r, c, 0); }
void runner_dopair1_branch_density(struct runner *r, struct cell *ci, struct cell *cj) {
  pair_branch(r, ci, cj, 0);
}
void runner_doself1_branch_gradient(struct runner *r, struct cell *c) { self_branch(r, c, 1); }
void runner_dopair1_branch_gradient(struct runner *r, struct cell *ci, struct cell *cj) {
  pair_branch(r, ci, cj, 1);
}
void runner_doself2_branch_force(struct runner *r, struct cell *c) { self_branch(r, c, 2); }
void runner_dopair2_branch_force(struct runner *r, struct cell *ci, struct cell *cj) {
  pair_branch(r, ci, cj, 2);
}

/* DOSELF_SUBSET_BRANCH (runner_doiact_functions_hydro.h:1048-1057) */
void runner_doself_subset_branch_density(struct runner *r, struct cell *ci, struct part *parts,
                                         int *ind, int count) {
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  swh_hydro_params P;
  params_of(r->e, &P);
  swh_cell_view v;
  view_of(ci, r->e, &v);
  report(swh_doself_subset_density(swhs_ctx, &v, parts, ind, count, &swhs_layout, &P));
}

/* DOPAIR_SUBSET_BRANCH (runner_doiact_functions_hydro.h:884-937): the periodic
 * shift from the cell offsets, no swap (the flipped flag only orders the
 * sorted window walk, which the GPU does not need). */
void runner_dopair_subset_branch_density(struct runner *r, struct cell *ci,
                                         struct part *parts_i, int *ind, int count,
                                         struct cell *cj) {
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (cj->hydro.count == 0) return;
  double shift[3] = {0.0, 0.0, 0.0};
  for (int k = 0; k < 3; k++) {
    if (cj->loc[k] - ci->loc[k] < -e->s->dim[k] / 2)
      shift[k] = e->s->dim[k];
    else if (cj->loc[k] - ci->loc[k] > e->s->dim[k] / 2)
      shift[k] = -e->s->dim[k];
  }
  swh_hydro_params P;
  params_of(e, &P);
  swh_cell_view vi, vj;
  view_of(ci, e, &vi);
  view_of(cj, e, &vj);
  report(swh_dopair_subset_density(swhs_ctx, &vi, parts_i, ind, count, &vj, shift,
                                   &swhs_layout, &P));
}

/* ------------------------------------------------------------------------ */
/* Sub-cell recursion (DOSUB_SELF1/PAIR1/SELF2/PAIR2/SUBSET,                 */
/* src/runner_doiact_functions_hydro.h:2524-2805): the same descent as the   */
/* CPU runner, down to the leaf self/pair tasks above.                       */
/* ------------------------------------------------------------------------ */

/* cell_split_pairs (src/cell.c:62): for the 13 pair directions of
 * sortlistID (cj relative to ci after space_getsid's flip), the progeny
 * pairs (pid of ci, pjd of cj) that touch. Progeny k sits at offset
 * ((k >> 2) & 1, (k >> 1) & 1, k & 1) half-widths (space_split.c:233);
 * two progeny touch when every component of 2 d + off_j - off_i is in
 * [-1, 1]. Built at init instead of tabulated: the SET of pairs per sid is
 * the reference's (tests/test_dosub.py checks it against the table), their
 * ORDER is (pid, pjd) ascending, not the table's. The order only decides in
 * which order the leaf tasks of one DOSUB add into a particle's float sums,
 * and inside a leaf pair the device kernels sum in their own order anyway,
 * so the DOSUB parity tests compare with order-insensitive tolerances. */
static const int swhs_sid_dir[13][3] = {{1, 1, 1},  {1, 1, 0},  {1, 1, -1}, {1, 0, 1},
                                        {1, 0, 0},  {1, 0, -1}, {1, -1, 1}, {1, -1, 0},
                                        {1, -1, -1}, {0, 1, 1}, {0, 1, 0},  {0, 1, -1},
                                        {0, 0, 1}};
static int swhs_split_count[13];
static int swhs_split_pairs[13][16][2];

static void split_pairs_init(void) {
  for (int sid = 0; sid < 13; sid++) {
    int n = 0;
    for (int a = 0; a < 8; a++)
      for (int b = 0; b < 8; b++) {
        int ok = 1;
        for (int k = 0; k < 3; k++) {
          const int oa = (a >> (2 - k)) & 1, ob = (b >> (2 - k)) & 1;
          const int d = 2 * swhs_sid_dir[sid][k] + ob - oa;
          if (d < -1 || d > 1) ok = 0;
        }
        if (ok && n < 16) {
          swhs_split_pairs[sid][n][0] = a;
          swhs_split_pairs[sid][n][1] = b;
          n++;
        }
      }
    swhs_split_count[sid] = n;
  }
}

/* Number of progeny pairs of sid (tests compare with src/cell.c:62). */
int swifthip_swift_split_pairs(int sid, int *pairs) {
  if (sid < 0 || sid > 12) return -1;
  if (!swhs_split_count[12]) split_pairs_init();
  for (int k = 0; k < swhs_split_count[sid]; k++) {
    pairs[2 * k] = swhs_split_pairs[sid][k][0];
    pairs[2 * k + 1] = swhs_split_pairs[sid][k][1];
  }
  return swhs_split_count[sid];
}

/* src/cell.h:761-782 */
static int cell_can_recurse_in_pair_hydro_task(const struct cell *c) {
  return c->split &&
         ((kernel_gamma * c->hydro.h_max_old + c->hydro.dx_max_part_old) < 0.5f * c->dmin);
}
static int cell_can_recurse_in_self_hydro_task(const struct cell *c) {
  return c->split && (kernel_gamma * c->hydro.h_max_old < 0.5f * c->dmin);
}

/* DOSUB_PAIR1 (loop 0, 1) / DOSUB_PAIR2 (loop 2) */
static void dosub_pair(struct runner *r, struct cell *ci, struct cell *cj, int loop) {
  const struct engine *e = r->e;
  if (!cell_is_active_hydro(ci, e) && !cell_is_active_hydro(cj, e)) return;
  if (ci->hydro.count == 0 || cj->hydro.count == 0) return;
  double shift[3];
  const int sid = space_getsid(e->s, &ci, &cj, shift);
  if (cell_can_recurse_in_pair_hydro_task(ci) && cell_can_recurse_in_pair_hydro_task(cj)) {
    for (int k = 0; k < swhs_split_count[sid]; k++) {
      struct cell *pi = ci->progeny[swhs_split_pairs[sid][k][0]];
      struct cell *pj = cj->progeny[swhs_split_pairs[sid][k][1]];
      if (pi != NULL && pj != NULL) {
        dosub_pair(r, pi, pj, loop);
        if (swhs_err[0]) return;
      }
    }
  } else if (cell_is_active_hydro(ci, e) || cell_is_active_hydro(cj, e)) {
    /* the branch re-derives sid/shift and checks drift + sort state */
    pair_branch(r, ci, cj, loop);
  }
}

/* DOSUB_SELF1 / DOSUB_SELF2 */
static void dosub_self(struct runner *r, struct cell *ci, int loop) {
  if (ci->hydro.count == 0 || !cell_is_active_hydro(ci, r->e)) return;
  if (cell_can_recurse_in_self_hydro_task(ci)) {
    for (int k = 0; k < 8; k++)
      if (ci->progeny[k] != NULL) {
        dosub_self(r, ci->progeny[k], loop);
        if (swhs_err[0]) return;
        for (int j = k + 1; j < 8; j++)
          if (ci->progeny[j] != NULL) {
            dosub_pair(r, ci->progeny[k], ci->progeny[j], loop);
            if (swhs_err[0]) return;
          }
      }
  } else {
    if (loop != 2 && !cell_are_part_drifted(ci, r->e))
      SWH_ADAPTER_ERROR("Interacting undrifted cell.");
    self_branch(r, ci, loop);
  }
}

void runner_dosub_self1_density(struct runner *r, struct cell *ci, int gettimer) {
  (void)gettimer;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  dosub_self(r, ci, 0);
}
void runner_dosub_pair1_density(struct runner *r, struct cell *ci, struct cell *cj,
                                int gettimer) {
  (void)gettimer;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  dosub_pair(r, ci, cj, 0);
}
void runner_dosub_self1_gradient(struct runner *r, struct cell *ci, int gettimer) {
  (void)gettimer;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  dosub_self(r, ci, 1);
}
void runner_dosub_pair1_gradient(struct runner *r, struct cell *ci, struct cell *cj,
                                 int gettimer) {
  (void)gettimer;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  dosub_pair(r, ci, cj, 1);
}
void runner_dosub_self2_force(struct runner *r, struct cell *ci, int gettimer) {
  (void)gettimer;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  dosub_self(r, ci, 2);
}
void runner_dosub_pair2_force(struct runner *r, struct cell *ci, struct cell *cj,
                              int gettimer) {
  (void)gettimer;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  dosub_pair(r, ci, cj, 2);
}

/* DOSUB_SUBSET (runner_doiact_functions_hydro.h:2721-2805): density of the
 * particles parts[ind[0..count)] (all inside one progeny `sub` of ci) against
 * ci itself (cj == NULL) or cj, descending while the cells can recurse. */
void runner_dosub_subset_density(struct runner *r, struct cell *ci, struct part *parts,
                                 int *ind, int count, struct cell *cj, int gettimer) {
  const struct engine *e = r->e;
  (void)gettimer;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (!cell_is_active_hydro(ci, e) && (cj == NULL || !cell_is_active_hydro(cj, e))) return;
  if (ci->hydro.count == 0 || (cj != NULL && cj->hydro.count == 0)) return;
  /* the progeny of ci holding the subset */
  struct cell *sub = NULL;
  if (ci->split) {
    for (int k = 0; k < 8; k++) {
      struct cell *p = ci->progeny[k];
      if (p != NULL && &parts[ind[0]] >= &p->hydro.parts[0] &&
          &parts[ind[0]] < &p->hydro.parts[p->hydro.count]) {
        sub = p;
        break;
      }
    }
  }
  if (cj == NULL) {
    if (cell_can_recurse_in_self_hydro_task(ci)) {
      runner_dosub_subset_density(r, sub, parts, ind, count, NULL, 0);
      for (int j = 0; j < 8; j++)
        if (ci->progeny[j] != sub && ci->progeny[j] != NULL) {
          if (swhs_err[0]) return;
          runner_dosub_subset_density(r, sub, parts, ind, count, ci->progeny[j], 0);
        }
    } else {
      runner_doself_subset_branch_density(r, ci, parts, ind, count);
    }
  } else {
    if (cell_can_recurse_in_pair_hydro_task(ci) && cell_can_recurse_in_pair_hydro_task(cj)) {
      double shift[3] = {0.0, 0.0, 0.0};
      const int sid = space_getsid(e->s, &ci, &cj, shift);
      for (int k = 0; k < swhs_split_count[sid]; k++) {
        struct cell *pi = ci->progeny[swhs_split_pairs[sid][k][0]];
        struct cell *pj = cj->progeny[swhs_split_pairs[sid][k][1]];
        if (swhs_err[0]) return;
        if (pi == sub && pj != NULL)
          runner_dosub_subset_density(r, pi, parts, ind, count, pj, 0);
        if (pi != NULL && pj == sub)
          runner_dosub_subset_density(r, pj, parts, ind, count, pi, 0);
      }
    } else if (cell_is_active_hydro(ci, e) || cell_is_active_hydro(cj, e)) {
      if (!cell_are_part_drifted(cj, e)) SWH_ADAPTER_ERROR("Cell should be drifted!");
      runner_dopair_subset_branch_density(r, ci, parts, ind, count, cj);
    }
  }
}

static void grav_params_of(const struct engine *e, swh_grav_params *G) {
  memset(G, 0, sizeof(*G));
  G->periodic = e->mesh->periodic;
  for (int k = 0; k < 3; k++) G->dim[k] = (float)e->mesh->dim[k];
  G->r_s_inv = e->mesh->r_s_inv;
  G->r_cut_min = e->mesh->r_cut_min;
  G->r_cut_max = e->mesh->r_cut_max;
  G->max_active_bin = e->max_active_bin;
  const struct gravity_props *gp = e->gravity_properties;
  if (gp) {  /* gravity_M2P_accept's inputs (multipole_accept.h:290-373) */
    G->theta_crit = (float)gp->theta_crit;
    G->adaptive_tolerance = gp->adaptive_tolerance;
    G->use_advanced_MAC = gp->use_advanced_MAC;
    G->use_gadget_tolerance = gp->use_gadget_tolerance;
    G->use_tree_below_softening = gp->use_tree_below_softening;
    G->consider_truncation_in_MAC = gp->consider_truncation_in_MAC;
  }
}

/* struct gravity_tensors -> swh_multipole (include/swifthip.h's M order) */
static void multipole_of(const struct gravity_tensors *t, swh_multipole *o) {
  const struct multipole *m = &t->m_pole;
  for (int k = 0; k < 3; k++) o->CoM[k] = t->CoM[k];
  o->r_max = t->r_max;
  const float M[SWH_MPOLE_TERMS] = {
      m->M_000, 0.f,      0.f,      0.f,      m->M_200, m->M_020, m->M_002, m->M_110, m->M_101,
      m->M_011, m->M_300, m->M_030, m->M_003, m->M_210, m->M_201, m->M_120, m->M_021, m->M_102,
      m->M_012, m->M_111, m->M_400, m->M_040, m->M_004, m->M_310, m->M_301, m->M_130, m->M_031,
      m->M_103, m->M_013, m->M_220, m->M_202, m->M_022, m->M_211, m->M_121, m->M_112};
  memcpy(o->M, M, sizeof(M));
  for (int k = 0; k < 5; k++) o->power[k] = m->power[k];
  o->max_softening = m->max_softening;
  o->min_old_a_grav_norm = m->min_old_a_grav_norm;
}

static void gview_of(const struct cell *c, int active, swh_gcell_view *v) {
  v->gparts = c->grav.parts;
  v->count = c->grav.count;
  v->active = active;
  for (int k = 0; k < 3; k++) {
    v->loc[k] = c->loc[k];
    v->width[k] = c->width[k];
    v->CoM[k] = c->grav.multipole ? c->grav.multipole->CoM[k] : 0.;
  }
  v->r_max = c->grav.multipole ? c->grav.multipole->r_max : 0.;
  v->multipole = NULL;
}

/* runner_doself_grav_pp (runner_doiact_grav.c:1788-1871) */
void runner_doself_grav_pp(struct runner *r, struct cell *c) {
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (!cell_is_active_gravity(c, e)) return;
  if (c->split) SWH_ADAPTER_ERROR("Running P-P on a splitable cell");
  swh_grav_params G;
  grav_params_of(e, &G);
  swh_gcell_view v;
  gview_of(c, 1, &v);
  report(swh_grav_self_pp(swhs_ctx, &v, &swhs_glayout, &G));
}

/* runner_dopair_grav_pp (runner_doiact_grav.c:1202-1425), including the M2P
 * branch: with allow_mpole (the recursive pair task always passes 1,
 * runner_doiact_grav.c:2315) the particles that pass gravity_M2P_accept
 * against the other cell's multipole take runner_dopair_grav_pm_* instead of
 * P2P; the library evaluates the acceptance in float exactly as
 * gravity_cache_populate does. */
void runner_dopair_grav_pp(struct runner *r, struct cell *ci, struct cell *cj,
                           const int symmetric, const int allow_mpole) {
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  const int ci_active = cell_is_active_gravity(ci, e) && (ci->nodeID == e->nodeID);
  const int cj_active = cell_is_active_gravity(cj, e) && (cj->nodeID == e->nodeID);
  if (!ci_active && !cj_active) return;
  if (!ci_active && !symmetric) return;
  if (allow_mpole && (!ci->grav.multipole || !cj->grav.multipole))
    SWH_ADAPTER_ERROR("allow_mpole without cell multipoles");
  if (allow_mpole && !e->gravity_properties)
    SWH_ADAPTER_ERROR("allow_mpole without e->gravity_properties");
  swh_grav_params G;
  grav_params_of(e, &G);
  swh_gcell_view vi, vj;
  gview_of(ci, ci_active, &vi);
  gview_of(cj, cj_active, &vj);
  swh_multipole mi, mj;
  if (allow_mpole) {
    multipole_of(ci->grav.multipole, &mi);
    multipole_of(cj->grav.multipole, &mj);
    vi.multipole = &mi;
    vj.multipole = &mj;
  }
  report(swh_grav_pair_pp(swhs_ctx, &vi, &vj, symmetric, allow_mpole, &swhs_glayout, &G));
}


/* ------------------------------------------------------------------------ */
/* Tree gravity per task: runner_doself_recursive_grav /                     */
/* runner_dopair_recursive_grav (runner_doiact_grav.c:2386, 2208) and        */
/* runner_do_grav_down (65-164). The task's cell tree(s) are flattened into  */
/* libswifthip's swh_gcell table with SWIFT's own multipoles                 */
/* (swh_gspace_set_multipoles); the library makes the recursion's decisions  */
/* on the device (r_cut_max skip, P-P of <= 1-particle cells, M-M under      */
/* gravity_M2L_accept_symmetric, leaf P-P with M2P, split the larger cell)   */
/* and returns the P-P accelerations and the M2L field tensors, which are    */
/* added into c->grav.multipole->pot as the reference's M-M interactions do  */
/* (the down pass is its own task, as in SWIFT).                             */
/* ------------------------------------------------------------------------ */

struct swhs_tree {
  swh_gcell *cells;
  struct cell **cptr;
  int n, cap;
};

static int swhs_tree_add(struct swhs_tree *t, struct cell *c, const struct gpart *base,
                         int offset) {
  if (t->n == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 64;
    t->cells = (swh_gcell *)realloc(t->cells, (size_t)t->cap * sizeof(swh_gcell));
    t->cptr = (struct cell **)realloc(t->cptr, (size_t)t->cap * sizeof(struct cell *));
  }
  const int id = t->n++;
  swh_gcell *g = &t->cells[id];
  memset(g, 0, sizeof(*g));
  g->start = offset + (int)(c->grav.parts - base);
  g->count = c->grav.count;
  g->split = c->split;
  for (int k = 0; k < 3; k++) {
    g->loc[k] = c->loc[k];
    g->width[k] = c->width[k];
  }
  t->cptr[id] = c;
  for (int k = 0; k < 8; k++) {
    t->cells[id].progeny[k] = -1;
    if (c->split && c->progeny[k] && c->progeny[k]->grav.count > 0) {
      const int p = swhs_tree_add(t, c->progeny[k], base, offset);
      t->cells[id].progeny[k] = p;
    }
  }
  return id;
}

static void swhs_tree_free(struct swhs_tree *t) {
  free(t->cells);
  free(t->cptr);
}

/* struct grav_tensor <-> the library's 35 floats (swh_multipole::M order) */
static void tensor_to(const struct grav_tensor *p, float *f) {
  const float v[SWH_MPOLE_TERMS] = {
      p->F_000, p->F_100, p->F_010, p->F_001, p->F_200, p->F_020, p->F_002, p->F_110, p->F_101,
      p->F_011, p->F_300, p->F_030, p->F_003, p->F_210, p->F_201, p->F_120, p->F_021, p->F_102,
      p->F_012, p->F_111, p->F_400, p->F_040, p->F_004, p->F_310, p->F_301, p->F_130, p->F_031,
      p->F_103, p->F_013, p->F_220, p->F_202, p->F_022, p->F_211, p->F_121, p->F_112};
  memcpy(f, v, sizeof(v));
}
static void tensor_from(struct grav_tensor *p, const float *f, int add) {
  float *d[SWH_MPOLE_TERMS] = {
      &p->F_000, &p->F_100, &p->F_010, &p->F_001, &p->F_200, &p->F_020, &p->F_002, &p->F_110,
      &p->F_101, &p->F_011, &p->F_300, &p->F_030, &p->F_003, &p->F_210, &p->F_201, &p->F_120,
      &p->F_021, &p->F_102, &p->F_012, &p->F_111, &p->F_400, &p->F_040, &p->F_004, &p->F_310,
      &p->F_301, &p->F_130, &p->F_031, &p->F_103, &p->F_013, &p->F_220, &p->F_202, &p->F_022,
      &p->F_211, &p->F_121, &p->F_112};
  for (int k = 0; k < SWH_MPOLE_TERMS; k++) *d[k] = add ? *d[k] + f[k] : f[k];
}

/* Upload the task's gparts (roots' slices, concatenated in a staging copy)
 * with its tree and SWIFT's multipoles. */
static swh_status swhs_gspace_for(swh_gspace **gs, struct swhs_tree *t, struct cell **roots,
                                  const int *offs, int nroots, char **stage, int total) {
  const size_t st = (size_t)swhs_glayout.stride;
  const size_t need = (size_t)(total > 0 ? total : 1) * st;
  if (need > swhs_tls_stage_cap) {
    char *b = (char *)realloc(swhs_tls_stage, need);
    if (!b) return SWH_ERR_OOM;
    swhs_tls_stage = b;
    swhs_tls_stage_cap = need;
  }
  *stage = swhs_tls_stage;
  for (int r = 0; r < nroots; r++)
    memcpy(*stage + (size_t)offs[r] * st, roots[r]->grav.parts, (size_t)roots[r]->grav.count * st);
  swh_status s = SWH_OK;
  if (swhs_tls_gs && swhs_tls_gen == swhs_ctx_gen) {
    *gs = swhs_tls_gs;
  } else {
    swhs_tls_gs = NULL;
    s = swh_gspace_create(swhs_ctx, gs);
    if (s != SWH_OK) return s;
    pthread_mutex_lock(&swhs_reg_lock);
    if (swhs_nreg < SWHS_MAX_GSPACES) {
      swhs_reg[swhs_nreg++] = *gs;
      swhs_tls_gs = *gs;
      swhs_tls_gen = swhs_ctx_gen;
    }
    pthread_mutex_unlock(&swhs_reg_lock);
  }
  s = swh_gspace_upload(*gs, *stage, total, &swhs_glayout, 0);
  if (s == SWH_OK) s = swh_gspace_set_tree(*gs, t->cells, t->n);
  if (s == SWH_OK) {
    swh_multipole *mp = (swh_multipole *)calloc((size_t)t->n, sizeof(swh_multipole));
    for (int c = 0; c < t->n; c++) multipole_of(t->cptr[c]->grav.multipole, &mp[c]);
    s = swh_gspace_set_multipoles(*gs, mp);
    free(mp);
  }
  return s;
}

/* After the tasks: the gparts of the local roots get their results back
 * (swh_gspace_download adds them to the staging copy), the local cells'
 * field tensors receive their M2L sums. */
static swh_status swhs_gspace_finish(swh_gspace *gs, struct swhs_tree *t, struct cell **roots,
                                     const int *offs, int nroots, char *stage,
                                     const struct engine *e, int tensors_add) {
  swh_status s = swh_gspace_download(gs, stage, &swhs_glayout, 0);
  const size_t st = (size_t)swhs_glayout.stride;
  if (s == SWH_OK)
    for (int r = 0; r < nroots; r++)
      if (roots[r]->nodeID == e->nodeID)
        memcpy(roots[r]->grav.parts, stage + (size_t)offs[r] * st,
               (size_t)roots[r]->grav.count * st);
  if (s == SWH_OK) {
    float *f = (float *)malloc((size_t)t->n * SWH_MPOLE_TERMS * sizeof(float));
    s = swh_gspace_field_tensors(gs, f);
    for (int c = 0; s == SWH_OK && c < t->n; c++) {
      struct cell *cc = t->cptr[c];
      if (cc->nodeID != e->nodeID || !cc->grav.multipole) continue;
      const float *fc = f + (size_t)c * SWH_MPOLE_TERMS;
      if (tensors_add) {
        int any = 0;
        for (int k = 0; k < SWH_MPOLE_TERMS; k++) any |= fc[k] != 0.f;
        if (!any) continue; /* no M-M interaction reached this cell */
        tensor_from(&cc->grav.multipole->pot, fc, 1);
        cc->grav.multipole->pot.interacted = 1;
      } else if (c > 0 && cell_is_active_gravity(cc, e)) {
        /* grav_down: the progeny tensors with their parents' pushed in
         * (gravity_field_tensors_add marks them interacted) */
        tensor_from(&cc->grav.multipole->pot, fc, 0);
        int any = 0;
        for (int k = 0; k < SWH_MPOLE_TERMS; k++) any |= fc[k] != 0.f;
        if (any) cc->grav.multipole->pot.interacted = 1;
      }
    }
    free(f);
  }
  (void)stage;                            /* the thread's staging buffer, kept */
  if (gs != swhs_tls_gs) swh_gspace_destroy(gs);  /* unregistered: a task's own */
  return s;
}

/* runner_doself_recursive_grav (runner_doiact_grav.c:2386-2431) */
void runner_doself_recursive_grav(struct runner *r, struct cell *c, int gettimer) {
  (void)gettimer;
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (c->grav.count == 0) SWH_ADAPTER_ERROR("Doing self gravity on an empty cell !");
  if (!cell_is_active_gravity(c, e)) return;
  if (!c->grav.multipole) SWH_ADAPTER_ERROR("self gravity without cell multipoles");
  swh_grav_params G;
  grav_params_of(e, &G);
  struct swhs_tree t = {0};
  swhs_tree_add(&t, c, c->grav.parts, 0);
  swh_gspace *gs = NULL;
  char *stage = NULL;
  const int off = 0;
  swh_status s = swhs_gspace_for(&gs, &t, &c, &off, 1, &stage, c->grav.count);
  const int32_t self = 0;
  if (s == SWH_OK) s = swh_grav_tree_tasks(gs, &G, &self, 1, NULL, 0, SWH_TREE_NO_DOWN, NULL);
  if (gs) {
    const swh_status s2 = swhs_gspace_finish(gs, &t, &c, &off, 1, stage, e, 1);
    if (s == SWH_OK) s = s2;
  }
  swhs_tree_free(&t);
  report(s);
}

/* runner_dopair_recursive_grav (runner_doiact_grav.c:2208-2370) */
void runner_dopair_recursive_grav(struct runner *r, struct cell *ci, struct cell *cj,
                                  int gettimer) {
  (void)gettimer;
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (!((cell_is_active_gravity(ci, e) && ci->nodeID == e->nodeID) ||
        (cell_is_active_gravity(cj, e) && cj->nodeID == e->nodeID)))
    return;
  if (ci->grav.count == 0 || cj->grav.count == 0)
    SWH_ADAPTER_ERROR("Doing pair gravity on an empty cell !");
  if (ci == cj) SWH_ADAPTER_ERROR("Pair interaction between a cell and itself.");
  if (!ci->grav.multipole || !cj->grav.multipole)
    SWH_ADAPTER_ERROR("pair gravity without cell multipoles");
  swh_grav_params G;
  grav_params_of(e, &G);
  struct cell *roots[2] = {ci, cj};
  const int offs[2] = {0, ci->grav.count};
  struct swhs_tree t = {0};
  const int32_t pair[2] = {swhs_tree_add(&t, ci, ci->grav.parts, 0),
                           swhs_tree_add(&t, cj, cj->grav.parts, ci->grav.count)};
  swh_gspace *gs = NULL;
  char *stage = NULL;
  swh_status s = swhs_gspace_for(&gs, &t, roots, offs, 2, &stage, ci->grav.count + cj->grav.count);
  if (s == SWH_OK) s = swh_grav_tree_tasks(gs, &G, NULL, 0, pair, 1, SWH_TREE_NO_DOWN, NULL);
  if (gs) {
    const swh_status s2 = swhs_gspace_finish(gs, &t, roots, offs, 2, stage, e, 1);
    if (s == SWH_OK) s = s2;
  }
  swhs_tree_free(&t);
  report(s);
}

/* runner_do_grav_down (runner_doiact_grav.c:65-164) */
void runner_do_grav_down(struct runner *r, struct cell *c, int timer) {
  (void)timer;
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  if (!c->grav.multipole) SWH_ADAPTER_ERROR("grav_down without cell multipoles");
  if (c->grav.count == 0) return;
  swh_grav_params G;
  grav_params_of(e, &G);
  struct swhs_tree t = {0};
  swhs_tree_add(&t, c, c->grav.parts, 0);
  swh_gspace *gs = NULL;
  char *stage = NULL;
  const int off = 0;
  swh_status s = swhs_gspace_for(&gs, &t, &c, &off, 1, &stage, c->grav.count);
  if (s == SWH_OK) {
    /* the cells' tensors; those that received nothing (interacted == 0) push
     * nothing, as the reference's test skips them */
    float *f = (float *)calloc((size_t)t.n * SWH_MPOLE_TERMS, sizeof(float));
    for (int k = 0; k < t.n; k++)
      if (t.cptr[k]->grav.multipole && t.cptr[k]->grav.multipole->pot.interacted)
        tensor_to(&t.cptr[k]->grav.multipole->pot, f + (size_t)k * SWH_MPOLE_TERMS);
    s = swh_gspace_grav_down(gs, &G, f);
    free(f);
  }
  if (gs) {
    const swh_status s2 = swhs_gspace_finish(gs, &t, &c, &off, 1, stage, e, 0);
    if (s == SWH_OK) s = s2;
  }
  swhs_tree_free(&t);
  report(s);
}

/* ------------------------------------------------------------------------ */
/* The M-M tasks outside the recursive walk: runner_dopair_grav_mm_progenies */
/* (runner_doiact_grav.c:2067-2093) and runner_do_grav_long_range            */
/* (2441-2530). Each task's M-M pairs go to the GPU as one batch             */
/* (swh_grav_m2l_pairs: the tree's M2L kernel on SWIFT's own multipoles); the */
/* sums are added into c->grav.multipole->pot as gravity_M2L_apply does.     */
/* ------------------------------------------------------------------------ */

/* SWIFT's cell_drift_multipole (src/cell_drift.c:1178) when the adapter is
 * linked into SWIFT; absent here (the tests hand in drifted multipoles). */
extern void cell_drift_multipole(struct cell *c, const struct engine *e) __attribute__((weak));

static int cell_is_active_gravity_mm(const struct cell *c, const struct engine *e) {
  return c->grav.ti_end_min == e->ti_current; /* src/active.h:258-262 */
}

static int swhs_drift_multipole(struct cell *c, const struct engine *e) {
  if (c->grav.ti_old_multipole >= e->ti_current) return 1;
  if (!cell_drift_multipole) {
    SWH_ADAPTER_ERROR("Undrifted multipole (cell_drift_multipole is SWIFT's)");
    return 0;
  }
  cell_drift_multipole(c, e);
  return 1;
}

struct swhs_mm {
  struct cell **cells; /* distinct cells, index = multipole slot */
  int32_t *pairs;      /* {target, source, symmetric} */
  int ncells, npairs, cap_c, cap_p;
};

static int swhs_mm_slot(struct swhs_mm *b, struct cell *c) {
  for (int k = 0; k < b->ncells; k++)
    if (b->cells[k] == c) return k;
  if (b->ncells == b->cap_c) {
    b->cap_c = b->cap_c ? 2 * b->cap_c : 16;
    b->cells = (struct cell **)realloc(b->cells, (size_t)b->cap_c * sizeof(struct cell *));
  }
  b->cells[b->ncells] = c;
  return b->ncells++;
}

static void swhs_mm_add(struct swhs_mm *b, struct cell *t, struct cell *s, int sym) {
  if (b->npairs == b->cap_p) {
    b->cap_p = b->cap_p ? 2 * b->cap_p : 64;
    b->pairs = (int32_t *)realloc(b->pairs, (size_t)b->cap_p * 3 * sizeof(int32_t));
  }
  int32_t *q = b->pairs + 3 * (size_t)b->npairs++;
  q[0] = swhs_mm_slot(b, t);
  q[1] = swhs_mm_slot(b, s);
  q[2] = sym;
}

/* runner_dopair_grav_mm (runner_doiact_grav.c:2032-2064): symmetric when both
 * cells are active and local, else the active local one receives. */
static int swhs_mm_pair(struct swhs_mm *b, const struct engine *e, struct cell *ci,
                        struct cell *cj) {
  const int do_i = cell_is_active_gravity_mm(ci, e) && (ci->nodeID == e->nodeID);
  const int do_j = cell_is_active_gravity_mm(cj, e) && (cj->nodeID == e->nodeID);
  if (!ci->grav.multipole || !cj->grav.multipole) {
    SWH_ADAPTER_ERROR("M-M interaction without cell multipoles");
    return 0;
  }
  if (!swhs_drift_multipole(ci, e) || !swhs_drift_multipole(cj, e)) return 0;
  if (do_i && do_j) {
    swhs_mm_add(b, ci, cj, 1);
    swhs_mm_add(b, cj, ci, 1);
  } else if (do_i) {
    swhs_mm_add(b, ci, cj, 0);
  } else if (do_j) {
    swhs_mm_add(b, cj, ci, 0);
  }
  return 1;
}

/* The batch on the GPU; each target's sums added into its field tensor. */
static void swhs_mm_run(struct swhs_mm *b, const struct engine *e) {
  if (b->npairs > 0) {
    swh_grav_params G;
    grav_params_of(e, &G);
    swh_multipole *mp = (swh_multipole *)calloc((size_t)b->ncells, sizeof(swh_multipole));
    float *f = (float *)malloc((size_t)b->ncells * SWH_MPOLE_TERMS * sizeof(float));
    for (int k = 0; k < b->ncells; k++) multipole_of(b->cells[k]->grav.multipole, &mp[k]);
    const swh_status s = swh_grav_m2l_pairs(swhs_ctx, &G, mp, b->ncells, b->pairs, b->npairs, f);
    if (s == SWH_OK) {
      char *target = (char *)calloc((size_t)b->ncells, 1);
      for (int q = 0; q < b->npairs; q++) target[b->pairs[3 * q]] = 1;
      for (int k = 0; k < b->ncells; k++) {
        if (!target[k]) continue;
        struct grav_tensor *pot = &b->cells[k]->grav.multipole->pot;
        tensor_from(pot, f + (size_t)k * SWH_MPOLE_TERMS, 1);
        pot->interacted = 1;
      }
      free(target);
    }
    free(f);
    free(mp);
    report(s);
  }
  free(b->cells);
  free(b->pairs);
}

/* runner_dopair_grav_mm_progenies (runner_doiact_grav.c:2067-2093) */
void runner_dopair_grav_mm_progenies(struct runner *r, const long long flags, struct cell *ci,
                                     struct cell *cj) {
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  /* (runner_clear_grav_flags: the cells' unskip flags are the scheduler's,
   * which this drop-in does not hold) */
  struct swhs_mm b = {0};
  int ok = 1;
  for (int i = 0; ok && i < 8; i++) {
    if (ci->progeny[i] == NULL) continue;
    for (int j = 0; ok && j < 8; j++) {
      if (cj->progeny[j] == NULL) continue;
      /* did the last rebuild flag this progeny pair well separated? */
      if (flags & (1ULL << (i * 8 + j))) ok = swhs_mm_pair(&b, e, ci->progeny[i], cj->progeny[j]);
    }
  }
  if (!ok) b.npairs = 0;
  swhs_mm_run(&b, e);
}

/* cell_min_dist2_same_size (src/cell.h:696-750) */
static double swhs_nearest(double d, double L) {
  return d > 0.5 * L ? d - L : (d < -0.5 * L ? d + L : d);
}
static double swhs_min4(double a, double b, double c, double d) {
  const double x = a < b ? a : b, y = c < d ? c : d;
  return x < y ? x : y;
}
static double cell_min_dist2_same_size(const struct cell *ci, const struct cell *cj, int periodic,
                                       const double dim[3]) {
  double d2 = 0.;
  for (int k = 0; k < 3; k++) {
    const double imin = ci->loc[k], imax = ci->loc[k] + ci->width[k];
    const double jmin = cj->loc[k], jmax = cj->loc[k] + cj->width[k];
    double dk;
    if (periodic)
      dk = swhs_min4(fabs(swhs_nearest(imin - jmin, dim[k])), fabs(swhs_nearest(imin - jmax, dim[k])),
                     fabs(swhs_nearest(imax - jmin, dim[k])), fabs(swhs_nearest(imax - jmax, dim[k])));
    else
      dk = swhs_min4(fabs(imin - jmin), fabs(imin - jmax), fabs(imax - jmin), fabs(imax - jmax));
    d2 += dk * dk;
  }
  return d2;
}

/* cell_can_use_pair_mm (src/cell.c:1420-1460) with use_rebuild_data = 1,
 * is_tree_walk = 0: the MAC of the rebuild-time CoMs and sizes */
static int cell_can_use_pair_mm_rebuild(const struct cell *ci, const struct cell *cj,
                                        const struct engine *e, const swh_grav_params *G) {
  const struct gravity_tensors *A = ci->grav.multipole, *B = cj->grav.multipole;
  double r2 = 0.;
  for (int k = 0; k < 3; k++) {
    double d = A->CoM_rebuild[k] - B->CoM_rebuild[k];
    if (e->s->periodic) d = swhs_nearest(d, e->s->dim[k]);
    r2 += d * d;
  }
  swh_multipole ma, mb;
  multipole_of(A, &ma);
  multipole_of(B, &mb);
  ma.r_max = A->r_max_rebuild;
  mb.r_max = B->r_max_rebuild;
  return swh_grav_m2l_accept(G, &ma, &mb, r2);
}

/* runner_do_grav_long_range (runner_doiact_grav.c:2441-2530) */
void runner_do_grav_long_range(struct runner *r, struct cell *ci, int timer) {
  (void)timer;
  const struct engine *e = r->e;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  const struct space *s = e->s;
  const int periodic = e->mesh->periodic;
  const double dim[3] = {e->mesh->dim[0], e->mesh->dim[1], e->mesh->dim[2]};
  const double max_distance2 = e->mesh->r_cut_max * e->mesh->r_cut_max;
  if (!cell_is_active_gravity(ci, e)) return;
  if (ci->nodeID != e->nodeID) {
    SWH_ADAPTER_ERROR("Non-local cell in long-range gravity task!");
    return;
  }
  if (!ci->grav.multipole) {
    SWH_ADAPTER_ERROR("long-range gravity without cell multipoles");
    return;
  }
  if (!swhs_drift_multipole(ci, e)) return;
  struct gravity_tensors *const multi_i = ci->grav.multipole;
  struct cell *top = ci;
  while (top->parent != NULL) top = top->parent;
  swh_grav_params G;
  grav_params_of(e, &G);
  struct swhs_mm b = {0};
  for (int n = 0; n < s->nr_cells_with_particles; ++n) {
    struct cell *cj = &s->cells_top[s->cells_with_particles_top[n]];
    const struct gravity_tensors *multi_j = cj->grav.multipole;
    if (top == cj) continue;                /* no self contribution */
    if (multi_j->m_pole.M_000 == 0.f) continue;  /* empty */
    if (periodic && cell_min_dist2_same_size(top, cj, periodic, dim) > max_distance2) {
      multi_i->pot.interacted = 1; /* beyond the truncated forces: the mesh's */
      continue;
    }
    if (cell_can_use_pair_mm_rebuild(top, cj, e, &G)) {
      /* runner_dopair_grav_mm_nonsym(r, ci, cj): the active local ci receives */
      if (cell_is_active_gravity_mm(ci, e) && ci->nodeID == e->nodeID)
        swhs_mm_add(&b, ci, cj, 0);
      multi_i->pot.interacted = 1;
    }
  }
  swhs_mm_run(&b, e);
}
