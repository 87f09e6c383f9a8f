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
#include <stdio.h>
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

#define kernel_gamma ((float)(1.825742)) /* src/kernel_hydro.h:51 */
#define space_maxreldx 0.1f              /* src/space.h:66 */

/* src/sort_part.h:59-92 */
static const int swhs_runner_flip[27] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0,
                                         0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static const int swhs_sortlistID[27] = {0, 1, 2, 3, 4,  5,  6,  7,  8,  9,  10, 11, 12, 0,
                                        12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0};

int swifthip_swift_init(int device, int precision) {
  if (swhs_ctx) return 0;
  if (swh_init(&swhs_ctx, device) != SWH_OK) return -1;
  swh_set_precision(swhs_ctx, precision ? SWH_PRECISION_F32 : SWH_PRECISION_F64);
  swh_part_layout_sphenix(&swhs_layout);
  swh_gpart_layout_multisoftening(&swhs_glayout);
  return 0;
}

int swifthip_swift_set_precision(int precision) {
  if (!swhs_ctx) return -1;
  return swh_set_precision(swhs_ctx, precision ? SWH_PRECISION_F32 : SWH_PRECISION_F64) ==
                 SWH_OK
             ? 0
             : -1;
}

void swifthip_swift_finalize(void) {
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

static void grav_params_of(const struct engine *e, swh_grav_params *G) {
  memset(G, 0, sizeof(*G));
  G->periodic = e->mesh->periodic;
  for (int k = 0; k < 3; k++) G->dim[k] = (float)e->mesh->dim[k];
  G->r_s_inv = e->mesh->r_s_inv;
  G->r_cut_min = e->mesh->r_cut_min;
  G->max_active_bin = e->max_active_bin;
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

/* runner_dopair_grav_pp (runner_doiact_grav.c:1202-1425). The M2P branch
 * (allow_mpole) is outside this path: every particle takes the P2P route,
 * i.e. the result equals the reference with no particle passing
 * gravity_M2P_accept. */
void runner_dopair_grav_pp(struct runner *r, struct cell *ci, struct cell *cj,
                           const int symmetric, const int allow_mpole) {
  const struct engine *e = r->e;
  (void)allow_mpole;
  if (!swhs_ctx) SWH_ADAPTER_ERROR("swifthip_swift_init() was not called");
  const int ci_active = cell_is_active_gravity(ci, e) && (ci->nodeID == e->nodeID);
  const int cj_active = cell_is_active_gravity(cj, e) && (cj->nodeID == e->nodeID);
  if (!ci_active && !cj_active) return;
  if (!ci_active && !symmetric) return;
  swh_grav_params G;
  grav_params_of(e, &G);
  swh_gcell_view vi, vj;
  gview_of(ci, ci_active, &vi);
  gview_of(cj, cj_active, &vj);
  report(swh_grav_pair_pp(swhs_ctx, &vi, &vj, symmetric, &swhs_glayout, &G));
}
