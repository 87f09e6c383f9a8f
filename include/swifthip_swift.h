/*
 * swifthip_swift.h — SWIFT's per-task hot-path entry points, implemented on
 * the GPU by libswifthip_swift (swift_subtask_dev_amd/csrc/swh_swift_adapter.c).
 *
 * Signatures are exactly SWIFT's (reference file:line of the function each one
 * replaces; names and argument meaning unchanged):
 *   runner_doself1_branch_density      src/runner_doiact_hydro.h:168-170 -> DOSELF1_BRANCH
 *   runner_dopair1_branch_density      src/runner_doiact_hydro.h:171     -> DOPAIR1_BRANCH
 *   runner_doself1_branch_gradient / runner_dopair1_branch_gradient (same template,
 *                                      src/runner_doiact_hydro.c:48-53)
 *   runner_doself2_branch_force        -> DOSELF2_BRANCH (runner_doiact_functions_hydro.h:2486)
 *   runner_dopair2_branch_force        -> DOPAIR2_BRANCH (runner_doiact_functions_hydro.h:1972)
 *   runner_doself_subset_branch_density src/runner_doiact_hydro.h:182   -> DOSELF_SUBSET_BRANCH
 *   runner_dopair_subset_branch_density src/runner_doiact_hydro.h:185   -> DOPAIR_SUBSET_BRANCH
 *   runner_doself_grav_pp               src/runner_doiact_grav.h:41     (runner_doiact_grav.c:1788)
 *   runner_dopair_grav_pp               src/runner_doiact_grav.h:44-50  (runner_doiact_grav.c:1202)
 *
 * Inside a SWIFT build these are compiled against SWIFT's headers and linked
 * instead of the CPU template instances; in this repo they are
 * compiled against include/swift_compat.h (same field names).
 *
 * Error behaviour: where SWIFT calls error() (abort) the adapter calls
 * SWH_ADAPTER_ERROR(msg) — SWIFT's error() in a SWIFT build; in this repo it
 * records the message (swifthip_swift_last_error) and returns.
 */
#ifndef SWIFTHIP_SWIFT_H
#define SWIFTHIP_SWIFT_H

#include "swift_compat.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define SWHS_API __attribute__((visibility("default")))
#else
#define SWHS_API
#endif

/* Process-wide GPU context of the adapter (device ordinal; call once before
 * the first task, e.g. from engine_config). Precision: 0 = fp64, 1 = fp32. */
SWHS_API int swifthip_swift_init(int device, int precision);
SWHS_API void swifthip_swift_finalize(void);
/* Switch the arithmetic of subsequent tasks: 0 = fp64, 1 = fp32. */
SWHS_API int swifthip_swift_set_precision(int precision);
/* Last adapter error ("Interacting unsorted cells." ...) or "" . */
SWHS_API const char *swifthip_swift_last_error(void);
SWHS_API void swifthip_swift_clear_error(void);

SWHS_API void runner_doself1_branch_density(struct runner *r, struct cell *c);
SWHS_API void runner_dopair1_branch_density(struct runner *r, struct cell *ci, struct cell *cj);
SWHS_API void runner_doself1_branch_gradient(struct runner *r, struct cell *c);
SWHS_API void runner_dopair1_branch_gradient(struct runner *r, struct cell *ci, struct cell *cj);
SWHS_API void runner_doself2_branch_force(struct runner *r, struct cell *c);
SWHS_API void runner_dopair2_branch_force(struct runner *r, struct cell *ci, struct cell *cj);
SWHS_API void runner_doself_subset_branch_density(struct runner *r, struct cell *ci,
                                                  struct part *parts, int *ind, int count);
SWHS_API void runner_dopair_subset_branch_density(struct runner *r, struct cell *ci,
                                                  struct part *parts_i, int *ind, int count,
                                                  struct cell *cj);
SWHS_API void runner_doself_grav_pp(struct runner *r, struct cell *c);
SWHS_API void runner_dopair_grav_pp(struct runner *r, struct cell *ci, struct cell *cj,
                                    const int symmetric, const int allow_mpole);

#ifdef __cplusplus
}
#endif

#endif /* SWIFTHIP_SWIFT_H */
