/*
 * solver.h -- the pivot loop (replaces reference include/solver.h:1-25, solver.cu:128-149).
 *
 * int solve(tabular_t*, int* base): runs simplex pivots on the device tableau until the
 * reduced costs are all >= 0 (FEASIBLE, 0) or the entering column has no entry >= 1e-9
 * (UNBOUNDED, -2).  `base` is a host array of `cols` ints (basic variable per constraint
 * row), read on entry and written back on return (the reference used mapped pinned
 * memory, twoPhaseMethod.cu:391-393).  No iteration cap, as in the reference.
 */
#ifndef SIMPLEX_SOLVER_H
#define SIMPLEX_SOLVER_H

#include "tabular.h"

#ifdef __cplusplus
extern "C" {
#endif

int solve(tabular_t *tabular, int *base);

#ifdef __cplusplus
}
#endif
#endif
