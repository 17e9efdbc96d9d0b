/*
 * twoPhaseMethod.h -- the drop-in entry point (replaces reference include/twoPhaseMethod.h:1-23).
 *
 * int twoPhaseMethod(problem_t*, TYPE* solution, TYPE* optimalValue)
 *   returns FEASIBLE (0, optimum found), INFEASIBLE (-1), UNBOUNDED (-2) or DEGENERATE (-3:
 *   an artificial variable is still basic after phase 1; phase 2 is skipped).
 *   solution (caller-allocated, >= vars doubles) and *optimalValue are written only on 0.
 * enableBenchmarkMode/disableBenchmarkMode exist unconditionally (the reference had them
 * only under -D TIMER): they switch the timing CSV to benchmark_<n>_<m>.txt naming.
 */
#ifndef SIMPLEX_TWO_PHASE_METHOD_H
#define SIMPLEX_TWO_PHASE_METHOD_H

#include "macro.h"
#include "solver.h"
#include "tabular.h"

#define INFEASIBLE -1
#define UNBOUNDED -2
#define DEGENERATE -3
#define FEASIBLE 0

#ifdef __cplusplus
extern "C" {
#endif

int twoPhaseMethod(problem_t *problem, TYPE *solution, TYPE *optimalValue);

void enableBenchmarkMode(void);
void disableBenchmarkMode(void);

#ifdef __cplusplus
}
#endif
#endif
