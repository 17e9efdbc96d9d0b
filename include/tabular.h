/*
 * tabular.h -- device tableau (replaces reference include/tabular.cuh:1-51).
 *
 * Field names are the reference's.  Their MEANING follows the reference's counting
 * convention, but the storage is the textbook orientation, row-major in HBM:
 *   rows  = tableau width N in the reference's sense (1 + n + 2m in phase 1, reduced by
 *           cols to 1 + n + m in phase 2, twoPhaseMethod.cu:288)
 *   cols  = m (number of constraints)
 *   table = m constraint rows of `rows` doubles each, row stride `pitch` BYTES;
 *           element (i, 0) is b_i, element (i, v+1) is variable v
 *   knownTermsVector = table (column 0 of every row, stride pitch)
 *   constraintsMatrix = table + 1 (variable columns)
 *   costsVector = device objective row d[0 .. rows)
 * No external caller touches the fields (only twoPhaseMethod does).
 */
#ifndef SIMPLEX_TABULAR_H
#define SIMPLEX_TABULAR_H

#include <stdio.h>
#include "problem.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    problem_t *problem;
    TYPE *table;
    TYPE *knownTermsVector;
    TYPE *constraintsMatrix;
    TYPE *costsVector;
    size_t pitch;
    int rows;
    int cols;
} tabular_t;

/* tabular.cu:25-39: allocates device memory for the phase-1 tableau (not filled) */
tabular_t *newTabular(problem_t *problem);

/* tabular.cu:41-98: prints in the reference's transposed orientation (one line per
 * tableau column: the m constraint entries, then the objective entry), then the base. */
void printTableauToStream(FILE *Stream, tabular_t *tabular, int *base);

/* tabular.cu:100-109 */
void freeTabular(tabular_t *tabular);

#ifdef __cplusplus
}
#endif
#endif
