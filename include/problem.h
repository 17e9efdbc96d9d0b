/*
 * problem.h -- LP instance type and I/O (replaces reference include/problem.h:1-72).
 *
 * max c^T x  s.t.  A x <= b, x >= 0.  Byte-identical struct layout to problem.h:10-26:
 * constraintsMatrix is COLUMN-major, A(i,j) at [j*constraints + i] (problem.cu:41).
 * Ownership as in the reference: the library mallocs the arrays, freeProblem() frees the
 * three arrays (not the struct itself, problem.cu:183-188).
 */
#ifndef SIMPLEX_PROBLEM_H
#define SIMPLEX_PROBLEM_H

#include <stdio.h>
#include "macro.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    TYPE *constraintsMatrix; /* column-major m x n */
    TYPE *knownTermsVector;  /* b, length m */
    TYPE *objectiveFunction; /* c, length n */
    int vars;                /* n */
    int constraints;         /* m */
} problem_t;

/* problem.cu:20-47: "n m" / c[n] / m lines of "a_i1 .. a_in b_i" */
problem_t *readProblemFromFile(FILE *file);

/* problem.cu:128-139: "n m seed min max" */
problem_t *readRandomProblemFromFile(FILE *file);

/* problem.cu:49-126: srand(seed); seeds for b, c, A from rand(); cuRAND-XORWOW uniforms
 * scaled to [min, max].  The reference's C++ default arguments (min=-100, max=100,
 * problem.h:54) are kept for C++ callers. */
#ifdef __cplusplus
problem_t *generateRandomProblem(int nVars, int nConstraints, unsigned int seed, int minGenerator = -100,
                                 int maxGenerator = 100);
#else
problem_t *generateRandomProblem(int nVars, int nConstraints, unsigned int seed, int minGenerator,
                                 int maxGenerator);
#endif

/* problem.cu:141-181 */
void printProblemToStream(FILE *Stream, problem_t *problem);

/* problem.cu:183-188 */
void freeProblem(problem_t *problem);

#ifdef __cplusplus
}
#endif
#endif
