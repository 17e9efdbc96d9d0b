/*
 * macro.h -- shared definitions of the C-ABI (replaces reference include/macro.h:1-52).
 *
 * TYPE is fixed to double (macro.h:6).  compare() is the reference's epsilon comparison
 * (macro.h:28-42) and is THE semantics of every simplex decision; the HIP kernels use the
 * same expression.  Host-only here: no __host__/__device__ qualifiers leak into the C-ABI.
 * In C++ the reference's default arguments are kept; C callers pass all three arguments.
 */
#ifndef SIMPLEX_MACRO_H
#define SIMPLEX_MACRO_H

#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#define TYPE double
#define TYPE_SIZE sizeof(TYPE)
#define BYTE_SIZE(count) ((size_t)(count) * TYPE_SIZE)
#define SIMPLEX_EPSILON 1e-9

#ifdef __cplusplus
static inline int compare(double x, double y = 0.0, double epsilon = SIMPLEX_EPSILON)
#else
static inline int compare(double x, double y, double epsilon)
#endif
{
    if (fabs(x - y) < epsilon) return 0;
    if (x < y) return -1;
    return 1;
}

/* macro.h:44-53: open or die with "Cannot open file!" and exit(-1) */
static inline FILE *openFile(const char *path, const char *mode) {
    FILE *file = fopen(path, mode);
    if (file == NULL) {
        fprintf(stderr, "Cannot open file!\n");
        exit(-1);
    }
    return file;
}

#endif
