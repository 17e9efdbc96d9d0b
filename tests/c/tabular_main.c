/* A caller of the inner entry point, as twoPhaseMethod.cu:225-356 uses it: newTabular
 * (tabular.cu:25-39) -> fill the device tableau and costs vector -> solve (solver.cu:128-149)
 * -> read back -> freeTabular.  The layout is the one include/tabular.h documents: m rows of
 * `rows` doubles at `pitch` bytes, column 0 = b, column v+1 = variable v.
 * usage: tabular_main <in.bin> <out.bin>
 *   in.bin : int32 n, m, W; T (m x W doubles, row-major); d (W doubles); base (m int32).
 *            W = 1+n+2m (phase 1) or 1+n+m (phase 2: the caller shrinks rows by cols,
 *            twoPhaseMethod.cu:288, before calling solve)
 *   out.bin: int32 status, rows, cols; int64 pitch; T (m x W); d (W); base (m) after solve */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>

#include "problem.h"
#include "solver.h"
#include "tabular.h"

#define CHECK(x)                                                       \
    do {                                                               \
        if ((x) != hipSuccess) {                                       \
            fprintf(stderr, "HIP error at %s:%d\n", __FILE__, __LINE__); \
            return 4;                                                  \
        }                                                              \
    } while (0)

static int read_all(FILE *f, void *p, size_t bytes) { return fread(p, 1, bytes, f) == bytes; }

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    int hdr[3];
    if (!read_all(f, hdr, sizeof(hdr))) return 2;
    const int n = hdr[0], m = hdr[1], W = hdr[2];
    double *T = (double *)malloc(sizeof(double) * (size_t)m * W);
    double *d = (double *)malloc(sizeof(double) * W);
    int *base = (int *)malloc(sizeof(int) * m);
    if (!read_all(f, T, sizeof(double) * (size_t)m * W) || !read_all(f, d, sizeof(double) * W) ||
        !read_all(f, base, sizeof(int) * m))
        return 2;
    fclose(f);

    problem_t P = {0};  /* newTabular reads the sizes only */
    P.vars = n;
    P.constraints = m;
    tabular_t *t = newTabular(&P);
    if (t->rows != 1 + n + 2 * m || t->cols != m || t->pitch < sizeof(double) * (size_t)t->rows ||
        t->knownTermsVector != t->table || t->constraintsMatrix != t->table + 1) {
        fprintf(stderr, "tabular_t fields: rows %d cols %d pitch %zu\n", t->rows, t->cols, t->pitch);
        return 5;
    }
    t->rows = W;  /* phase 2: rows -= cols */
    CHECK(hipMemcpy2D(t->table, t->pitch, T, sizeof(double) * W, sizeof(double) * W, m, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(t->costsVector, d, sizeof(double) * W, hipMemcpyHostToDevice));
    const int st = solve(t, base);
    CHECK(hipMemcpy2D(T, sizeof(double) * W, t->table, t->pitch, sizeof(double) * W, m, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(d, t->costsVector, sizeof(double) * W, hipMemcpyDeviceToHost));
    FILE *dn = fopen("/dev/null", "w");
    printTableauToStream(dn, t, base);  /* tabular.cu:87-98 */
    fclose(dn);

    FILE *o = fopen(argv[2], "wb");
    if (!o) return 2;
    const int oh[3] = {st, t->rows, t->cols};
    const long long pitch = (long long)t->pitch;
    fwrite(oh, sizeof(oh), 1, o);
    fwrite(&pitch, sizeof(pitch), 1, o);
    fwrite(T, sizeof(double), (size_t)m * W, o);
    fwrite(d, sizeof(double), W, o);
    fwrite(base, sizeof(int), m, o);
    fclose(o);
    freeTabular(t);
    free(T);
    free(d);
    free(base);
    return 0;
}
