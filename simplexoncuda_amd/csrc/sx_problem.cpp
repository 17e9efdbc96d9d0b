// sx_problem.cpp -- problem_t I/O and the random-instance generator of the C-ABI
// (replaces reference src/problem.cu:1-188 and src/generator.cu:1-77).
//
// Generator semantics (problem.cu:49-126, generator.cu:9-32):
//   srand(seed); sB = rand(); sC = rand(); sA = rand();          (host CRT rand)
//   b_i    = U(XORWOW(sB) draw #i),  c_j = U(XORWOW(sC) draw #j)
//   A(i,j) = U(XORWOW(sA) draw #(i*n + j))   -- one thread per constraint i does
//            curand_init(sA, 0, i*n) and n draws, so row-major A is one sequential stream
//   U(x)   = fma((double)fmaf((float)x, 2^-32, 2^-33), max - min, min)
// The XORWOW seeding and uniform mapping follow cuRAND's published curand_init /
// curand_uniform (not rocRAND's, whose seeding constants differ).  The CRT is MSVC's LCG
// by default: with it the generated instances reproduce the reference's published pivot
// counts exactly (tests/golden/published_pivots.json).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/problem.h"
#include "../../include/simplex_hip.h"

namespace {

struct Xorwow {
    uint32_t d, v[5];
    explicit Xorwow(uint64_t seed) {
        const uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
        const uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
        const uint32_t t0 = 1099087573u * s0;
        const uint32_t t1 = 2591861531u * s1;
        d = 6615241u + t1 + t0;
        v[0] = 123456789u + t0;
        v[1] = 362436069u ^ t0;
        v[2] = 521288629u + t1;
        v[3] = 88675123u ^ t1;
        v[4] = 5783321u + t0;
    }
    inline uint32_t next() {
        const uint32_t t = v[0] ^ (v[0] >> 2);
        v[0] = v[1];
        v[1] = v[2];
        v[2] = v[3];
        v[3] = v[4];
        v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
        d += 362437u;
        return v[4] + d;
    }
};

inline double draw_value(Xorwow &g, double lo, double span) {
    const float u = std::fmaf((float)g.next(), 2.3283064e-10f, 2.3283064e-10f / 2.0f);
    return std::fma((double)u, span, lo);
}

}  // namespace

// problem.cu:63-67: srand(seed); three rand() calls (MSVC LCG or glibc TYPE_3)
void sx_crt_seeds(unsigned seed, int kind, uint32_t out[3]) {
    if (kind == 0) {  // MSVC: holdrand = holdrand * 214013 + 2531011; (holdrand >> 16) & 0x7fff
        uint32_t h = seed;
        for (int k = 0; k < 3; ++k) {
            h = h * 214013u + 2531011u;
            out[k] = (h >> 16) & 0x7fffu;
        }
        return;
    }
    // glibc random(): TYPE_3 additive feedback generator, 310 discarded outputs
    int32_t r[34 + 310 + 3];
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        int64_t v = (16807LL * r[i - 1]) % 2147483647LL;
        if (v < 0) v += 2147483647LL;
        r[i] = (int32_t)v;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 34; i < 34 + 310 + 3; ++i) r[i] = (int32_t)((uint32_t)r[i - 31] + (uint32_t)r[i - 3]);
    for (int k = 0; k < 3; ++k) out[k] = ((uint32_t)r[344 + k]) >> 1;
}

namespace {

problem_t *malloc_problem(int n, int m) {  // problem.cu:7-18
    problem_t *p = (problem_t *)malloc(sizeof(problem_t));
    p->constraints = m;
    p->vars = n;
    p->objectiveFunction = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    p->constraintsMatrix = (double *)malloc(sizeof(double) * (size_t)n * (size_t)m + 1);
    p->knownTermsVector = (double *)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
    return p;
}

}  // namespace

extern "C" {

problem_t *simplex_generate_problem_ex(int n, int m, unsigned int seed, int lo, int hi, int rand_kind) {
    problem_t *p = malloc_problem(n, m);
    uint32_t sd[3];
    sx_crt_seeds(seed, rand_kind, sd);
    const double dlo = (double)lo, span = (double)hi - (double)lo;
    {
        Xorwow g(sd[0]);
        for (int i = 0; i < m; ++i) p->knownTermsVector[i] = draw_value(g, dlo, span);
    }
    {
        Xorwow g(sd[1]);
        for (int j = 0; j < n; ++j) p->objectiveFunction[j] = draw_value(g, dlo, span);
    }
    {
        Xorwow g(sd[2]);
        double *A = p->constraintsMatrix;
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < n; ++j) A[(size_t)j * m + i] = draw_value(g, dlo, span);
    }
    return p;
}

problem_t *generateRandomProblem(int nVars, int nConstraints, unsigned int seed, int minGenerator, int maxGenerator) {
    return simplex_generate_problem_ex(nVars, nConstraints, seed, minGenerator, maxGenerator, 0);
}

problem_t *readProblemFromFile(FILE *file) {  // problem.cu:20-47
    int n = 0, m = 0;
    if (fscanf(file, "%d %d", &n, &m) != 2) return nullptr;
    problem_t *p = malloc_problem(n, m);
    for (int j = 0; j < n; ++j)
        if (fscanf(file, "%lf", &p->objectiveFunction[j]) != 1) return p;
    for (int i = 0; i < m; ++i) {
        for (int j = 0; j < n; ++j)
            if (fscanf(file, "%lf", &p->constraintsMatrix[(size_t)j * m + i]) != 1) return p;
        if (fscanf(file, "%lf\n", &p->knownTermsVector[i]) != 1) return p;
    }
    return p;
}

problem_t *readRandomProblemFromFile(FILE *file) {  // problem.cu:128-139
    int n = 0, m = 0, lo = 0, hi = 0;
    unsigned int seed = 0;
    if (fscanf(file, "%d %d %u %d %d", &n, &m, &seed, &lo, &hi) != 5) return nullptr;
    return generateRandomProblem(n, m, seed, lo, hi);
}

void printProblemToStream(FILE *Stream, problem_t *problem) {  // problem.cu:141-181
    const int n = problem->vars, m = problem->constraints;
    fprintf(Stream, "max ");
    for (int j = 0; j < n; ++j) {
        const double v = problem->objectiveFunction[j];
        fprintf(Stream, v >= 0 ? "+ " : "- ");
        fprintf(Stream, "%.2lf X%d ", std::fabs(v), j + 1);
    }
    fprintf(Stream, "\nsubject to \n");
    for (int i = 0; i < m; ++i) {
        for (int j = 0; j < n; ++j) {
            const double v = problem->constraintsMatrix[(size_t)j * m + i];
            fprintf(Stream, v >= 0 ? "+ " : "- ");
            fprintf(Stream, "%.2lf X%d ", std::fabs(v), j + 1);
        }
        fprintf(Stream, "<= %.2lf\n", problem->knownTermsVector[i]);
    }
}

void freeProblem(problem_t *problem) {  // problem.cu:183-188 (the struct itself is the caller's)
    free(problem->constraintsMatrix);
    free(problem->knownTermsVector);
    free(problem->objectiveFunction);
}

problem_t *sx_malloc_problem(int n, int m) { return malloc_problem(n, m); }

problem_t *simplex_problem_from_arrays(int n, int m, const double *A_colmajor, const double *b, const double *c) {
    problem_t *p = malloc_problem(n, m);
    if (n > 0 && m > 0) std::memcpy(p->constraintsMatrix, A_colmajor, sizeof(double) * (size_t)n * m);
    if (m > 0) std::memcpy(p->knownTermsVector, b, sizeof(double) * m);
    if (n > 0) std::memcpy(p->objectiveFunction, c, sizeof(double) * n);
    return p;
}

void simplex_free_problem_struct(problem_t *problem) {
    if (!problem) return;
    freeProblem(problem);
    free(problem);
}

}  // extern "C"
