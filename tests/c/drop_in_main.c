/* A reference-style C caller (main.cu:14-115 flow) linked against libsimplex_hip.so.
 * usage: drop_in_main host            -- generator + print only (no GPU)
 *        drop_in_main solve <file>    -- readProblemFromFile + twoPhaseMethod */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "problem.h"
#include "solver.h"
#include "tabular.h"
#include "twoPhaseMethod.h"

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "host") == 0) {
        problem_t *p = generateRandomProblem(4, 3, 2010, 1, 100);
        printProblemToStream(stdout, p);
        printf("compare(1e-10)=%d compare(-1)=%d\n", compare(1e-10, 0.0, 1e-9), compare(-1.0, 0.0, 1e-9));
        freeProblem(p);
        free(p);
        return 0;
    }
    if (argc > 2 && strcmp(argv[1], "solve") == 0) {
        FILE *f = openFile(argv[2], "r");
        problem_t *p = readProblemFromFile(f);
        fclose(f);
        double *x = (double *)malloc(sizeof(double) * p->vars);
        double z = 0.0;
        enableBenchmarkMode();
        int st = twoPhaseMethod(p, x, &z);
        disableBenchmarkMode();
        printf("status %d z %.6f x0 %.6f\n", st, z, x[0]);
        free(x);
        freeProblem(p);
        free(p);
        return st == FEASIBLE ? 0 : 3;
    }
    return 2;
}
