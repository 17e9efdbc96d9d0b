// sx_cli.cpp -- command-line front end over libsimplex_hip.so (replaces reference main.cu).
//
//   simplex_cli -f <file>            solve a problem file (problem.cu:20-47 format)
//   simplex_cli -r <n> <m> [seed]    random problem in [-100, 100] (main.cu:7-8, 135-139)
//   simplex_cli -rs <n> <m> [seed]   same, and save the seed file "n m seed min max"
//   simplex_cli -rf <seedfile>       regenerate a problem from a seed file (problem.cu:128-139)
//   simplex_cli -t                   the reference's benchmark sweep (main.cu:50-77): n, m in
//                                    256..8192, seed n*100+m (+1 at n=1024, m=8192), [1, 100]
// Messages, status handling and the solution file format follow main.cu:14-115.  Paths: the
// solution goes to $SIMPLEX_SOLUTION (default "solution.txt"), seed files and TIMER CSVs to
// $SIMPLEX_DATA_DIR (default "."); -t enables the TIMER CSV (benchmark_<n>_<m>.txt) there.
// Extension options before the mode:
//   --gpus N              N GPUs (devices 0..N-1) for the solve, as SIMPLEX_GPUS=N
//   --pivot-budget K      at most K pivots per phase (twoPhaseMethodEx; off = parity mode)
//   --rand msvc|glibc     the CRT rand() of the generator's seeds (default msvc: the published
//                         pivot counts were produced by MSVC builds)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>

#include "../../include/problem.h"
#include "../../include/simplex_hip.h"
#include "../../include/twoPhaseMethod.h"

static const int MIN_V = -100;
static const int MAX_V = +100;

static std::string data_dir() {
    const char *e = getenv("SIMPLEX_DATA_DIR");
    return e ? e : ".";
}

static int g_rand_kind = 0;             // --rand: 0 MSVC, 1 glibc
static long long g_pivot_budget = -1;   // --pivot-budget

static problem_t *generate(int vars, int constraints, unsigned seed, int lo, int hi) {
    return g_rand_kind ? simplex_generate_problem_ex(vars, constraints, seed, lo, hi, g_rand_kind)
                       : generateRandomProblem(vars, constraints, seed, lo, hi);
}

static problem_t *random_input(int vars, int constraints, int seed) {
    printf("Generating random problem with %d variables, %d contraints with seed: %d\n", vars, constraints, seed);
    return generate(vars, constraints, (unsigned)seed, MIN_V, MAX_V);
}

// twoPhaseMethod, or twoPhaseMethodEx under a pivot budget.  Returns FEASIBLE / INFEASIBLE /
// UNBOUNDED / DEGENERATE, or SIMPLEX_PIVOT_CAP under a budget; every other engine outcome is
// fatal, as twoPhaseMethod itself makes it (error.cu:5-12 convention: message, exit non-zero).
static int solve_problem(problem_t *p, double *solution, double *optimalValue) {
    if (g_pivot_budget < 0) return twoPhaseMethod(p, solution, optimalValue);
    long long piv[2] = {0, 0};
    const int st = twoPhaseMethodEx(p, solution, optimalValue, nullptr, piv, g_pivot_budget);
    switch (st) {
    case FEASIBLE:
    case INFEASIBLE:
    case UNBOUNDED:
    case DEGENERATE:
        return st;
    case SIMPLEX_PIVOT_CAP:
        printf("\nPivot budget of %lld reached (phase pivots %lld + %lld)\n", g_pivot_budget, piv[0], piv[1]);
        return st;
    case SIMPLEX_NUMERIC_FAIL:
        fprintf(stderr, "simplex: the ratio test found no leaving row although a pivot is eligible\n");
        break;
    case SIMPLEX_HANG:
        fprintf(stderr, "simplex: a fused-batch hand-off between GPUs timed out\n");
        break;
    default:
        fprintf(stderr, "simplex: unexpected solver status %d\n", st);
        break;
    }
    exit(EXIT_FAILURE);
}

static void save_random_input(int vars, int constraints, int seed) {
    time_t timer = time(nullptr);
    char ts[20];
    strftime(ts, sizeof(ts), "%Y%m%d%H%M", localtime(&timer));
    std::string name = data_dir() + "/random_" + ts + ".txt";
    FILE *f = openFile(name.c_str(), "w");
    fprintf(f, "%d %d %d %d %d", vars, constraints, seed, MIN_V, MAX_V);
    fclose(f);
}

int main(int argc, const char *argv[]) {
    printf("Starting...\n");
    // extension options, then the reference's arguments
    while (argc > 2 && strncmp(argv[1], "--", 2) == 0) {
        if (strcmp(argv[1], "--gpus") == 0) {
            const int n = atoi(argv[2]);
            if (n < 1 || n > SIMPLEX_MAX_GPUS) {
                fprintf(stderr, "--gpus: expected 1..%d GPUs, got %s\n", SIMPLEX_MAX_GPUS, argv[2]);
                exit(-1);
            }
            int devs[SIMPLEX_MAX_GPUS];
            for (int k = 0; k < n; ++k) devs[k] = k;
            simplex_set_gpus(devs, n);
        } else if (strcmp(argv[1], "--pivot-budget") == 0) {
            g_pivot_budget = atoll(argv[2]);
        } else if (strcmp(argv[1], "--rand") == 0) {
            if (strcmp(argv[2], "msvc") == 0) {
                g_rand_kind = 0;
            } else if (strcmp(argv[2], "glibc") == 0) {
                g_rand_kind = 1;
            } else {
                fprintf(stderr, "--rand: expected msvc or glibc\n");
                exit(-1);
            }
        } else {
            fprintf(stderr, "Unknown option %s\n", argv[1]);
            exit(-1);
        }
        argc -= 2;
        argv += 2;
    }
    if (argc < 2) {
        fprintf(stderr, "Not enough arguments!\n");
        exit(-1);
    }
    if (getenv("SIMPLEX_VERBOSE")) simplex_set_verbose(1);
    problem_t *problem = nullptr;
    if (strcmp(argv[1], "-f") == 0 && argc > 2) {
        printf("Reading problem from file...\n");
        FILE *file = openFile(argv[2], "r");
        problem = readProblemFromFile(file);
        fclose(file);
    } else if (strcmp(argv[1], "-r") == 0 && argc > 3) {
        problem = random_input(atoi(argv[2]), atoi(argv[3]), argc > 4 ? atoi(argv[4]) : (int)time(nullptr));
    } else if (strcmp(argv[1], "-rs") == 0 && argc > 3) {
        const int seed = argc > 4 ? atoi(argv[4]) : (int)time(nullptr);
        problem = random_input(atoi(argv[2]), atoi(argv[3]), seed);
        save_random_input(atoi(argv[2]), atoi(argv[3]), seed);
    } else if (strcmp(argv[1], "-rf") == 0 && argc > 2) {
        printf("Reading seed from file\n");
        FILE *file = openFile(argv[2], "r");
        if (g_rand_kind) {  // (the seed file "n m seed min max", problem.cu:128-139, under --rand glibc)
            int n = 0, m = 0, seed = 0, lo = 0, hi = 0;
            if (fscanf(file, "%d %d %d %d %d", &n, &m, &seed, &lo, &hi) == 5) problem = generate(n, m, (unsigned)seed, lo, hi);
        } else {
            problem = readRandomProblemFromFile(file);
        }
        fclose(file);
    } else if (strcmp(argv[1], "-t") == 0) {
        enableBenchmarkMode();
        simplex_set_timer_dir(data_dir().c_str());
        fprintf(stderr, "Running a benchmark (max 8192*8192)... \n\n\n");
        const int max_side = argc > 2 ? atoi(argv[2]) : 8192;  // extension: cap the sweep
        const time_t start = time(nullptr);
        for (int constraints = 256; constraints <= max_side; constraints *= 2) {
            for (int vars = 256; vars <= max_side; vars *= 2) {
                fprintf(stdout, "\nCurrent matrix: %d*%d\n\n", vars, constraints);
                const int seed = vars * 100 + constraints + (vars == 1024 && constraints == 8192 ? 1 : 0);
                problem_t *p = generate(vars, constraints, (unsigned)seed, +1, +100);
                double *solution = (double *)malloc(sizeof(double) * p->vars);
                double optimalValue = 0;
                solve_problem(p, solution, &optimalValue);
                freeProblem(p);
                free(p);
                free(solution);
            }
        }
        const time_t end = time(nullptr);
        fprintf(stdout, "Benchmark terminato...\n Sono stati necessari %.3lfs", (double)(end - start));
        return 0;
    } else {
        fprintf(stderr, "Not enough arguments!\n");
        exit(-1);
    }
    if (problem == nullptr) {
        fprintf(stderr, "Cannot read the problem!\n");
        exit(-1);
    }
    double *solution = (double *)malloc(sizeof(double) * (problem->vars > 0 ? problem->vars : 1));
    double optimalValue = 0;
    const char *sol_path = getenv("SIMPLEX_SOLUTION") ? getenv("SIMPLEX_SOLUTION") : "solution.txt";
    FILE *fileSolution = openFile(sol_path, "w");
    printf("Resolving....\n");
    switch (solve_problem(problem, solution, &optimalValue)) {
    case INFEASIBLE:
        printf("\nProblem INFEASIBLE!\n");
        break;
    case UNBOUNDED:
        printf("\nProblem UNBOUNDED!\n");
        break;
    case DEGENERATE:
        printf("\nProblem DEGENERATE!\n");
        break;
    case SIMPLEX_PIVOT_CAP:  // (no solution: the phase did not finish)
        break;
    case FEASIBLE:
        printf("\nProblem solved!\n");
        for (int i = 0; i < problem->vars; i++) fprintf(fileSolution, "%lf\n", solution[i]);
        fprintf(fileSolution, "\nOptimal value: %lf\n", optimalValue);
    }
    fclose(fileSolution);
    free(solution);
    freeProblem(problem);
    free(problem);
    return 0;
}
