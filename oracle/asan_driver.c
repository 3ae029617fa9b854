/*
 * asan_driver.c -- TEST INFRASTRUCTURE ONLY (SURVEY.md §5 sanitizer row).
 *
 * A standalone executable over rips_oracle.c, built with
 * -fsanitize=address,undefined (oracle/Makefile target asan_driver), so the
 * sanitizer runtime is the program's own: no LD_PRELOAD of the Python
 * interpreter.  Reads cases from stdin -- "n maxdim thresh" then n*n floats
 * (a square distance matrix) -- runs oracle_rips_dm on each and prints, per
 * dim, the emitted pair count, all-pair count and checksum, so
 * tests/test_oracle.py can compare them with the regular oracle build.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define OR_MAXDIM 3
typedef struct {
    int64_t n_pairs[OR_MAXDIM + 1];
    float *births[OR_MAXDIM + 1];
    float *deaths[OR_MAXDIM + 1];
    int64_t *birth_idx[OR_MAXDIM + 1];
    int64_t *death_idx[OR_MAXDIM + 1];
    int64_t n_all_pairs[OR_MAXDIM + 1];
    uint64_t checksum[OR_MAXDIM + 1];
    int64_t n_columns[OR_MAXDIM + 1];
    int64_t n_apparent[OR_MAXDIM + 1];
    int64_t n_adds[OR_MAXDIM + 1];
    int64_t max_heap[OR_MAXDIM + 1];
    int64_t max_live[OR_MAXDIM + 1];
    int64_t sum_live[OR_MAXDIM + 1];
    int64_t sum_heap_steps[OR_MAXDIM + 1];
    int64_t num_edges;
    float thresh;
} oracle_result;
int oracle_rips_dm(const float *dist, int64_t n, int maxdim, float thresh, oracle_result *res);
void oracle_free(oracle_result *r);

int main(void) {
    long n;
    int maxdim;
    double thresh;
    while (scanf("%ld %d %lf", &n, &maxdim, &thresh) == 3) {
        float *d = (float *)malloc(sizeof(float) * (size_t)(n * n > 0 ? n * n : 1));
        for (long i = 0; i < n * n; ++i)
            if (scanf("%f", &d[i]) != 1) return 2;
        oracle_result r;
        if (oracle_rips_dm(d, n, maxdim, isinf(thresh) ? INFINITY : (float)thresh, &r)) return 3;
        printf("edges %lld", (long long)r.num_edges);
        for (int k = 0; k <= maxdim; ++k)
            printf(" | %lld %lld %llu", (long long)r.n_pairs[k], (long long)r.n_all_pairs[k], (unsigned long long)r.checksum[k]);
        printf("\n");
        oracle_free(&r);
        free(d);
    }
    return 0;
}
