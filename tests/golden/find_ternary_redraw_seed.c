/* Finds a Blake2xbPRNG seed {s, 2, 3, 4, 5, 6, 7, 8} whose first 4096 32-bit words (the draws of
 * sample_poly_ternary at n = 2^12) contain a zero word, which libstdc++'s uniform_int_distribution
 * redraws (tests/golden/ternary_redraw_seed.json; used by tests/test_sample.py).  Links the oracle:
 *   gcc -O2 -fopenmp find_ternary_redraw_seed.c -L../../oracle -loracle -o /tmp/find && /tmp/find */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

void or_prng_bytes(const uint64_t seed[8], size_t count, uint8_t *out);

int main(void)
{
    long found = -1;
#pragma omp parallel for schedule(dynamic, 256)
    for (long s = 1; s < 40000000; s++)
    {
        if (found >= 0) continue;
        uint64_t seed[8] = { (uint64_t)s, 2, 3, 4, 5, 6, 7, 8 };
        uint32_t w[4096];
        or_prng_bytes(seed, sizeof(w), (uint8_t *)w);
        for (int i = 0; i < 4096; i++)
            if (w[i] == 0)
            {
#pragma omp critical
                if (found < 0 || s < found) found = s;
                break;
            }
    }
    printf("{\"seed0\": %ld, \"log_n\": 12}\n", found);
    return found < 0;
}
