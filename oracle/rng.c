/*
 * rng.c -- TEST INFRASTRUCTURE ONLY.  Random-number restatements used by the oracle and the fixtures:
 * Philox4x32-10 (Random123 algorithm; the engine's production noise stream), std::seed_seq,
 * std::mt19937_64, libstdc++ normal_distribution<double> and the store's quantize().
 * Compiled WITHOUT fp contraction or unsafe-math so the libstdc++ restatements are bit-exact
 * (checked against g++-generated fixtures in tests/golden/).
 */
#include "gcs_oracle.h"

#include <math.h>
#include <stdint.h>

/* ------------------------------------------------------------------------------------------------ */
/* random numbers                                                                                   */

void gcso_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0;
        c1 = n1;
        c2 = n2;
        c3 = n3;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

/* The engine's production noise: counter (particle, step_lo, step_hi, 'GCS1'), key (seed_lo, seed_hi);
 * u = ((r >> 8) + 0.5) 2^-24 (exact in fp32 and fp64); Box-Muller on (u0,u1) -> x, y and (u2,u3) -> z. */
void gcso_philox_normals(uint64_t seed, int64_t step, int64_t n, double* out)
{
    const double two_pi = 6.283185307179586476925286766559;
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int64_t i = 0; i < n; i++) {
        uint32_t ctr[4] = {(uint32_t)i, (uint32_t)step, (uint32_t)((uint64_t)step >> 32), 0x47435331u};
        uint32_t r[4];
        gcso_philox4x32_10(ctr, key, r);
        double u[4];
        for (int k = 0; k < 4; k++) u[k] = ((double)(r[k] >> 8) + 0.5) * (1.0 / 16777216.0);
        double rad1 = sqrt(-2.0 * log(u[0])), rad2 = sqrt(-2.0 * log(u[2]));
        out[3 * i + 0] = rad1 * cos(two_pi * u[1]);
        out[3 * i + 1] = rad1 * sin(two_pi * u[1]);
        out[3 * i + 2] = rad2 * cos(two_pi * u[3]);
    }
}

/* std::seed_seq::generate ([rand.util.seedseq]); used by stage_prepare/prepare.cpp:549-562 */
void gcso_seed_seq_generate(const uint32_t* v, int64_t s, uint32_t* b, int64_t n)
{
    if (n == 0) return;
    for (int64_t i = 0; i < n; i++) b[i] = 0x8b8b8b8bu;
    int64_t t = (n >= 623) ? 11 : (n >= 68) ? 7 : (n >= 39) ? 5 : (n >= 7) ? 3 : (n - 1) / 2;
    int64_t p = (n - t) / 2, q = p + t;
    int64_t m = (s + 1 > n) ? s + 1 : n;
    for (int64_t k = 0; k < m; k++) {
        uint32_t x = b[k % n] ^ b[(k + p) % n] ^ b[(k + n - 1) % n];
        uint32_t r1 = 1664525u * (x ^ (x >> 27));
        uint32_t r2 = r1;
        if (k == 0)
            r2 += (uint32_t)s;
        else if (k <= s)
            r2 += (uint32_t)(k % n) + v[k - 1];
        else
            r2 += (uint32_t)(k % n);
        b[(k + p) % n] += r1;
        b[(k + q) % n] += r2;
        b[k % n] = r2;
    }
    for (int64_t k = m; k < m + n; k++) {
        uint32_t x = b[k % n] + b[(k + p) % n] + b[(k + n - 1) % n];
        uint32_t r3 = 1566083941u * (x ^ (x >> 27));
        uint32_t r4 = r3 - (uint32_t)(k % n);
        b[(k + p) % n] ^= r3;
        b[(k + q) % n] ^= r4;
        b[k % n] = r4;
    }
}

void gcso_mt19937_64_seed(gcso_mt19937_64* g, uint64_t seed)
{
    g->mt[0] = seed;
    for (int i = 1; i < 312; i++) g->mt[i] = 6364136223846793005ULL * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
    g->index = 312;
}

uint64_t gcso_mt19937_64_next(gcso_mt19937_64* g)
{
    if (g->index >= 312) {
        for (int i = 0; i < 312; i++) {
            uint64_t x = (g->mt[i] & 0xFFFFFFFF80000000ULL) | (g->mt[(i + 1) % 312] & 0x7FFFFFFFULL);
            uint64_t xa = x >> 1;
            if (x & 1) xa ^= 0xB5026F5AA96619E9ULL;
            g->mt[i] = g->mt[(i + 156) % 312] ^ xa;
        }
        g->index = 0;
    }
    uint64_t y = g->mt[g->index++];
    y ^= (y >> 29) & 0x5555555555555555ULL;
    y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
    y ^= (y << 37) & 0xFFF7EEE000000000ULL;
    y ^= y >> 43;
    return y;
}

/* libstdc++ generate_canonical<double, 53>(mt19937_64): one 64-bit draw, u64 -> double (round to
 * nearest), / 2^64, clamped below 1 (/usr/include/c++/11/bits/random.tcc:3348-3380). */
static double canonical(gcso_mt19937_64* g)
{
    double r = (double)gcso_mt19937_64_next(g) / 18446744073709551616.0;
    if (r >= 1.0) r = nextafter(1.0, 0.0);
    return r;
}

/* libstdc++ normal_distribution<double> (Marsaglia polar, random.tcc:1795-1830); mean 0, stddev 1 */
void gcso_reference_normals(uint64_t seed, int64_t count, double* out)
{
    gcso_mt19937_64 g;
    gcso_mt19937_64_seed(&g, seed);
    int saved_available = 0;
    double saved = 0;
    for (int64_t c = 0; c < count; c++) {
        if (saved_available) {
            saved_available = 0;
            out[c] = saved;
            continue;
        }
        double x, y, r2;
        do {
            x = 2.0 * canonical(&g) - 1.0;
            y = 2.0 * canonical(&g) - 1.0;
            r2 = x * x + y * y;
        } while (r2 > 1.0 || r2 == 0.0);
        double mult = sqrt(-2 * log(r2) / r2);
        saved = x * mult;
        saved_available = 1;
        out[c] = y * mult;
    }
}

/* simulation_store.cpp:22-33 (binary mantissa quantisation before the f32 HDF5 write) */
double gcso_quantize(double value, int bits)
{
    int ex;
    double mant = frexp(value, &ex);
    double scaled = nearbyint(ldexp(mant, bits));
    return ldexp(scaled, ex - bits);
}
