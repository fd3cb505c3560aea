/* ORACLE — test infrastructure only (never linked into the product).
 *
 * CPU restatement of numpy's legacy RandomState integer sampling, the
 * generator behind rltoolkit's replay sampling:
 *   idx = np.random.randint(0, len, B)   rltoolkit/buffer/replay_buffer.py:234, :418
 * Third-party algorithm (numpy 1.18 pinned by the reference, 2.2.6 here; the
 * legacy stream is frozen by numpy's compatibility policy):
 *   seeding   np.random.seed(s), 0 <= s < 2^32  -> MT19937 init_genrand(s)
 *   randint   rng = high-1-low; rng == 0 -> low, no draw; else
 *             mask = 2^ceil(log2(rng+1))-1, draw 32-bit words, keep (w & mask) <= rng
 *             (numpy random_bounded_uint64_fill, use_masked=1, rng <= 0xFFFFFFFF)
 * Pinned by tests/golden/mt19937_randint.npz.
 */
#include <stdint.h>

typedef struct { uint32_t mt[624]; int mti; } oracle_mt;

void oracle_mt_seed(oracle_mt *s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = 624;
}

static void regen(oracle_mt *s) {
    for (int k = 0; k < 624; k++) {
        uint32_t y = (s->mt[k] & 0x80000000u) | (s->mt[(k + 1) % 624] & 0x7fffffffu);
        s->mt[k] = s->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    s->mti = 0;
}

uint32_t oracle_mt_next32(oracle_mt *s) {
    if (s->mti >= 624) regen(s);
    uint32_t y = s->mt[s->mti++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* np.random.randint(0, high, n) for 1 <= high <= 2^32 */
void oracle_mt_randint(oracle_mt *s, int64_t high, int64_t n, int64_t *out) {
    uint64_t rng = (uint64_t)(high - 1);
    if (rng == 0) {
        for (int64_t i = 0; i < n; i++) out[i] = 0;
        return;
    }
    uint64_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16;
    for (int64_t i = 0; i < n; i++) {
        uint32_t v;
        do { v = oracle_mt_next32(s) & (uint32_t)mask; } while (v > rng);
        out[i] = (int64_t)v;
    }
}

int oracle_mt_state_size(void) { return (int)sizeof(oracle_mt); }
