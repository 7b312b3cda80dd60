/*
 * plssvm oracle — TEST INFRASTRUCTURE ONLY (see oracle.h): parity checker and CPU baseline
 * ("port") for the MI355X backend. Never linked into the product library.
 */
#include "oracle.h"

#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

#define REAL double
#define SUF f64
#define FMA fma
#define POW pow
#define EXP exp
#include "oracle_tmpl.h"
#undef REAL
#undef SUF
#undef FMA
#undef POW
#undef EXP

#define REAL float
#define SUF f32
#define FMA fmaf
#define POW powf
#define EXP expf
#include "oracle_tmpl.h"
#undef REAL
#undef SUF
#undef FMA
#undef POW
#undef EXP

/* ---- packed FP22 (build-defined, not in the reference) ---- */
static uint32_t f2u(float v) {
    uint32_t u;
    memcpy(&u, &v, 4);
    return u;
}

uint32_t orc_fp22_encode(float v) {
    const uint32_t u = f2u(v);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) {
        return ((u >> 10) | 0x1000u) & 0x3FFFFFu; /* NaN stays a (quiet) NaN */
    }
    const uint32_t lsb = (u >> 10) & 1u; /* round to nearest even on the 10 dropped bits */
    return ((u + 0x1FFu + lsb) >> 10) & 0x3FFFFFu;
}

float orc_fp22_decode(uint32_t code) {
    const uint32_t u = (code & 0x3FFFFFu) << 10;
    float v;
    memcpy(&v, &u, 4);
    return v;
}

int64_t orc_fp22_words(int64_t n) { return ((n + 15) / 16) * 11; }

void orc_fp22_pack(const float *v, int64_t n, uint32_t *words) {
    const int64_t nw = orc_fp22_words(n);
    memset(words, 0, sizeof(uint32_t) * (size_t) nw);
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t code = orc_fp22_encode(v[i]);
        const int64_t g = i / 16, k = i % 16;
        const int64_t bit = 22 * k, w = g * 11 + bit / 32, s = bit % 32;
        words[w] |= (uint32_t) (code << s);
        if (s + 22 > 32) words[w + 1] |= (uint32_t) (code >> (32 - s));
    }
}

void orc_fp22_unpack(const uint32_t *words, int64_t n, float *v) {
    for (int64_t i = 0; i < n; ++i) {
        const int64_t g = i / 16, k = i % 16;
        const int64_t bit = 22 * k, w = g * 11 + bit / 32, s = bit % 32;
        uint64_t x = words[w] >> s;
        if (s + 22 > 32) x |= (uint64_t) words[w + 1] << (32 - s);
        v[i] = orc_fp22_decode((uint32_t) (x & 0x3FFFFFu));
    }
}
