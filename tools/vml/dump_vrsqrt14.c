// Dumps this CPU's VRSQRT14 approximation (AVX-512F) as the 2 x 2^15-entry table the scheduler's
// host-independent sqrt restatement reads (weatherconverter_amd/diffusion_model/scheduler/vml_sqrt.py).
// VRSQRT14's result depends only on the input's exponent parity and its top 15 mantissa bits (the one
// exception: exact powers of four, whose root is exact) -- checked here over every significand of both
// parities and every normal exponent before the table is written; the program fails otherwise.
// Build and run on the reference host (the one tests/golden/make_golden.py ran on):
//   gcc -O2 -mavx512f tools/vml/dump_vrsqrt14.c -o /tmp/dump_vrsqrt14 && /tmp/dump_vrsqrt14 out.bin
// Output: 65536 little-endian uint16, entry (parity * 32768 + top15) = bits 22..7 of the significand
// of VRSQRT14(x) for x in [0.25, 1) (parity 0: [0.25, 0.5), parity 1: [0.5, 1)); the result's exponent
// is the one of 1 / sqrt(x) (checked too).
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float fr(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ur(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint32_t rs(uint32_t u) { return ur(_mm_cvtss_f32(_mm_rsqrt14_ss(_mm_setzero_ps(), _mm_set_ss(fr(u))))); }

int main(int argc, char** argv) {
    if (argc != 2) { fprintf(stderr, "usage: %s out.bin\n", argv[0]); return 2; }
    static uint16_t tab[65536];
    long bad = 0;
    for (uint32_t idx = 0; idx < 65536; ++idx) {
        const uint32_t par = idx >> 15, top = idx & 0x7fff;
        const uint32_t base = ((par ? 126u : 125u) << 23) | (top << 8);  // [0.25, 0.5) / [0.5, 1)
        const uint32_t v0 = rs(base | (top == 0 && par == 0 ? 1u : 0u));
        if (v0 & 0x7f) bad++;  // the low 7 significand bits are always zero
        tab[idx] = (uint16_t)((v0 >> 7) & 0xffff);
        for (uint32_t lo = 0; lo < 256; ++lo) {
            const uint32_t u = base | lo;
            const uint32_t v = rs(u);
            if (top == 0 && par == 0 && lo == 0) {  // 0.25: exact 2
                if (v != 0x40000000u) bad++;
                continue;
            }
            if ((v >> 7 & 0xffff) != tab[idx]) bad++;
            // every other even exponent: the same significand, the exponent of the exact root's
            for (int e = 1; e < 254; ++e) {
                if ((e & 1) != (int)((u >> 23) & 1)) continue;
                const uint32_t w = ((uint32_t)e << 23) | (u & 0x7fffff);
                const uint32_t vw = rs(w);
                const int ew = (int)(vw >> 23) - 127, eu = (int)(v >> 23) - 127;
                if ((vw & 0x7fffff) != (v & 0x7fffff) || ew - eu != -(e - (int)((u >> 23) & 0xff)) / 2) bad++;
            }
        }
    }
    if (bad) { fprintf(stderr, "VRSQRT14 is not a function of (parity, top 15 bits) here: %ld exceptions\n", bad); return 1; }
    FILE* f = fopen(argv[1], "wb");
    if (!f || fwrite(tab, 2, 65536, f) != 65536) return 1;
    fclose(f);
    printf("ok: 65536 entries, checked over every significand and normal exponent\n");
    return 0;
}
