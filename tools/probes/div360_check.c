/* Exhaustive check (every f32 a in [0, 12960]) that the reciprocal-and-correction division
   used for the orientation bin, q = a*y; r = fma(-q, 360, a); q + r*y with y = RN(1/360),
   gives the same bin rint(a / 360) as the IEEE division (mismatches only for subnormal
   quotients, all bin 0).  gcc -O2 -ffp-contract=off div360_check.c -lm; ~40 s.
   With 360 -> 255 and the range [0, 256] (localize's DoG / 255): 0 mismatches. */
#include <stdio.h>
#include <math.h>
#include <string.h>
#include <stdint.h>
int main(void) {
    const float y = 1.0f / 360.0f;
    uint32_t lo, hi; float a0 = 0.0f, a1 = 12960.0f;
    memcpy(&lo, &a0, 4); memcpy(&hi, &a1, 4);
    long bad = 0, badbin = 0;
    for (uint32_t u = lo; u <= hi; ++u) {
        float a; memcpy(&a, &u, 4);
        volatile float ref = a / 360.0f;
        float q = a * y;
        float r = fmaf(-q, 360.0f, a);
        float qd = fmaf(r, y, q);
        if (qd != ref) { if (bad < 5) printf("a=%a ref=%a got=%a\n", a, ref, qd); ++bad;
            if ((int)rintf(qd) != (int)rintf(ref)) ++badbin; }
    }
    printf("mismatches %ld (bin-changing %ld)\n", bad, badbin);
    return 0;
}
