/* The oracle's float alpha (hlgs_oracle.c: expf, no contraction) vs the exact double alpha near 1/255. */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
static uint32_t st = 12345;
static float u01(void) { st = st * 1664525u + 1013904223u; return (st >> 8) * (1.0f / 16777216.0f); }
int main(void) {
    double worst = 0; long n = 0;
    for (long it = 0; it < 200000000L; it++) {
        float s1 = expf(-1.2f + 4.6f * u01()), s2 = expf(-1.2f + 4.6f * u01()), th = 3.1415926f * u01();
        float c = cosf(th), sn = sinf(th);
        float cxx = c * c * s1 * s1 + sn * sn * s2 * s2 + 0.3f, cyy = sn * sn * s1 * s1 + c * c * s2 * s2 + 0.3f;
        float cxy = c * sn * (s1 * s1 - s2 * s2), det = cxx * cyy - cxy * cxy, inv = 1.f / det;
        float a = cyy * inv, b = -cxy * inv, cc = cxx * inv, o = 0.01f + 0.98f * u01();
        float t = sqrtf(fmaxf(2.f * logf(255.f * o), 0.f)) * (0.98f + 0.04f * u01()), ang = 6.2831853f * u01();
        float ux = cosf(ang), uy = sinf(ang), qf = a * ux * ux + 2.f * b * ux * uy + cc * uy * uy, r = t / sqrtf(qf);
        float x = 100.f + 37.f * u01(), px = floorf(x + r * ux), y = 200.f + 41.f * u01(), py = floorf(y + r * uy);
        float dx = x - px, dy = y - py;
        float power = -0.5f * (a * dx * dx + cc * dy * dy) - b * dx * dy;
        float af = fminf(0.99f, o * expf(power));
        double pd = -0.5 * ((double)a * dx * dx + (double)cc * dy * dy) - (double)b * dx * dy;
        double ad = fmin(0.99, (double)o * exp(pd));
        if (ad > 1.0 / 255 * 0.5 && ad < 1.0 / 255 * 2) { double d = fabs(af / ad - 1.0); if (d > worst) worst = d; n++; }
    }
    printf("oracle float alpha vs exact: max relative deviation %.3e over %ld near-threshold samples\n", worst, n);
    return 0;
}
