// orbx_sincos.h — cos/sin of the BRIEF steering angle, shared by the gfx950 kernel and its host check.
//
// computeOrbDescriptor (reference src/ORBextractor.cc:112-113) takes a = cos(angle), b = sin(angle) of a
// float angle in radians; the build pins that to the correctly rounded float value, (float)cos((double)x)
// (the oracle calls libm's double cos/sin).  A generic double cos/sin costs ~150 FP64
// instructions per call on the GPU, so the kernel uses this short form instead: the angle is
// angle_deg * (pi/180) with angle_deg in [0, 360] (fastAtan2), i.e. x in [0, 6.2832], which needs only
// a two-constant Cody-Waite reduction by pi/2 (fdlibm's pio2_1 has 33 trailing zero bits, so x - n*pio2_1
// is exact for n <= 4) and fdlibm's minimax kernels on |r| <= pi/4 (error < 1 ulp in double).  Rounded
// to float, the result equals (float)cos((double)x) unless the double value lies within about an ulp of a
// float rounding boundary; tests/test_sincos.py checks EVERY float x in [0, 6.2832] against libm
// (oracle/sincos_check.c), so the two agree on the whole input domain of the kernel.
//
// Every operation is written out (explicit fma, no contraction) so host and device round identically.
#pragma once

#if defined(__HIPCC__)
#define ORBX_HD __host__ __device__ __forceinline__
#define ORBX_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define ORBX_RINT(a) __builtin_rint(a)
#else
#include <math.h>
#define ORBX_HD static inline
#define ORBX_FMA(a, b, c) fma((a), (b), (c))
#define ORBX_RINT(a) rint(a)
#endif

// x in [0, 8): *c = cos(x), *s = sin(x) to double accuracy, then rounded to float.
ORBX_HD void orbx_sincos_brief(float xf, float* c, float* s) {
    const double x = (double)xf;
    const double invpio2 = 6.36619772367581382433e-01;   // 2/pi
    const double pio2_1 = 1.57079632673412561417e+00;    // first 33 bits of pi/2
    const double pio2_1t = 6.07710050650619224932e-11;   // pi/2 - pio2_1
    const double fn = ORBX_RINT(x * invpio2);
    const int n = (int)fn;
    const double r = x - fn * pio2_1;                    // exact
    const double y = r - fn * pio2_1t;
    const double z = y * y;
    // fdlibm __kernel_sin (tail y = 0)
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double rs = ORBX_FMA(z, ORBX_FMA(z, ORBX_FMA(z, ORBX_FMA(z, S6, S5), S4), S3), S2);
    const double v = z * y;
    const double ks = y + v * ORBX_FMA(z, rs, S1);
    // fdlibm __kernel_cos (tail y = 0)
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double rc = z * ORBX_FMA(z, ORBX_FMA(z, ORBX_FMA(z, ORBX_FMA(z, ORBX_FMA(z, C6, C5), C4), C3), C2), C1);
    unsigned long long yb;
    const double ay = y < 0 ? -y : y;
    __builtin_memcpy(&yb, &ay, 8);
    const unsigned int ix = (unsigned int)(yb >> 32);    // high word of |y|
    double kc;
    if (ix < 0x3FD33333u) {                              // |y| < 0.3
        kc = 1.0 - (0.5 * z - z * rc);
    } else {
        double qx;
        if (ix > 0x3fe90000u) {                          // |y| > 0.78125
            qx = 0.28125;
        } else {                                         // |y|/4 with the low word cleared
            const unsigned long long qb = (unsigned long long)(ix - 0x00200000u) << 32;
            __builtin_memcpy(&qx, &qb, 8);
        }
        const double hz = 0.5 * z - qx;
        const double a = 1.0 - qx;
        kc = a - (hz - z * rc);
    }
    double cs, sn;
    switch (n & 3) {
        case 0: cs = kc; sn = ks; break;
        case 1: cs = -ks; sn = kc; break;
        case 2: cs = -kc; sn = -ks; break;
        default: cs = ks; sn = -kc; break;
    }
    *c = (float)cs;
    *s = (float)sn;
}
