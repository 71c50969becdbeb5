/* sincos_check.c — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
 *
 * Exhaustive check of the kernel's BRIEF-angle cos/sin (multiagent_orb_slam2_amd/csrc/orbx_sincos.h)
 * against the oracle's definition, (float)cos((double)x) / (float)sin((double)x) with libm
 * (oracle/orb_oracle.cpp computeOrbDescriptor, reference src/ORBextractor.cc:112-113), for EVERY float x
 * in [0, hi] (default hi = 6.2832f > 360 * (float)(pi/180), the largest steering angle fastAtan2 can give).
 *
 * usage: sincos_check [threads] [hi]   -> prints "checked N mismatches M" (+ the first mismatches), exit 0
 * iff M == 0.  Built by oracle/Makefile with the oracle's FP pins (no contraction, no fast-math).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../multiagent_orb_slam2_amd/csrc/orbx_sincos.h"

typedef struct {
    uint32_t b0, b1;
    unsigned long long mism;
    uint32_t first[4];
    int nfirst;
} Job;

static float f_of(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }

static void* run(void* p) {
    Job* j = (Job*)p;
    for (uint32_t b = j->b0; b < j->b1; ++b) {
        const float x = f_of(b);
        float c, s;
        orbx_sincos_brief(x, &c, &s);
        const float rc = (float)cos((double)x), rs = (float)sin((double)x);
        if (memcmp(&c, &rc, 4) != 0 || memcmp(&s, &rs, 4) != 0) {
            if (j->nfirst < 4) j->first[j->nfirst++] = b;
            j->mism++;
        }
    }
    return NULL;
}

int main(int argc, char** argv) {
    int nt = argc > 1 ? atoi(argv[1]) : 8;
    const float hi = argc > 2 ? (float)atof(argv[2]) : 6.2832f;
    if (nt < 1) nt = 1;
    if (nt > 64) nt = 64;
    uint32_t bhi;
    memcpy(&bhi, &hi, 4);
    const uint32_t total = bhi + 1;   /* every non-negative float up to hi, +0 included */
    pthread_t th[64];
    Job jobs[64];
    for (int t = 0; t < nt; ++t) {
        jobs[t].b0 = (uint32_t)((unsigned long long)total * t / nt);
        jobs[t].b1 = (uint32_t)((unsigned long long)total * (t + 1) / nt);
        jobs[t].mism = 0;
        jobs[t].nfirst = 0;
        pthread_create(&th[t], NULL, run, &jobs[t]);
    }
    unsigned long long mism = 0;
    for (int t = 0; t < nt; ++t) {
        pthread_join(th[t], NULL);
        mism += jobs[t].mism;
        for (int k = 0; k < jobs[t].nfirst; ++k) {
            const float x = f_of(jobs[t].first[k]);
            float c, s;
            orbx_sincos_brief(x, &c, &s);
            printf("mismatch x=%.9g: cos %.9g vs %.9g, sin %.9g vs %.9g\n", x, c, (float)cos((double)x), s,
                   (float)sin((double)x));
        }
    }
    printf("checked %u mismatches %llu\n", total, mism);
    return mism == 0 ? 0 : 1;
}
