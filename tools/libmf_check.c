/* libmf_check -- pins include/pbrt_libmf.h to the system libm (TEST INFRASTRUCTURE).
 *
 * The renderer's GPU core and CPU oracle evaluate the reference's float transcendentals with
 * the restatement in include/pbrt_libmf.h.  This program compares it with the C library the
 * reference itself calls (glibc 2.35, x86-64, FMA builds selected at run time):
 *   tables    every table / coefficient block of the header is found byte for byte in the
 *             loaded libm's data (glibc's own memory layout);
 *   unary     sinf cosf sincosf expf logf acosf atanf tanf: every one of the 2^32 float inputs
 *             (--stride S tests every S-th bit pattern instead);
 *   binary    powf, atan2f: N random bit patterns plus N structured pairs each (powf: base in
 *             [0, 1], exponents 0..1e4 as Blinn / microfacet lookups use; atan2f: directions).
 * NaN results compare equal whatever their bits.  Prints one line per function and exits 1
 * on any mismatch.
 *
 * Build: gcc -O2 -ffp-contract=off -I include tools/libmf_check.c -o tools/libmf_check -lm -lpthread -ldl
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pbrt_libmf.h"

static float (*volatile ref_sinf)(float) = sinf;
static float (*volatile ref_cosf)(float) = cosf;
static void (*volatile ref_sincosf)(float, float *, float *) = sincosf;
static float (*volatile ref_expf)(float) = expf;
static float (*volatile ref_logf)(float) = logf;
static float (*volatile ref_acosf)(float) = acosf;
static float (*volatile ref_atanf)(float) = atanf;
static float (*volatile ref_tanf)(float) = tanf;
static float (*volatile ref_powf)(float, float) = powf;
static float (*volatile ref_atan2f)(float, float) = atan2f;

static int same(float a, float b) {
    if (a != a && b != b) return 1;
    return libmf_asuint(a) == libmf_asuint(b);
}

enum { F_SIN, F_COS, F_SINCOS, F_EXP, F_LOG, F_ACOS, F_ATAN, F_TAN, F_POW, F_ATAN2, F_N };
static const char *NAMES[F_N] = { "sinf", "cosf", "sincosf", "expf", "logf", "acosf", "atanf", "tanf", "powf", "atan2f" };

typedef struct {
    int fn, tid, nthreads;
    uint64_t stride, nbin, bad, tested;
    uint32_t first_bad[2];
} job_t;

static uint64_t splitmix(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int check1(int fn, float x) {
    switch (fn) {
    case F_SIN: return same(libmf_sinf(x), ref_sinf(x));
    case F_COS: return same(libmf_cosf(x), ref_cosf(x));
    case F_SINCOS: {
        float s, c, rs, rc;
        libmf_sincosf(x, &s, &c);
        ref_sincosf(x, &rs, &rc);
        return same(s, rs) && same(c, rc) && same(s, ref_sinf(x)) && same(c, ref_cosf(x));
    }
    case F_EXP: return same(libmf_expf(x), ref_expf(x));
    case F_LOG: return same(libmf_logf(x), ref_logf(x));
    case F_ACOS: return same(libmf_acosf(x), ref_acosf(x));
    case F_ATAN: return same(libmf_atanf(x), ref_atanf(x));
    case F_TAN: return same(libmf_tanf(x), ref_tanf(x));
    }
    return 0;
}

static int check2(int fn, float a, float b) {
    if (fn == F_POW) return same(libmf_powf(a, b), ref_powf(a, b));
    return same(libmf_atan2f(a, b), ref_atan2f(a, b));
}

static void *run(void *arg) {
    job_t *j = (job_t *)arg;
    if (j->fn < F_POW) {
        const uint64_t total = 1ull << 32;
        for (uint64_t u = (uint64_t)j->tid * j->stride; u < total; u += (uint64_t)j->nthreads * j->stride) {
            float x = libmf_asfloat((uint32_t)u);
            j->tested++;
            if (!check1(j->fn, x)) {
                if (!j->bad) j->first_bad[0] = (uint32_t)u;
                j->bad++;
            }
        }
    } else {
        uint64_t s = 0x1234567ull + (uint64_t)j->tid * 0x9E3779B97F4A7C15ull + (uint64_t)j->fn;
        for (uint64_t i = j->tid; i < j->nbin; i += j->nthreads) {
            uint64_t r = splitmix(&s);
            float a = libmf_asfloat((uint32_t)r), b = libmf_asfloat((uint32_t)(r >> 32));
            float c, d;
            uint64_t r2 = splitmix(&s);
            if (j->fn == F_POW) {   /* base in [0, 1], exponent in [0, 1e4] and small integers */
                c = (float)((r2 & 0xffffff) * 0x1p-24);
                d = (i & 3) == 0 ? (float)((r2 >> 24) % 64) : (float)((r2 >> 24 & 0xffffff) * 0x1p-24) * 1.0e4f;
            } else {                /* direction components in [-1, 1], some exact zeros */
                c = (float)((int32_t)(r2 & 0xffffff) - 0x800000) * 0x1p-23f;
                d = (float)((int32_t)(r2 >> 24 & 0xffffff) - 0x800000) * 0x1p-23f;
                if ((i & 255) == 0) c = 0.0f;
            }
            j->tested += 2;
            if (!check2(j->fn, a, b)) {
                if (!j->bad) { j->first_bad[0] = libmf_asuint(a); j->first_bad[1] = libmf_asuint(b); }
                j->bad++;
            }
            if (!check2(j->fn, c, d)) {
                if (!j->bad) { j->first_bad[0] = libmf_asuint(c); j->first_bad[1] = libmf_asuint(d); }
                j->bad++;
            }
        }
    }
    return NULL;
}

/* find a byte block in the loaded libm's image */
static int in_libm(const void *blk, size_t n, const char *what) {
    Dl_info info;
    if (!dladdr((void *)ref_sinf, &info) || !info.dli_fname) { printf("tables: cannot locate libm\n"); return 0; }
    FILE *f = fopen(info.dli_fname, "rb");
    if (!f) { printf("tables: cannot read %s\n", info.dli_fname); return 0; }
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *buf = (unsigned char *)malloc((size_t)sz);
    size_t got = fread(buf, 1, (size_t)sz, f);
    fclose(f);
    int found = 0;
    for (size_t i = 0; i + n <= got && !found; i += 4) found = memcmp(buf + i, blk, n) == 0;
    free(buf);
    printf("table %-22s %s in %s\n", what, found ? "found" : "NOT FOUND", info.dli_fname);
    return found;
}

static int check_tables(void) {
    int ok = 1;
    for (int t = 0; t < 2; ++t) {   /* glibc 2.35's sincos_t order: sign, hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4 */
        const libmf_sincos_t *p = &libmf_sincosf_table[t];
        double g[14] = { p->sign[0], p->sign[1], p->sign[2], p->sign[3], p->hpi_inv, p->hpi, p->c0, p->c1, p->s1,
                         p->c2, p->s2, p->c3, p->s3, p->c4 };
        ok &= in_libm(g, sizeof g, t ? "sincosf_table[1]" : "sincosf_table[0]");
    }
    ok &= in_libm(libmf_inv_pio4, sizeof libmf_inv_pio4, "inv_pio4");
    {   /* __exp2f_data: tab, shift_scaled, poly, shift, invln2_scaled, poly_scaled */
        double rest[9] = { 0x1.8p+52 / 32, LIBMF_EXP2F_C0, LIBMF_EXP2F_C1, LIBMF_EXP2F_C2, 0x1.8p+52, LIBMF_EXPF_INVLN2N,
                           LIBMF_EXP2F_C0 / 32768.0, LIBMF_EXP2F_C1 / 1024.0, LIBMF_EXP2F_C2 / 32.0 };
        unsigned char blk[256 + sizeof rest];
        memcpy(blk, libmf_exp2f_tab, 256);
        memcpy(blk + 256, rest, sizeof rest);
        ok &= in_libm(blk, sizeof blk, "exp2f_data");
    }
    {
        double rest[4] = { LIBMF_LOGF_LN2, LIBMF_LOGF_A0, LIBMF_LOGF_A1, LIBMF_LOGF_A2 };
        unsigned char blk[256 + sizeof rest];
        memcpy(blk, libmf_logf_tab, 256);
        memcpy(blk + 256, rest, sizeof rest);
        ok &= in_libm(blk, sizeof blk, "logf_data");
    }
    {
        double rest[5] = { LIBMF_POWF_A0, LIBMF_POWF_A1, LIBMF_POWF_A2, LIBMF_POWF_A3, LIBMF_POWF_A4 };
        unsigned char blk[256 + sizeof rest];
        memcpy(blk, libmf_powf_log2_tab, 256);
        memcpy(blk + 256, rest, sizeof rest);
        ok &= in_libm(blk, sizeof blk, "powf_log2_data");
    }
    return ok;
}

int main(int argc, char **argv) {
    uint64_t stride = 1, nbin = 1ull << 26;
    int nthreads = 8, only = -1;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--stride")) stride = strtoull(argv[++i], NULL, 0);
        else if (!strcmp(argv[i], "--pairs")) nbin = strtoull(argv[++i], NULL, 0);
        else if (!strcmp(argv[i], "--threads")) nthreads = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--only")) {
            for (int f = 0; f < F_N; ++f)
                if (!strcmp(argv[i + 1], NAMES[f])) only = f;
            ++i;
        } else { fprintf(stderr, "usage: libmf_check [--stride S] [--pairs N] [--threads T] [--only fn]\n"); return 2; }
    }
    int fail = !check_tables();
    for (int fn = 0; fn < F_N; ++fn) {
        if (only >= 0 && fn != only) continue;
        job_t jobs[256];
        pthread_t th[256];
        if (nthreads > 256) nthreads = 256;
        for (int t = 0; t < nthreads; ++t) {
            memset(&jobs[t], 0, sizeof jobs[t]);
            jobs[t].fn = fn; jobs[t].tid = t; jobs[t].nthreads = nthreads; jobs[t].stride = stride; jobs[t].nbin = nbin;
            pthread_create(&th[t], NULL, run, &jobs[t]);
        }
        uint64_t bad = 0, tested = 0;
        uint32_t fb[2] = { 0, 0 };
        for (int t = 0; t < nthreads; ++t) {
            pthread_join(th[t], NULL);
            if (jobs[t].bad && !bad) { fb[0] = jobs[t].first_bad[0]; fb[1] = jobs[t].first_bad[1]; }
            bad += jobs[t].bad;
            tested += jobs[t].tested;
        }
        if (fn < F_POW)
            printf("%-8s %llu inputs, %llu differ%s", NAMES[fn], (unsigned long long)tested, (unsigned long long)bad,
                   bad ? "" : "\n");
        else
            printf("%-8s %llu pairs, %llu differ%s", NAMES[fn], (unsigned long long)tested, (unsigned long long)bad,
                   bad ? "" : "\n");
        if (bad) {
            float a = libmf_asfloat(fb[0]), b = libmf_asfloat(fb[1]);
            if (fn < F_POW) printf(" (first x = %a: %a vs libm)\n", a, 0.0);
            else printf(" (first (%a, %a))\n", a, b);
            fail = 1;
        }
        fflush(stdout);
    }
    return fail;
}
