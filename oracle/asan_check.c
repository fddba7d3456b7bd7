/* oracle/asan_check.c -- AddressSanitizer / UBSan driver of the C oracle (TEST INFRASTRUCTURE
 * ONLY; SURVEY.md §5 "Race detection / sanitizers": an ASan build of the CPU restatement).
 *
 * Built by `make -C oracle asan` with -fsanitize=address,undefined into oracle/_asan/ and run by
 * tests/test_oracle_asan.py.  Every entry point of dsp_oracle.h runs on edge-case inputs (empty,
 * 1-sample, shorter than a frame, exactly one frame, 1 s, 1.5 s, silence, DC, clipping) for several
 * (L, S) and the three reference windows, VAD on and off; the threaded batch entry must equal the
 * per-clip one, and the KNN runs at D = 15 / 40, k = 3 / 5 / 21, with and without self exclusion.
 * Exit status 0 and no sanitizer report = clean.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dsp_oracle.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static double urand(void)
{
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(rng_state >> 11) * (1.0 / 9007199254740992.0);
}

static void make_clip(int16_t *x, int64_t n, int kind)
{
    for (int64_t i = 0; i < n; i++) {
        double v = (urand() - 0.5) * 200.0;
        if (kind == 1) v = 0.0;                                    /* silence */
        if (kind == 2) v = 1000.0;                                 /* constant DC */
        if (kind == 3) v = (i & 64) ? 32767.0 : -32768.0;          /* full-scale square */
        if (kind == 0 && i > n / 4 && i < n / 2) v += 8000.0 * sin(0.05 * (double)i);
        if (v > 32767.0) v = 32767.0;
        if (v < -32768.0) v = -32768.0;
        x[i] = (int16_t)v;
    }
}

static void make_window(double *w, int64_t L, int type)
{
    for (int64_t j = 0; j < L; j++) {
        const double c = L > 1 ? cos(M_PI * (double)(2 * j - (L - 1)) / (double)(L - 1)) : 1.0;
        w[j] = type == 0 ? 1.0 : type == 1 ? 0.54 + 0.46 * c : 0.5 + 0.5 * c;
    }
    if (type == 2 && L > 1) w[0] = w[L - 1] = 0.0;
}

static int check_clips(void)
{
    static const int64_t lens[] = {0, 1, 5, 255, 256, 257, 1101, 1102, 1103, 5000, 44100, 66150};
    static const int64_t LS[][2] = {{1102, 441}, {1024, 512}, {256, 100}, {2205, 441}, {1, 1}};
    const int nlen = (int)(sizeof(lens) / sizeof(lens[0]));
    int64_t total = 0;
    for (int i = 0; i < nlen; i++) total += lens[i];
    int16_t *pcm = (int16_t *)malloc(sizeof(int16_t) * (size_t)(total + 1));
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nlen + 1));
    off[0] = 0;
    for (int i = 0; i < nlen; i++) {
        make_clip(pcm + off[i], lens[i], i % 4);
        off[i + 1] = off[i] + lens[i];
    }
    int bad = 0;
    for (int c = 0; c < (int)(sizeof(LS) / sizeof(LS[0])); c++) {
        const int64_t L = LS[c][0], S = LS[c][1];
        double *w = (double *)malloc(sizeof(double) * (size_t)L);
        for (int wt = 0; wt < 3; wt++) {
            make_window(w, L, wt);
            for (int vad = 0; vad < 2; vad++) {
                double *feat = (double *)malloc(sizeof(double) * 15 * (size_t)nlen);
                int64_t *se = (int64_t *)malloc(sizeof(int64_t) * 2 * (size_t)nlen);
                int64_t *nf = (int64_t *)malloc(sizeof(int64_t) * (size_t)nlen);
                int32_t *st = (int32_t *)malloc(sizeof(int32_t) * (size_t)nlen);
                ora_process_batch_i16(pcm, off, nlen, L, S, w, vad, 0.5, 0.1, 1.5, feat, se, nf, st, 4);
                for (int i = 0; i < nlen; i++) {
                    const int64_t n = lens[i];
                    const int64_t nv = ora_vad_frame_count(n, L, S), F = ora_frame_count(n, L, S);
                    double *ve = (double *)malloc(sizeof(double) * (size_t)(nv > 0 ? nv : 1));
                    double *vz = (double *)malloc(sizeof(double) * (size_t)(nv > 0 ? nv : 1));
                    double *seq = (double *)malloc(sizeof(double) * 3 * (size_t)(F > 0 ? F : 1));
                    double f1[15];
                    int64_t se1[2], nf1 = 0, nv1 = 0;
                    const int rc = ora_process_pcm_i16(pcm + off[i], n, L, S, w, vad, 0.5, 0.1, 1.5, f1, se1, &nf1,
                                                       ve, vz, &nv1, seq, F);
                    if (rc != st[i]) bad++;
                    if (rc == ORA_OK) {
                        if (se1[0] != se[2 * i] || se1[1] != se[2 * i + 1] || nf1 != nf[i]) bad++;
                        if (memcmp(f1, feat + 15 * i, sizeof(f1)) != 0) bad++;
                    }
                    free(ve);
                    free(vz);
                    free(seq);
                }
                free(feat);
                free(se);
                free(nf);
                free(st);
            }
        }
        free(w);
    }
    free(pcm);
    free(off);
    return bad;
}

static int check_knn(void)
{
    static const int dims[] = {15, 40};
    static const int ks[] = {3, 5, 21};
    int bad = 0;
    for (int di = 0; di < 2; di++)
        for (int ki = 0; ki < 3; ki++) {
            const int D = dims[di], k = ks[ki];
            const int64_t Nr = 300, Nq = 50;
            double *ref = (double *)malloc(sizeof(double) * (size_t)(Nr * D));
            int32_t *lbl = (int32_t *)malloc(sizeof(int32_t) * (size_t)Nr);
            for (int64_t i = 0; i < Nr * D; i++) ref[i] = urand() * 2.0 - 1.0;
            for (int64_t i = 0; i < Nr; i++) lbl[i] = (int32_t)(i % 7);
            double *mean = (double *)malloc(sizeof(double) * (size_t)D), *sd = (double *)malloc(sizeof(double) * (size_t)D);
            ora_zscore_fit(ref, Nr, D, mean, sd);
            int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)(Nq * k));
            double *dist = (double *)malloc(sizeof(double) * (size_t)(Nq * k));
            int32_t *pred = (int32_t *)malloc(sizeof(int32_t) * (size_t)Nq);
            for (int self = 0; self < 2; self++) {
                /* self-query: queries are reference rows 100 .. 149 */
                ora_knn(ref, lbl, Nr, ref + 100 * D, Nq, D, k, self ? 100 : -1, 7, idx, dist, pred);
                for (int64_t q = 0; q < Nq; q++) {
                    for (int j = 0; j < k; j++) {
                        if (idx[q * k + j] < 0 || idx[q * k + j] >= Nr) bad++;
                        if (self && idx[q * k + j] == 100 + q) bad++;
                        if (j && dist[q * k + j] < dist[q * k + j - 1]) bad++;
                    }
                    if (!self && dist[q * k] != 0.0) bad++;
                    if (pred[q] < 0 || pred[q] >= 7) bad++;
                }
            }
            free(ref);
            free(lbl);
            free(mean);
            free(sd);
            free(idx);
            free(dist);
            free(pred);
        }
    return bad;
}

int main(void)
{
    const int a = check_clips(), b = check_knn();
    printf("asan_check: clip mismatches %d, knn violations %d\n", a, b);
    return (a || b) ? 1 : 0;
}
