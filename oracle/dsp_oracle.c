/*
 * oracle/dsp_oracle.c -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the *checker*: it is linked only by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
 * product path (dsp-audioreclabs_amd/csrc/ HIP sources) never calls it.
 *
 * Parity status: PINNED.  Every function below reproduces the float64
 * arithmetic of the reference (Hypersonic-cpu/DSP-AudioRecLabs, numpy 2.2.6 /
 * scikit-learn 1.7.2 as installed in the survey container) operation for
 * operation, including numpy's summation order, and is checked bit-for-bit
 * against golden vectors produced by importing the reference's own src/
 * modules (tests/golden/make_golden.py -> tests/golden/ fixtures,
 * tests/test_oracle_golden.py).
 *
 * Arithmetic facts restated here (verified empirically):
 *  - np.sum / np.mean of a contiguous 1-D float64 array = sequential sum over
 *    8192-element buffer chunks, each chunk reduced by numpy's pairwise_sum
 *    (8 interleaved accumulators for n <= 128, recursive halving at
 *    multiples of 8 above, plain loop for n < 8).
 *  - np.mean/np.std along axis 0 of a C-contiguous 2-D array are plain
 *    sequential row sums.
 *  - np.percentile(q=90, method='linear'): virtual index (n-1)*0.9, numpy's
 *    _lerp (b - d*(1-g) when g >= 0.5, a + d*g otherwise).
 *  - sklearn KDTree euclidean distances: sequential d += t*t, no FMA, sqrt.
 *
 * Build: make -C oracle  (gcc -O2 -ffp-contract=off; never -ffast-math).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dsp_oracle.h"

/* ------------------------------------------------------------------------ */
/* per-thread LIFO scratch arena: no malloc/free (and no page faults) per clip */
/* ------------------------------------------------------------------------ */
static __thread char *tl_buf;
static __thread size_t tl_cap, tl_top;

/* called by public entry points before any allocation; grows only when idle */
static void ws_reserve(size_t bytes)
{
    if (tl_top == 0 && bytes > tl_cap) {
        free(tl_buf);
        tl_buf = (char *)malloc(bytes);
        tl_cap = bytes;
    }
}
static size_t ws_round(size_t bytes) { return (bytes + 63) & ~(size_t)63; }
static double *ws_alloc(size_t n_doubles)
{
    size_t b = ws_round(n_doubles * sizeof(double) + 8);
    if (tl_top + b > tl_cap) abort(); /* reservation bug */
    double *p = (double *)(tl_buf + tl_top);
    tl_top += b;
    return p;
}
static void ws_free(size_t n_doubles) { tl_top -= ws_round(n_doubles * sizeof(double) + 8); }
/* a worker thread's arena dies with it (found by the ASan build, oracle/asan_check.c) */
static void ws_release(void)
{
    free(tl_buf);
    tl_buf = NULL;
    tl_cap = tl_top = 0;
}
static size_t ws_bound(int64_t n, int64_t L, int64_t S)
{
    int64_t nf = n / (S > 0 ? S : 1) + 4;
    return (size_t)(2 * n + 8 * nf + 4 * L + 64) * sizeof(double) + 64 * 64;
}

/* ------------------------------------------------------------------------ */
/* numpy float64 summation                                                  */
/* ------------------------------------------------------------------------ */

/* numpy/_core/src/umath/loops_utils.h.src: DOUBLE_pairwise_sum */
static double pairwise_block(const double *a, int64_t n)
{
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_block(a, n2) + pairwise_block(a + n2, n - n2);
    }
}

/* np.add.reduce over a contiguous 1-D float64 array (buffered in 8192 chunks) */
double ora_np_sum(const double *a, int64_t n)
{
    double r = 0.0;
    for (int64_t i = 0; i < n; i += 8192) {
        int64_t m = n - i < 8192 ? n - i : 8192;
        r += pairwise_block(a + i, m);
    }
    return r;
}

static int cmp_double(const void *pa, const void *pb)
{
    double a = *(const double *)pa, b = *(const double *)pb;
    return (a > b) - (a < b);
}

/* src/feature_extraction.py:46-62 compute_statistics -> mean, std, max, min, median */
void ora_compute_statistics(const double *seq, int64_t n, double out[5])
{
    ws_reserve(ws_bound(n, 1, 1));
    size_t tn = (size_t)(n > 0 ? n : 1);
    double *tmp = ws_alloc(tn);
    double mean = ora_np_sum(seq, n) / (double)n;
    for (int64_t i = 0; i < n; i++) {
        double d = seq[i] - mean;
        tmp[i] = d * d;
    }
    double var = ora_np_sum(tmp, n) / (double)n;
    double mx = seq[0], mn = seq[0];
    for (int64_t i = 1; i < n; i++) {
        if (seq[i] > mx) mx = seq[i];
        if (seq[i] < mn) mn = seq[i];
    }
    memcpy(tmp, seq, sizeof(double) * (size_t)n);
    qsort(tmp, (size_t)n, sizeof(double), cmp_double);
    double med;
    if (n % 2) {
        med = tmp[n / 2];
    } else {
        double two[2] = {tmp[n / 2 - 1], tmp[n / 2]};
        med = ora_np_sum(two, 2) / 2.0; /* np.mean of the two middle values */
    }
    out[0] = mean;
    out[1] = sqrt(var);
    out[2] = mx;
    out[3] = mn;
    out[4] = med;
    ws_free(tn);
}

/* ------------------------------------------------------------------------ */
/* src/audio_processing.py                                                  */
/* ------------------------------------------------------------------------ */

/* :49-90 remove_dc + normalize_audio.  out may alias x. */
int ora_preprocess(const double *x, int64_t n, double *out)
{
    if (n <= 0) return ORA_ERR_EMPTY; /* np.max of an empty array raises */
    double m = ora_np_sum(x, n) / (double)n;
    double mx = 0.0;
    for (int64_t i = 0; i < n; i++) {
        out[i] = x[i] - m;
        double a = fabs(out[i]);
        if (a > mx) mx = a;
    }
    if (mx > 0.0)
        for (int64_t i = 0; i < n; i++) out[i] = out[i] / mx;
    return ORA_OK;
}

/* :93-103 np.sum(frame ** 2) */
double ora_short_time_energy(const double *frame, int64_t L, double *scratch)
{
    for (int64_t j = 0; j < L; j++) scratch[j] = frame[j] * frame[j];
    return ora_np_sum(scratch, L);
}

/* :106-116 np.sum(np.abs(frame)) */
double ora_short_time_magnitude(const double *frame, int64_t L, double *scratch)
{
    for (int64_t j = 0; j < L; j++) scratch[j] = fabs(frame[j]);
    return ora_np_sum(scratch, L);
}

/* :119-132 sign (0 -> -1), sum |diff| / 2 == number of sign changes */
double ora_zero_crossing_rate(const double *frame, int64_t L)
{
    int64_t c = 0;
    for (int64_t j = 0; j + 1 < L; j++) c += ((frame[j] > 0.0) != (frame[j + 1] > 0.0));
    return (double)c;
}

/* numpy percentile, method='linear' (numpy/lib/_function_base_impl.py _quantile/_lerp) */
static double np_percentile(const double *v, int64_t n, double q, double *scratch)
{
    memcpy(scratch, v, sizeof(double) * (size_t)n);
    qsort(scratch, (size_t)n, sizeof(double), cmp_double);
    double qq = q / 100.0;
    double vi = (double)(n - 1) * qq;
    double a, b, g;
    if (vi >= (double)(n - 1)) {
        a = b = scratch[n - 1];
        g = vi + 1.0; /* previous index forced to -1 */
    } else {
        double prev = floor(vi);
        int64_t pi = (int64_t)prev;
        a = scratch[pi];
        b = scratch[pi + 1];
        g = vi - prev;
    }
    double d = b - a;
    if (g >= 0.5) return b - d * (1.0 - g);
    return a + d * g;
}

/* :188-195 / :239-245: mean of the first and last noise_frames values, else min */
static double noise_level(const double *v, int64_t n, int64_t nf, double *scratch)
{
    if (nf > 0) {
        memcpy(scratch, v, sizeof(double) * (size_t)nf);
        memcpy(scratch + nf, v + n - nf, sizeof(double) * (size_t)nf);
        return ora_np_sum(scratch, 2 * nf) / (double)(2 * nf);
    }
    double m = v[0];
    for (int64_t i = 1; i < n; i++)
        if (v[i] < m) m = v[i];
    return m;
}

int64_t ora_vad_frame_count(int64_t n, int64_t L, int64_t S)
{
    if (n < L) return 0;
    return (n - L) / S + 1;
}

/* :135-275 endpoint_detection.  E, Z need ora_vad_frame_count() slots.
 * Returns the number of VAD frames (0 when n < L). */
int64_t ora_endpoint_detection(const double *x, int64_t n, int64_t L, int64_t S,
                               double hi, double lo, double zr,
                               int64_t *start, int64_t *end, double *E, double *Z)
{
    if (n < L) { /* :162-163 */
        *start = 0;
        *end = n;
        return 0;
    }
    int64_t nfr = (n - L) / S + 1; /* :166 */
    ws_reserve(ws_bound(n, L, S));
    size_t sn = (size_t)(L > nfr ? L : nfr);
    double *scratch = ws_alloc(sn);
    for (int64_t f = 0; f < nfr; f++) { /* :172-181 */
        E[f] = ora_short_time_energy(x + f * S, L, scratch);
        Z[f] = ora_zero_crossing_rate(x + f * S, L);
    }
    int64_t noise_frames = nfr / 10 < 5 ? nfr / 10 : 5; /* :188 */
    double noise_e = noise_level(E, nfr, noise_frames, scratch);
    double speech_e = np_percentile(E, nfr, 90.0, scratch); /* :198 */
    double t1 = speech_e * hi;                               /* :202 */
    int64_t n3 = -1, n4 = -1;
    for (int64_t f = 0; f < nfr; f++)
        if (E[f] > t1) {
            if (n3 < 0) n3 = f;
            n4 = f;
        }
    if (n3 < 0) { /* :207-209 */
        *start = 0;
        *end = n;
        ws_free(sn);
        return nfr;
    }
    double t2 = noise_e + (speech_e - noise_e) * lo; /* :217 */
    int64_t n2 = 0, n5 = nfr - 1;
    for (int64_t i = n3 - 1; i >= 0; i--)
        if (E[i] <= t2) { n2 = i + 1; break; }
    for (int64_t i = n4 + 1; i < nfr; i++)
        if (E[i] <= t2) { n5 = i - 1; break; }
    double noise_z = noise_level(Z, nfr, noise_frames, scratch);
    double tz = noise_z * zr; /* :247 */
    int64_t n1 = 0, n6 = nfr - 1;
    for (int64_t i = n2 - 1; i >= 0; i--)
        if (Z[i] <= tz) { n1 = i + 1; break; }
    for (int64_t i = n5 + 1; i < nfr; i++)
        if (Z[i] <= tz) { n6 = i - 1; break; }
    *start = n1 * S;                                  /* :272 */
    *end = n6 * S + L < n ? n6 * S + L : n;           /* :273 */
    ws_free(sn);
    return nfr;
}

/* :299-333 frame_signal: number of frames for a segment of n samples */
int64_t ora_frame_count(int64_t n, int64_t L, int64_t S)
{
    if (n <= 0) return 0;
    int64_t f = 0, st = 0;
    for (;;) {
        f++;
        if (st + L >= n) break;
        st += S;
    }
    return f;
}

/* frame_signal + extract_frame_features (src/feature_extraction.py:12-43)
 * without materialising the [F, L] frame matrix. */
int64_t ora_frame_features(const double *x, int64_t n, int64_t L, int64_t S,
                           const double *window, double *E, double *M, double *Z)
{
    int64_t F = ora_frame_count(n, L, S);
    ws_reserve(ws_bound(n, L, S));
    double *fr = ws_alloc((size_t)L);
    double *scratch = ws_alloc((size_t)L);
    for (int64_t f = 0; f < F; f++) {
        int64_t st = f * S;
        for (int64_t j = 0; j < L; j++) {
            double v = (st + j < n) ? x[st + j] : 0.0; /* np.pad constant 0 */
            fr[j] = v * window[j];
        }
        E[f] = ora_short_time_energy(fr, L, scratch);
        M[f] = ora_short_time_magnitude(fr, L, scratch);
        Z[f] = ora_zero_crossing_rate(fr, L);
    }
    ws_free((size_t)L);
    ws_free((size_t)L);
    return F;
}

/* ------------------------------------------------------------------------ */
/* whole-clip pipeline: process_audio_file (:336-396) + extract_features_   */
/* from_frames(method='statistical') (src/feature_extraction.py:91-112)     */
/* on int PCM already decoded by load_wav (:9-46).                          */
/* ------------------------------------------------------------------------ */

static int process_double(double *x, int64_t n, int64_t L, int64_t S, const double *window,
                          int do_vad, double hi, double lo, double zr, double *feat15,
                          int64_t *start_end, int64_t *n_frames, double *vad_e, double *vad_z,
                          int64_t *n_vad, double *seq, int64_t seq_cap)
{
    int rc = ora_preprocess(x, n, x);
    if (rc) return rc;
    int64_t st = 0, en = n, nv = 0;
    if (do_vad) {
        int64_t cap = ora_vad_frame_count(n, L, S);
        double *e = vad_e, *z = vad_z;
        double *te = NULL;
        size_t tn = (size_t)(2 * (cap > 0 ? cap : 1));
        if (!e || !z) {
            te = ws_alloc(tn);
            e = te;
            z = te + (cap > 0 ? cap : 1);
        }
        nv = ora_endpoint_detection(x, n, L, S, hi, lo, zr, &st, &en, e, z);
        if (te) ws_free(tn);
    }
    if (start_end) {
        start_end[0] = st;
        start_end[1] = en;
    }
    if (n_vad) *n_vad = nv;
    int64_t m = en - st;
    if (m <= 0) return ORA_ERR_NO_AUDIO; /* :388-389 */
    int64_t F = ora_frame_count(m, L, S);
    if (n_frames) *n_frames = F;
    if (F == 0) return ORA_ERR_NO_FRAMES;
    double *buf = ws_alloc((size_t)(3 * F));
    double *E = buf, *M = buf + F, *Z = buf + 2 * F;
    ora_frame_features(x + st, m, L, S, window, E, M, Z);
    if (feat15) {
        ora_compute_statistics(E, F, feat15 + 0);
        ora_compute_statistics(M, F, feat15 + 5);
        ora_compute_statistics(Z, F, feat15 + 10);
    }
    if (seq) {
        for (int64_t f = 0; f < F && f < seq_cap; f++) {
            seq[3 * f + 0] = E[f];
            seq[3 * f + 1] = M[f];
            seq[3 * f + 2] = Z[f];
        }
    }
    ws_free((size_t)(3 * F));
    return ORA_OK;
}

int ora_process_pcm_i16(const int16_t *pcm, int64_t n, int64_t L, int64_t S, const double *window,
                        int do_vad, double hi, double lo, double zr, double *feat15,
                        int64_t *start_end, int64_t *n_frames, double *vad_e, double *vad_z,
                        int64_t *n_vad, double *seq, int64_t seq_cap)
{
    if (L <= 0 || S <= 0) return ORA_ERR_ARGS;
    ws_reserve(ws_bound(n, L, S));
    size_t xn = (size_t)(n > 0 ? n : 1);
    double *x = ws_alloc(xn);
    for (int64_t i = 0; i < n; i++) x[i] = pcm[i] / 32768.0; /* load_wav :35-38 */
    int rc = process_double(x, n, L, S, window, do_vad, hi, lo, zr, feat15, start_end, n_frames,
                            vad_e, vad_z, n_vad, seq, seq_cap);
    ws_free(xn);
    return rc;
}

int ora_process_f64(const double *audio, int64_t n, int64_t L, int64_t S, const double *window,
                    int do_vad, double hi, double lo, double zr, double *feat15,
                    int64_t *start_end, int64_t *n_frames, double *vad_e, double *vad_z,
                    int64_t *n_vad, double *seq, int64_t seq_cap)
{
    if (L <= 0 || S <= 0) return ORA_ERR_ARGS;
    ws_reserve(ws_bound(n, L, S));
    size_t xn = (size_t)(n > 0 ? n : 1);
    double *x = ws_alloc(xn);
    memcpy(x, audio, sizeof(double) * (size_t)n);
    int rc = process_double(x, n, L, S, window, do_vad, hi, lo, zr, feat15, start_end, n_frames,
                            vad_e, vad_z, n_vad, seq, seq_cap);
    ws_free(xn);
    return rc;
}

/* ---- batched driver (CPU baseline timing): clips are independent -------- */
typedef struct {
    const int16_t *pcm;
    const int64_t *offsets;
    int64_t b0, b1, L, S;
    const double *window;
    int do_vad;
    double hi, lo, zr;
    double *feat;
    int64_t *start_end, *n_frames;
    int32_t *status;
    int own_thread; /* runs on a thread of its own: release the arena at the end */
} batch_job;

static void *batch_worker(void *arg)
{
    batch_job *j = (batch_job *)arg;
    for (int64_t b = j->b0; b < j->b1; b++) {
        int64_t o = j->offsets[b], n = j->offsets[b + 1] - o;
        int rc = ora_process_pcm_i16(j->pcm + o, n, j->L, j->S, j->window, j->do_vad, j->hi, j->lo,
                                     j->zr, j->feat + 15 * b, j->start_end + 2 * b,
                                     j->n_frames + b, NULL, NULL, NULL, NULL, 0);
        j->status[b] = rc;
    }
    if (j->own_thread) ws_release();
    return NULL;
}

int ora_process_batch_i16(const int16_t *pcm, const int64_t *offsets, int64_t B, int64_t L,
                          int64_t S, const double *window, int do_vad, double hi, double lo,
                          double zr, double *feat, int64_t *start_end, int64_t *n_frames,
                          int32_t *status, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > B) nthreads = (int)(B > 0 ? B : 1);

    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    batch_job *jobs = (batch_job *)malloc(sizeof(batch_job) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) {
        batch_job j = {pcm, offsets, B * t / nthreads, B * (t + 1) / nthreads, L, S, window,
                       do_vad, hi, lo, zr, feat, start_end, n_frames, status, nthreads > 1};
        jobs[t] = j;
        if (nthreads == 1)
            batch_worker(&jobs[t]);
        else
            pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* src/feature_extraction.py:157-181 normalize_features (axis-0 stats)      */
/* ------------------------------------------------------------------------ */
void ora_zscore_fit(const double *X, int64_t n, int d, double *mean, double *std)
{
    for (int c = 0; c < d; c++) mean[c] = 0.0;
    for (int64_t i = 0; i < n; i++)
        for (int c = 0; c < d; c++) mean[c] += X[i * d + c];
    for (int c = 0; c < d; c++) mean[c] = mean[c] / (double)n;
    for (int c = 0; c < d; c++) std[c] = 0.0;
    for (int64_t i = 0; i < n; i++)
        for (int c = 0; c < d; c++) {
            double t = X[i * d + c] - mean[c];
            std[c] += t * t;
        }
    for (int c = 0; c < d; c++) std[c] = sqrt(std[c] / (double)n);
}

/* ------------------------------------------------------------------------ */
/* KNN: KNeighborsClassifier(n_neighbors=k) brute-force restatement         */
/* (src/models.py:33-35,52-58 -> sklearn KDTree exact k-NN + scipy mode)    */
/* Distances: sequential fp64 sum of squared differences, sqrt.  Exact-     */
/* distance ties are ordered by smaller reference index (sklearn's kd_tree  */
/* tie order is traversal-dependent: parity unpinned for exact ties).       */
/* ------------------------------------------------------------------------ */
typedef struct {
    double d;
    int64_t i;
} cand;

static int cand_less(cand a, cand b) { return a.d < b.d || (a.d == b.d && a.i < b.i); }

void ora_knn(const double *ref, const int32_t *ref_lbl, int64_t Nr, const double *q, int64_t Nq,
             int D, int k, int64_t self_offset, int n_classes, int32_t *idx, double *dist,
             int32_t *pred)
{
    cand *best = (cand *)malloc(sizeof(cand) * (size_t)(k + 1));
    int *cnt = (int *)malloc(sizeof(int) * (size_t)(n_classes > 0 ? n_classes : 1));
    for (int64_t qi = 0; qi < Nq; qi++) {
        int nb = 0;
        const double *x = q + qi * D;
        for (int64_t r = 0; r < Nr; r++) {
            if (self_offset >= 0 && r == self_offset + qi) continue;
            const double *y = ref + r * D;
            double acc = 0.0;
            for (int c = 0; c < D; c++) {
                double t = x[c] - y[c];
                acc += t * t;
            }
            cand cd = {acc, r};
            if (nb < k) {
                int p = nb++;
                while (p > 0 && cand_less(cd, best[p - 1])) { best[p] = best[p - 1]; p--; }
                best[p] = cd;
            } else if (cand_less(cd, best[k - 1])) {
                int p = k - 1;
                while (p > 0 && cand_less(cd, best[p - 1])) { best[p] = best[p - 1]; p--; }
                best[p] = cd;
            }
        }
        for (int j = 0; j < k; j++) {
            idx[qi * k + j] = j < nb ? (int32_t)best[j].i : -1;
            dist[qi * k + j] = j < nb ? sqrt(best[j].d) : INFINITY;
        }
        if (pred && ref_lbl && n_classes > 0) {
            memset(cnt, 0, sizeof(int) * (size_t)n_classes);
            for (int j = 0; j < nb; j++) cnt[ref_lbl[best[j].i]]++;
            int bl = 0;
            for (int c = 1; c < n_classes; c++)
                if (cnt[c] > cnt[bl]) bl = c; /* scipy.stats.mode: smallest label wins ties */
            pred[qi] = bl;
        }
    }
    free(best);
    free(cnt);
}
