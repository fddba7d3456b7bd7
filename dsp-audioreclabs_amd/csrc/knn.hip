// knn.hip -- exact k-nearest-neighbour classification for gfx950 (CDNA4).
//
// Replaces KNeighborsClassifier(n_neighbors=k).fit/predict/kneighbors as used by
// src/models.py:33-35,52-58 (sklearn 1.7.2: algorithm='auto' -> kd_tree, minkowski p=2,
// uniform weights, scipy.stats.mode vote).
//
// Pipeline (all stream-ordered, no host sync):
//   1. knn_convert      fp64 [N,D] -> fp32 [N,DP] zero-padded rows (+ max row norm^2, for the
//                       bound); D < DP: expanded form, references (-2 r, |r|^2), queries (q, 1)
//   2. screen           grid (query block, reference split); each query keeps the KC smallest
//                       fp32 squared distances (KC = k + 3 slack, rounded up) of its split; the
//                       [Nq x Nr] distance matrix is never materialised:
//        knn_screen_mfma  D < DP (the 15-d features): |q|^2 + q'.r' on v_mfma_f32_16x16x4_f32
//        knn_screen       D = 16 or 32: direct form (q - r)^2 on the VALU
//        knn_screen_hd    D > 32 (flattened sequences): direct form in chunks of 16 dimensions
//   3. knn_merge        one thread per query: re-ranks every surviving candidate with the
//                       reference's own fp64 distance (sequential sum of squared differences, no
//                       FMA -- sklearn euclidean_rdist), keeps the k best by (distance, index), and
//                       certifies that no screened-out row can beat the k-th; otherwise the query
//                       goes on a fallback list.
//   4. knn_fallback     exhaustive fp64 scan of the listed queries: each query's rows in parts,
//                       one wave per part, the parts' lists merged by the last wave done.
//   5. vote             majority label, smallest label on ties (scipy.stats.mode).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "dsp_audiorec.h"
#include "dsp_device.h"

namespace dsp {

static constexpr int KNN_TQ = 256;   // queries per screening workgroup (one per thread)
static constexpr int KNN_TR = 256;   // reference rows per LDS tile
static constexpr int KNN_SLACK = 3;  // extra screened candidates per split (k = 5 -> 8)
static constexpr int KNN_RU = 4;     // rows x queries per unrolled step of the screen
#ifndef DSP_KNN_QP
#define DSP_KNN_QP 2
#endif

static constexpr int KNN_QP = DSP_KNN_QP;  // queries per screening thread

// mode 0: plain rows (v, 0 ...); mode 1 (reference, expanded form): (-2 v, 0 ..., |v|^2);
// mode 2 (query, expanded form): (v, 0 ..., 1) -- so that |q - r|^2 = |q|^2 + q'.r'.
// One thread per row, its columns in chunks of 16 loaded together before any is used (the loads
// of a rolled column loop waited for each other: 16.9 us for 12 500 rows as for 100 000).
__global__ void knn_convert(const double *__restrict__ src, int64_t N, int D, int DP, int mode,
                            float *__restrict__ dst, unsigned int *maxnorm_bits)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float nrm = 0.f;
    if (i < N) {
        double n64 = 0.0;
        for (int c0 = 0; c0 < DP; c0 += 16) {
            double x[16];
#pragma unroll
            for (int c = 0; c < 16; c++) x[c] = c0 + c < D ? src[i * D + c0 + c] : 0.0;
#pragma unroll
            for (int c = 0; c < 16; c++) {
                const float v = (float)x[c];
                nrm = fmaf(v, v, nrm);
                n64 = fma(x[c], x[c], n64);
                float o = v;
                if (mode == 1) o = c0 + c < D ? (float)(-2.0 * x[c]) : 0.f;
                if (mode == 2 && c0 + c == DP - 1) o = 1.f;
                dst[i * DP + c0 + c] = o;
            }
        }
        if (mode == 1) dst[i * DP + DP - 1] = (float)n64;
    }
    // block max -> one atomic (non-negative floats order like their bit patterns)
    for (int o = 32; o > 0; o >>= 1) nrm = fmaxf(nrm, __shfl_xor(nrm, o, 64));
    if ((threadIdx.x & 63) == 0 && maxnorm_bits) atomicMax(maxnorm_bits, __float_as_uint(nrm));
}

// insert (d, r) into the ascending list (dl, il) of length KC if it beats the last entry:
// branch-free, dl'[i] = med3(dl[i-1], d, dl[i]) (an entry shifts down, takes d, or stays)
template <int KC>
__device__ __forceinline__ void topk_insert(float (&dl)[KC], int (&il)[KC], float d, int r)
{
    if (!(d < dl[KC - 1])) return;
    bool c[KC];
#pragma unroll
    for (int i = 0; i < KC; i++) c[i] = d < dl[i];
#pragma unroll
    for (int i = KC - 1; i > 0; i--) {
        il[i] = c[i - 1] ? il[i - 1] : (c[i] ? r : il[i]);
        dl[i] = __builtin_amdgcn_fmed3f(dl[i - 1], d, dl[i]);
    }
    il[0] = c[0] ? r : il[0];
    dl[0] = fminf(d, dl[0]);
}

// Direct form sum (q - r)^2 on the VALU, for D = 16 and D = 32 (no spare column for the expanded
// form of knn_screen_mfma).  QP queries per thread (queries q0 + tid + KNN_TQ * p): every 16-B LDS
// read of a reference row feeds QP FMA chains -- a broadcast ds_read_b128 costs the CU's LDS pipe
// 4 cycles, shared by 4 SIMDs, so at one query per thread the screen is LDS-bound
template <int DP, int KC, int QP>
__global__ __launch_bounds__(KNN_TQ) void knn_screen(const float *__restrict__ ref32, int64_t Nr,
                                                      const float *__restrict__ q32, int64_t Nq,
                                                      int64_t self_offset, int nsplit,
                                                      float *__restrict__ cand_d,
                                                      int *__restrict__ cand_i)
{
    __shared__ __attribute__((aligned(16))) float tile[KNN_TR * DP];
    const int qb = blockIdx.x, sp = blockIdx.y;
    const int tid = threadIdx.x;
    const int64_t per = (Nr + nsplit - 1) / nsplit;
    const int64_t r0 = (int64_t)sp * per, r1 = min(Nr, r0 + per);
    int64_t q[QP], self[QP];
    float qv[QP][DP];
    float dl[QP][KC];
    int il[QP][KC];
#pragma unroll
    for (int p = 0; p < QP; p++) {
        q[p] = (int64_t)qb * KNN_TQ * QP + tid + KNN_TQ * p;
#pragma unroll
        for (int c = 0; c < DP; c++) qv[p][c] = q[p] < Nq ? q32[q[p] * DP + c] : 0.f;
        self[p] = (self_offset >= 0 && q[p] < Nq) ? self_offset + q[p] : -1;
#pragma unroll
        for (int i = 0; i < KC; i++) {
            dl[p][i] = INFINITY;
            il[p][i] = -1;
        }
    }
    for (int64_t t0 = r0; t0 < r1; t0 += KNN_TR) {
        const int nt = (int)min((int64_t)KNN_TR, r1 - t0);
        __syncthreads();
        // cooperative tile load: KNN_TR rows x DP floats, float4 granules
        for (int e = tid; e < KNN_TR * DP / 4; e += KNN_TQ) {
            const int row = e / (DP / 4);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row < nt) v = reinterpret_cast<const float4 *>(ref32 + (t0 + row) * DP)[e % (DP / 4)];
            reinterpret_cast<float4 *>(tile)[e] = v;
        }
        __syncthreads();
        // rows in groups of RU: independent FMA chains, then the inserts in row order
        constexpr int RU = KNN_RU / QP > 0 ? KNN_RU / QP : 1;
        for (int j0 = 0; j0 < nt; j0 += RU) {
            float d[RU][QP];
#pragma unroll
            for (int u = 0; u < RU; u++) {
                const float4 *rv = reinterpret_cast<const float4 *>(tile + (j0 + u) * DP);  // rows >= nt are zero
#pragma unroll
                for (int p = 0; p < QP; p++) d[u][p] = 0.f;
#pragma unroll
                for (int c4 = 0; c4 < DP / 4; c4++) {
                    const float4 r = rv[c4];
#pragma unroll
                    for (int p = 0; p < QP; p++) {
                        float t;
                        t = qv[p][4 * c4 + 0] - r.x; d[u][p] = fmaf(t, t, d[u][p]);
                        t = qv[p][4 * c4 + 1] - r.y; d[u][p] = fmaf(t, t, d[u][p]);
                        t = qv[p][4 * c4 + 2] - r.z; d[u][p] = fmaf(t, t, d[u][p]);
                        t = qv[p][4 * c4 + 3] - r.w; d[u][p] = fmaf(t, t, d[u][p]);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < RU; u++) {
                const int64_t r = t0 + j0 + u;
#pragma unroll
                for (int p = 0; p < QP; p++)
                    if (j0 + u < nt && r != self[p]) topk_insert<KC>(dl[p], il[p], d[u][p], (int)r);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < QP; p++)
        if (q[p] < Nq) {
            const size_t o = ((size_t)sp * Nq + q[p]) * KC;
#pragma unroll
            for (int i = 0; i < KC; i++) {
                cand_d[o + i] = dl[p][i];
                cand_i[o + i] = il[p][i];
            }
        }
}

// Expanded-form screen on the matrix cores (D < DP, DP = 16 or 32): per 16 reference rows x 16
// queries, DP / 4 v_mfma_f32_16x16x4_f32 accumulate |q|^2 + q'.r'.  Measured on gfx950 this is
// bit for bit a k-ordered fp32 fmaf chain (MI355X_MICROARCH.md), but the certification does not
// depend on it: knn_err_coeffs' bound covers any summation order inside each K = 4 block with up
// to one rounding per product and per addition (see there).  A operand = reference rows
// (lane l: row l & 15), B = queries (lane l: query l & 15), lane l's dimensions in MFMA j are
// 16 (j / 4) + 4 (l >> 4) + (j & 3): one 16-B read per 4 MFMAs.  Result lane l: query l & 15,
// rows 4 (l >> 4) + v, v = 0..3, so four lanes keep partial top-KC lists of each query.
// Keeping the lists is the expensive part (an insertion costs the whole wave whenever one lane
// makes one), so each 16-row step first compares its distances with the query's threshold -- the
// smallest of the four lists' last entries: a row at or above it cannot be among the KC nearest
// of the union -- and inserts only when some lane has a distance below it.  Padding rows carry an
// infinite |r|^2 (distance +inf); the query's own row (self_offset) is masked only in the steps
// that can hold one of the wave's 32 own rows.
#ifndef KNN_MFMA_KC6
#define KNN_MFMA_KC6 1
#endif
#ifndef KNN_MQ_W
#define KNN_MQ_W 4
#endif
#ifndef KNN_MQ_T
#define KNN_MQ_T 2
#endif
#ifndef KNN_MQ_TR
#define KNN_MQ_TR 256
#endif
static constexpr int MQ_W = KNN_MQ_W;                  // waves per workgroup
// query tiles (16 queries) per wave: two while the lists are short, one for long lists (k > 13)
__host__ __device__ constexpr int mq_tiles(int KC) { return KC <= 16 ? KNN_MQ_T : 1; }
__host__ __device__ constexpr int mq_qpb(int KC) { return 16 * mq_tiles(KC) * MQ_W; }  // queries per workgroup
static constexpr int MQ_TR = KNN_MQ_TR;                // reference rows per LDS tile
__host__ __device__ constexpr int mq_stride(int DP) { return DP + 4; }  // conflict-free 16-B reads
typedef float mq_f4 __attribute__((ext_vector_type(4)));
// lane_xor_f (dsp_device.h): the value of lane ^ 16 / lane ^ 32 by the gfx950 permlane swaps
//
// Seeded thresholds: with `seed` non-null each query's threshold starts at seed[q] instead of +inf
// (knn_seed: the KC-th smallest distance over a strided sample of the reference rows, which bounds
// the KC-th smallest of the whole set from above), so a split no longer pays the list warm-up of a
// threshold at +inf -- nearly every 16-row step inserting while the lists fill.  A row is kept only
// below min(seed, the lists' thresholds); knn_merge starts its screening cut-off at the seed, so a
// query whose seed was too tight fails certification and is answered by the exhaustive fallback:
// exactness never depends on the seed.
// The same kernel screens that sample (the pilot; PILOT only names the instantiation, so that a
// profile separates the pilot from the main screen): rows are the sample's, sample row j =
// reference row j * rstride (rstride = 1: every row), and the query's own row is masked in global
// numbering.
template <int DP, int KC, bool PILOT = false>
__global__ __launch_bounds__(64 * MQ_W) void knn_screen_mfma(const float *__restrict__ ref32, int64_t Nr,
                                                           const float *__restrict__ q32, int64_t Nq,
                                                           int64_t self_offset, int nsplit,
                                                           float *__restrict__ cand_d, int *__restrict__ cand_i,
                                                           int rstride, const float *__restrict__ seed)
{
    constexpr int RS = mq_stride(DP), NJ = DP / 4, NV = DP / 16;
    constexpr int MQ_T = mq_tiles(KC), MQ_QPB = mq_qpb(KC);
    __shared__ __attribute__((aligned(16))) float tile[MQ_TR * RS];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, rg = lane >> 4;
    const int sp = blockIdx.y;
    const int64_t per = (Nr + nsplit - 1) / nsplit;  // Nr: rows of the (sampled) set
    const int64_t r0 = (int64_t)sp * per, r1 = min(Nr, r0 + per);
    const int64_t wq0 = (int64_t)blockIdx.x * MQ_QPB + wid * MQ_T * 16;  // the wave's first query
    // sample rows that can be one of the wave's own queries (self_offset >= 0): [slo, shi)
    const int64_t g0 = self_offset + wq0, g1 = g0 + 16 * MQ_T;
    const int64_t slo = self_offset >= 0 ? (g0 + rstride - 1) / rstride : INT64_MIN / 2;
    const int64_t shi = self_offset >= 0 ? (g1 + rstride - 1) / rstride : INT64_MIN / 2;
    int64_t q[MQ_T], self[MQ_T];
    float qb[MQ_T][NJ], qn[MQ_T], tau[MQ_T];
    float dl[MQ_T][KC];
    int il[MQ_T][KC];
#pragma unroll
    for (int t = 0; t < MQ_T; t++) {
        q[t] = wq0 + t * 16 + col;
        const float *qr = q32 + (q[t] < Nq ? q[t] : 0) * DP;
        float n = 0.f;  // |q|^2 as the VALU screen computes it (fmaf chain over the real columns)
#pragma unroll
        for (int c = 0; c < DP - 1; c++) n = fmaf(qr[c], qr[c], n);
        qn[t] = n;
#pragma unroll
        for (int h = 0; h < NV; h++) {
            const float4 v = *reinterpret_cast<const float4 *>(qr + 16 * h + 4 * rg);
            qb[t][4 * h] = v.x;
            qb[t][4 * h + 1] = v.y;
            qb[t][4 * h + 2] = v.z;
            qb[t][4 * h + 3] = v.w;
        }
        // the query's own row as a sample row (-1: not in the sample)
        const int64_t sg = (self_offset >= 0 && q[t] < Nq) ? self_offset + q[t] : -1;
        self[t] = (sg >= 0 && sg % rstride == 0) ? sg / rstride : -1;
        tau[t] = (seed && q[t] < Nq) ? seed[q[t]] : INFINITY;
#pragma unroll
        for (int i = 0; i < KC; i++) {
            dl[t][i] = INFINITY;
            il[t][i] = -1;
        }
    }
    for (int64_t t0 = r0; t0 < r1; t0 += MQ_TR) {
        const int nt = (int)min((int64_t)MQ_TR, r1 - t0);
        __syncthreads();
        for (int e = tid; e < MQ_TR * DP / 4; e += 64 * MQ_W) {
            const int row = e / (DP / 4), c4 = e % (DP / 4);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row < nt)
                v = reinterpret_cast<const float4 *>(ref32 + (t0 + row) * rstride * DP)[c4];
            else if (c4 == DP / 4 - 1)
                v.w = INFINITY;  // |r|^2 of a padding row: distance +inf
            *reinterpret_cast<float4 *>(tile + row * RS + 4 * c4) = v;
        }
        __syncthreads();
        const int nt16 = (nt + 15) & ~15;
        for (int s0 = 0; s0 < nt16; s0 += 16) {
            float a[NJ];
#pragma unroll
            for (int h = 0; h < NV; h++) {
                const float4 v = *reinterpret_cast<const float4 *>(tile + (s0 + col) * RS + 16 * h + 4 * rg);
                a[4 * h] = v.x;
                a[4 * h + 1] = v.y;
                a[4 * h + 2] = v.z;
                a[4 * h + 3] = v.w;
            }
            mq_f4 acc[MQ_T];
#pragma unroll
            for (int t = 0; t < MQ_T; t++) acc[t] = mq_f4{qn[t], qn[t], qn[t], qn[t]};
#pragma unroll
            for (int j = 0; j < NJ; j++)
#pragma unroll
                for (int t = 0; t < MQ_T; t++) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], qb[t][j], acc[t], 0, 0, 0);
            const int64_t rb = t0 + s0;  // the step's first row
            if (rb < shi && rb + 16 > slo)  // wave-uniform: a query's own row may be here
                for (int t = 0; t < MQ_T; t++)
                    for (int v = 0; v < 4; v++)
                        if (rb + 4 * rg + v == self[t]) acc[t][v] = INFINITY;
            for (int t = 0; t < MQ_T; t++) {
                bool c[4];
#pragma unroll
                for (int v = 0; v < 4; v++) c[v] = acc[t][v] < tau[t];
                if (__builtin_amdgcn_ballot_w64(c[0] | c[1] | c[2] | c[3])) {
#pragma unroll
                    for (int v = 0; v < 4; v++)
                        if (c[v]) topk_insert<KC>(dl[t], il[t], acc[t][v], (int)(rb + 4 * rg + v));
                    float th = dl[t][KC - 1];
                    th = fminf(th, lane_xor_f(th, 16, lane));
                    th = fminf(th, lane_xor_f(th, 32, lane));
                    tau[t] = fminf(tau[t], th);  // = min(seed, the lists' thresholds)
                }
            }
        }
    }
    // the four partial lists of each query (lanes col, col + 16, col + 32, col + 48; disjoint
    // rows) -> one, by a butterfly over lane ^ 16 and lane ^ 32
#pragma unroll
    for (int t = 0; t < MQ_T; t++) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int m = 16 << h;
            float pd[KC];
            int pi[KC];
#pragma unroll
            for (int i = 0; i < KC; i++) {
                pd[i] = __shfl_xor(dl[t][i], m, 64);
                pi[i] = __shfl_xor(il[t][i], m, 64);
            }
#pragma unroll
            for (int i = 0; i < KC; i++)
                if (pi[i] >= 0) topk_insert<KC>(dl[t], il[t], pd[i], pi[i]);
        }
        if (rg == 0 && q[t] < Nq) {
            const size_t o = ((size_t)sp * Nq + q[t]) * KC;
#pragma unroll
            for (int i = 0; i < KC; i++) {
                cand_d[o + i] = dl[t][i];
                if (cand_i) cand_i[o + i] = il[t][i];
            }
        }
    }
}

// The pilot (seeded thresholds): over the sampled rows (sample row j = reference row j * rstride)
// each query needs only an upper bound for the KC-th smallest distance of the whole set, and the
// KC-th smallest of any KC distinct rows' distances is one.  So instead of top-KC lists (whose
// insertions, from thresholds at +inf, were most of the old pilot's time) every lane keeps running
// minima: lane (col, rg) of a 16 x 16 MFMA tile sees rows rb + 4 rg + v, v = 0..3, and keeps one
// minimum per (v, step parity) -- PIL_CLS = 32 disjoint row classes per query and split, written
// to pilot_d[split][query][32]; knn_seed then takes the KC-th smallest of all of them, which is
// >= the KC-th smallest of the sample >= the KC-th smallest of the set.  Each class minimum over
// ~nsample / 32 rows sits near quantile 1/(nsample/32) of the query's distances, and the 6th of 32
// such near quantile 0.2 * 32 / nsample: as tight as the exact 6th smallest of the sample.
static constexpr int PIL_CLS = 32;
template <int DP>
__global__ __launch_bounds__(64 * MQ_W) void knn_pilot_mfma(const float *__restrict__ ref32, int64_t Nr,
                                                            const float *__restrict__ q32, int64_t Nq,
                                                            int64_t self_offset, int nsplit,
                                                            float *__restrict__ pilot_d, int rstride)
{
    constexpr int RS = mq_stride(DP), NJ = DP / 4, NV = DP / 16;
    constexpr int MQ_T = KNN_MQ_T, MQ_QPB = 16 * MQ_T * MQ_W;
    static_assert(MQ_TR % 32 == 0, "two 16-row steps per trip");
    __shared__ __attribute__((aligned(16))) float tile[MQ_TR * RS];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 15, rg = lane >> 4;
    const int sp = blockIdx.y;
    const int64_t per = (Nr + nsplit - 1) / nsplit;  // Nr: rows of the sample
    const int64_t r0 = (int64_t)sp * per, r1 = min(Nr, r0 + per);
    const int64_t wq0 = (int64_t)blockIdx.x * MQ_QPB + wid * MQ_T * 16;
    const int64_t g0 = self_offset + wq0, g1 = g0 + 16 * MQ_T;
    const int64_t slo = self_offset >= 0 ? (g0 + rstride - 1) / rstride : INT64_MIN / 2;
    const int64_t shi = self_offset >= 0 ? (g1 + rstride - 1) / rstride : INT64_MIN / 2;
    int64_t q[MQ_T], self[MQ_T];
    float qb[MQ_T][NJ], qn[MQ_T], mn[MQ_T][2][4];
#pragma unroll
    for (int t = 0; t < MQ_T; t++) {
        q[t] = wq0 + t * 16 + col;
        const float *qr = q32 + (q[t] < Nq ? q[t] : 0) * DP;
        float n = 0.f;  // |q|^2 as the screen computes it
#pragma unroll
        for (int c = 0; c < DP - 1; c++) n = fmaf(qr[c], qr[c], n);
        qn[t] = n;
#pragma unroll
        for (int h = 0; h < NV; h++) {
            const float4 v = *reinterpret_cast<const float4 *>(qr + 16 * h + 4 * rg);
            qb[t][4 * h] = v.x;
            qb[t][4 * h + 1] = v.y;
            qb[t][4 * h + 2] = v.z;
            qb[t][4 * h + 3] = v.w;
        }
        const int64_t sg = (self_offset >= 0 && q[t] < Nq) ? self_offset + q[t] : -1;
        self[t] = (sg >= 0 && sg % rstride == 0) ? sg / rstride : -1;
#pragma unroll
        for (int h = 0; h < 2; h++)
#pragma unroll
            for (int v = 0; v < 4; v++) mn[t][h][v] = INFINITY;
    }
    for (int64_t t0 = r0; t0 < r1; t0 += MQ_TR) {
        const int nt = (int)min((int64_t)MQ_TR, r1 - t0);
        __syncthreads();
        for (int e = tid; e < MQ_TR * DP / 4; e += 64 * MQ_W) {
            const int row = e / (DP / 4), c4 = e % (DP / 4);
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row < nt)
                v = reinterpret_cast<const float4 *>(ref32 + (t0 + row) * rstride * DP)[c4];
            else if (c4 == DP / 4 - 1)
                v.w = INFINITY;  // |r|^2 of a padding row: distance +inf
            *reinterpret_cast<float4 *>(tile + row * RS + 4 * c4) = v;
        }
        __syncthreads();
        const int nt32 = (nt + 31) & ~31;
        for (int s0 = 0; s0 < nt32; s0 += 32) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                float a[NJ];
#pragma unroll
                for (int u = 0; u < NV; u++) {
                    const float4 v = *reinterpret_cast<const float4 *>(tile + (s0 + 16 * h + col) * RS + 16 * u + 4 * rg);
                    a[4 * u] = v.x;
                    a[4 * u + 1] = v.y;
                    a[4 * u + 2] = v.z;
                    a[4 * u + 3] = v.w;
                }
                mq_f4 acc[MQ_T];
#pragma unroll
                for (int t = 0; t < MQ_T; t++) acc[t] = mq_f4{qn[t], qn[t], qn[t], qn[t]};
#pragma unroll
                for (int j = 0; j < NJ; j++)
#pragma unroll
                    for (int t = 0; t < MQ_T; t++) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], qb[t][j], acc[t], 0, 0, 0);
                const int64_t rb = t0 + s0 + 16 * h;
                if (rb < shi && rb + 16 > slo)  // wave-uniform: a query's own row may be here
                    for (int t = 0; t < MQ_T; t++)
                        for (int v = 0; v < 4; v++)
                            if (rb + 4 * rg + v == self[t]) acc[t][v] = INFINITY;
#pragma unroll
                for (int t = 0; t < MQ_T; t++)
#pragma unroll
                    for (int v = 0; v < 4; v++) mn[t][h][v] = fminf(mn[t][h][v], acc[t][v]);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < MQ_T; t++) {
        if (q[t] >= Nq) continue;
        float *o = pilot_d + ((size_t)sp * Nq + q[t]) * PIL_CLS + 8 * rg;
        *reinterpret_cast<float4 *>(o) = make_float4(mn[t][0][0], mn[t][0][1], mn[t][0][2], mn[t][0][3]);
        *reinterpret_cast<float4 *>(o + 4) = make_float4(mn[t][1][0], mn[t][1][1], mn[t][1][2], mn[t][1][3]);
    }
}

// the seed of each query: the KC-th smallest of the pilot's nsplit x KC screened distances (the KC
// smallest of the sample), one thread per query.  A pilot that was itself seeded (prev) kept only
// distances below prev[q]: its KC-th is then either the sample's own KC-th (< prev) or +inf (the
// sample's KC-th is >= prev), so the seed is the smaller of the two -- an upper bound either way.
template <int KC, int NPER = KC>
__global__ __launch_bounds__(256) void knn_seed(const float *__restrict__ cand_d, int nsplit, int64_t Nq,
                                                const float *__restrict__ prev, float *__restrict__ seed,
                                                float scale)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= Nq) return;
    float k32[KC];
#pragma unroll
    for (int i = 0; i < KC; i++) k32[i] = INFINITY;
    for (int s = 0; s < nsplit; s++) {
        const float *c = cand_d + ((size_t)s * Nq + q) * NPER;
#pragma unroll
        for (int i = 0; i < NPER; i++) {
            float v = c[i];
#pragma unroll
            for (int j = 0; j < KC; j++) {
                const float lo = fminf(v, k32[j]);
                v = fmaxf(v, k32[j]);
                k32[j] = lo;
            }
        }
    }
    const float kth = prev ? fminf(k32[KC - 1], prev[q]) : k32[KC - 1];
    seed[q] = kth * scale;  // scale: 1 (< 1 only in the diagnostic build's tests, final stage)
}

// High-dimensional rows (D > 32: the sequence method's flattened (E, ZCR) sequences,
// compare_feature_methods.py:117-154): direct form sum (q - r)^2 in fp32, the dimensions walked
// in chunks of 16 against LDS tiles of 64 reference rows; one query per thread, 64 running
// distances in registers, then the same top-KC insertion.
static constexpr int HD_ROWS = 64, HD_COLS = 16;
template <int KC>
__global__ __launch_bounds__(KNN_TQ) void knn_screen_hd(const float *__restrict__ ref32, int64_t Nr,
                                                         const float *__restrict__ q32, int64_t Nq, int DP,
                                                         int64_t self_offset, int nsplit,
                                                         float *__restrict__ cand_d, int *__restrict__ cand_i)
{
    __shared__ __attribute__((aligned(16))) float tile[HD_ROWS * HD_COLS];
    const int tid = threadIdx.x;
    const int64_t q = (int64_t)blockIdx.x * KNN_TQ + tid;
    const int sp = blockIdx.y;
    const int64_t per = (Nr + nsplit - 1) / nsplit;
    const int64_t r0 = (int64_t)sp * per, r1 = min(Nr, r0 + per);
    const int64_t self = (self_offset >= 0 && q < Nq) ? self_offset + q : -1;
    const float *qrow = q32 + (q < Nq ? q : 0) * DP;
    float dl[KC];
    int il[KC];
#pragma unroll
    for (int i = 0; i < KC; i++) {
        dl[i] = INFINITY;
        il[i] = -1;
    }
    for (int64_t t0 = r0; t0 < r1; t0 += HD_ROWS) {
        const int nt = (int)min((int64_t)HD_ROWS, r1 - t0);
        float d[HD_ROWS];
#pragma unroll
        for (int u = 0; u < HD_ROWS; u++) d[u] = 0.f;
        for (int c0 = 0; c0 < DP; c0 += HD_COLS) {
            float qc[HD_COLS];
#pragma unroll
            for (int c4 = 0; c4 < HD_COLS / 4; c4++) {
                const float4 v = reinterpret_cast<const float4 *>(qrow + c0)[c4];
                qc[4 * c4] = v.x;
                qc[4 * c4 + 1] = v.y;
                qc[4 * c4 + 2] = v.z;
                qc[4 * c4 + 3] = v.w;
            }
            __syncthreads();
            {  // 64 rows x 16 columns, one float4 per thread
                const int row = tid >> 2, c4 = tid & 3;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (row < nt) v = reinterpret_cast<const float4 *>(ref32 + (t0 + row) * DP + c0)[c4];
                reinterpret_cast<float4 *>(tile)[tid] = v;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < HD_ROWS; u++) {
                const float4 *rv = reinterpret_cast<const float4 *>(tile + u * HD_COLS);
#pragma unroll
                for (int c4 = 0; c4 < HD_COLS / 4; c4++) {
                    const float4 r = rv[c4];
                    float t;
                    t = qc[4 * c4 + 0] - r.x; d[u] = fmaf(t, t, d[u]);
                    t = qc[4 * c4 + 1] - r.y; d[u] = fmaf(t, t, d[u]);
                    t = qc[4 * c4 + 2] - r.z; d[u] = fmaf(t, t, d[u]);
                    t = qc[4 * c4 + 3] - r.w; d[u] = fmaf(t, t, d[u]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < HD_ROWS; u++) {
            const int64_t r = t0 + u;
            if (u < nt && r != self) topk_insert<KC>(dl, il, d[u], (int)r);
        }
    }
    if (q < Nq) {
        const size_t o = ((size_t)sp * Nq + q) * KC;
#pragma unroll
        for (int i = 0; i < KC; i++) {
            cand_d[o + i] = dl[i];
            cand_i[o + i] = il[i];
        }
    }
}

#pragma clang fp contract(off)
// sklearn euclidean_rdist: sequential d += t*t, no FMA
__device__ __forceinline__ double rdist64(const double *__restrict__ a, const double *__restrict__ b, int D)
{
    double d = 0.0;
    for (int c = 0; c < D; c++) {
        const double t = a[c] - b[c];
        d = d + t * t;
    }
    return d;
}
// The same for D <= 16 (the 15-d features) with the query in registers and the reference row's
// loads all issued before its first use: the rolled loop above waited for each of its loads in
// turn, so a re-rank or a fallback scan paid ~D memory latencies per row (round 6: the 3
// fallback queries of the 100k x 100k self-query on extracted features took 1.06 ms).
struct QRow16 {
    double v[16];
};
__device__ __forceinline__ QRow16 qrow16(const double *__restrict__ qx, int D)
{
    QRow16 q;
#pragma unroll
    for (int c = 0; c < 16; c++) q.v[c] = c < D ? qx[c] : 0.0;
    return q;
}
__device__ __forceinline__ void row16_load(double (&b)[16], const double *__restrict__ r, int D)
{
#pragma unroll
    for (int c = 0; c < 16; c++) b[c] = c < D ? r[c] : 0.0;
}
__device__ __forceinline__ double rdist64_16(const QRow16 &q, const double (&b)[16], int D)
{
    double d = 0.0;
#pragma unroll
    for (int c = 0; c < 16; c++)
        if (c < D) {
            const double t = q.v[c] - b[c];
            d = d + t * t;
        }
    return d;
}
// rdist64 through the register path when D <= 16
__device__ __forceinline__ double rdist64_q(const QRow16 &q, const double *__restrict__ qx, const double *__restrict__ r,
                                            int D)
{
    if (D <= 16) {
        double b[16];
        row16_load(b, r, D);
        return rdist64_16(q, b, D);
    }
    return rdist64(qx, r, D);
}
#pragma clang fp contract(on)

__device__ __forceinline__ bool cand_less(double da, int ia, double db, int ib)
{
    return da < db || (da == db && ia < ib);
}

template <int K>
__device__ __forceinline__ void topk64_insert(double (&dl)[K], int (&il)[K], int kk, double d, int r)
{
    if (!cand_less(d, r, dl[kk - 1], il[kk - 1])) return;
#pragma unroll
    for (int i = K - 1; i > 0; i--) {
        if (i >= kk) continue;
        const bool shift = cand_less(d, r, dl[i - 1], il[i - 1]);
        const bool here = !shift && cand_less(d, r, dl[i], il[i]);
        if (shift) {
            dl[i] = dl[i - 1];
            il[i] = il[i - 1];
        } else if (here) {
            dl[i] = d;
            il[i] = r;
        }
    }
    if (cand_less(d, r, dl[0], il[0])) {
        dl[0] = d;
        il[0] = r;
    }
}

__device__ int vote(const int *il, int k, const int32_t *labels)
{
    int best = -1, bestc = 0;
    for (int a = 0; a < k; a++) {
        if (il[a] < 0) continue;
        const int la = labels[il[a]];
        int c = 0;
        for (int b = 0; b < k; b++) c += il[b] >= 0 && labels[il[b]] == la;
        if (c > bestc || (c == bestc && la < best)) {
            bestc = c;
            best = la;
        }
    }
    return best;
}

static constexpr int KMAX = 32;

// the KM smallest (distance, index) pairs in ascending order, fixed length (no register array is
// indexed at run time, so the lists stay in registers)
template <int KM>
__device__ __forceinline__ void topk_fixed_insert(double (&dl)[KM], int (&il)[KM], double d, int r)
{
    if (!cand_less(d, r, dl[KM - 1], il[KM - 1])) return;
#pragma unroll
    for (int i = KM - 1; i > 0; i--) {
        const bool shift = cand_less(d, r, dl[i - 1], il[i - 1]);
        const bool here = !shift && cand_less(d, r, dl[i], il[i]);
        dl[i] = shift ? dl[i - 1] : here ? d : dl[i];
        il[i] = shift ? il[i - 1] : here ? r : il[i];
    }
    if (cand_less(d, r, dl[0], il[0])) {
        dl[0] = d;
        il[0] = r;
    }
}
template <int KM, typename T>
__device__ __forceinline__ T kth_of(const T (&a)[KM], int k)  // a[k - 1], k run-time
{
    T v = a[0];
#pragma unroll
    for (int i = 1; i < KM; i++) v = (i == k - 1) ? a[i] : v;
    return v;
}

// One thread per query, each split's KC candidates loaded together: lists of KM = 16 / 32 (k > 8;
// the group merge's networks at those lengths cost minutes of compile time per instantiation).
template <int KC, int KM>
__global__ __launch_bounds__(64) void knn_merge1(const double *__restrict__ ref, const double *__restrict__ query,
                          int64_t Nr, int64_t Nq, int D, int k, int nsplit, int64_t self_offset,
                          const float *__restrict__ cand_d, const int *__restrict__ cand_i,
                          const unsigned int *maxnorm_bits, double err_rel, double err_abs,
                          const int32_t *__restrict__ labels, int32_t *__restrict__ idx,
                          double *__restrict__ dist, int32_t *__restrict__ pred, int *fb_count,
                          int *fb_list, const float *__restrict__ seed)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= Nq) return;
    const double *qx = query + q * D;
    const QRow16 q16 = qrow16(qx, D <= 16 ? D : 0);
    double dl[KM];
    int il[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) {
        dl[i] = INFINITY;
        il[i] = 0x7fffffff;
    }
    double qn = 0.0;
    if (D <= 16) {
#pragma unroll
        for (int c = 0; c < 16; c++)
            if (c < D) qn += q16.v[c] * q16.v[c];
    } else {
        for (int c = 0; c < D; c++) qn += qx[c] * qx[c];
    }
    // |fp32 screened distance - fp64 distance| <= err(d): fp32 rounding of the inputs and of the
    // sum (direct or expanded form), coefficients from the host (knn_err_coeffs)
    const double rmax = (double)__uint_as_float(*maxnorm_bits);
    auto err = [&](double d) { return err_rel * d + err_abs * (qn + rmax) + 1e-30; };
    const int64_t self = self_offset >= 0 ? self_offset + q : -1;
    // pass 1 (fp32 only): the k-th smallest screened distance t32 and the screening cut-off of
    // every split whose candidate list is full
    float k32[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) k32[i] = INFINITY;
    // cut: every row the screen did not keep has a screened distance >= cut (a seeded screen keeps
    // only rows below min(seed, the lists' thresholds))
    float kth = INFINITY, cut = seed ? seed[q] : INFINITY;
    for (int s = 0; s < nsplit; s++) {
        const size_t o = ((size_t)s * Nq + q) * KC;
        int rr[KC];
        float dd[KC];
#pragma unroll
        for (int i = 0; i < KC; i++) {
            rr[i] = cand_i[o + i];
            dd[i] = cand_d[o + i];
        }
#pragma unroll
        for (int i = 0; i < KC; i++) {
            if (rr[i] < 0 || rr[i] == self || !(dd[i] < kth)) continue;
            float v = dd[i];  // sorted insert into the KM smallest
#pragma unroll
            for (int j = 0; j < KM; j++) {
                const float lo = fminf(v, k32[j]);
                v = fmaxf(v, k32[j]);
                k32[j] = lo;
            }
            kth = kth_of<KM>(k32, k);
        }
        if (rr[KC - 1] >= 0) cut = fminf(cut, dd[KC - 1]);
    }
    // pass 2: fp64 re-rank (sklearn's own distance) of the candidates that can still be among the
    // k nearest: a candidate with d - err(d) > t32 + err(t32) is farther (in fp64) than the k
    // candidates at or below t32
    const double t32 = (double)kth;
    const double keep = t32 < INFINITY ? t32 + err(t32) : INFINITY;
    for (int s = 0; s < nsplit; s++) {
        const size_t o = ((size_t)s * Nq + q) * KC;
        int rr[KC];
        float dd[KC];
#pragma unroll
        for (int i = 0; i < KC; i++) {
            rr[i] = cand_i[o + i];
            dd[i] = cand_d[o + i];
        }
#pragma unroll
        for (int i = 0; i < KC; i++) {
            const double d = (double)dd[i];
            if (rr[i] < 0 || rr[i] == self || d - err(d) > keep) continue;
            topk_fixed_insert<KM>(dl, il, rdist64_q(q16, qx, ref + (int64_t)rr[i] * D, D), rr[i]);
        }
    }
    // certification: any row that was screened out has fp32 distance >= cut; its true fp64
    // squared distance is >= cut - tol (fp32 rounding of inputs and of the sum).
    const double tol = err((double)cut);
    const bool ok = !(cut < INFINITY) || ((double)cut - tol > kth_of<KM>(dl, k));
    if (!ok) {
        const int slot = atomicAdd(fb_count, 1);
        fb_list[slot] = (int)q;
        return;
    }
    int outi[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) {
        const bool valid = dl[i] < INFINITY;
        outi[i] = valid ? il[i] : -1;
        if (i < k) {
            idx[q * k + i] = outi[i];
            dist[q * k + i] = valid ? sqrt(dl[i]) : INFINITY;
        }
    }
    if (pred && labels) {  // scipy.stats.mode of the k labels: the smallest most frequent
        int best = -1, bestc = 0;
#pragma unroll
        for (int a = 0; a < KM; a++) {
            if (a >= k || outi[a] < 0) continue;
            const int la = labels[outi[a]];
            int cnt = 0;
#pragma unroll
            for (int b2 = 0; b2 < KM; b2++) cnt += b2 < k && outi[b2] >= 0 && labels[outi[b2]] == la;
            if (cnt > bestc || (cnt == bestc && la < best)) {
                bestc = cnt;
                best = la;
            }
        }
        pred[q] = best;
    }
}

// the KM smallest of two ascending lists (a: this lane's, the partner's via shuffle) into a,
// ascending: elementwise min of a and the reversed partner list (a bitonic sequence holding the
// KM smallest of the union), then a bitonic merge network
template <int KM>
__device__ __forceinline__ void merge_sorted_f(float (&a)[KM], int m)
{
    float b[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) b[i] = __shfl_xor(a[i], m, 64);
#pragma unroll
    for (int i = 0; i < KM; i++) a[i] = fminf(a[i], b[KM - 1 - i]);
#pragma unroll
    for (int h = KM / 2; h > 0; h >>= 1)
#pragma unroll
        for (int i = 0; i < KM; i++)
            if ((i & h) == 0) {
                const float lo = fminf(a[i], a[i + h]), hi = fmaxf(a[i], a[i + h]);
                a[i] = lo;
                a[i + h] = hi;
            }
}
// the same for (distance, index) pairs in cand_less order (a strict total order: the result is
// the KM smallest pairs of the union whatever the lanes' shares were)
template <int KM>
__device__ __forceinline__ void merge_sorted_pairs(double (&dl)[KM], int (&il)[KM], int m)
{
    double bd[KM];
    int bi[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) {
        bd[i] = __shfl_xor(dl[i], m, 64);
        bi[i] = __shfl_xor(il[i], m, 64);
    }
#pragma unroll
    for (int i = 0; i < KM; i++) {
        const bool t = cand_less(bd[KM - 1 - i], bi[KM - 1 - i], dl[i], il[i]);
        dl[i] = t ? bd[KM - 1 - i] : dl[i];
        il[i] = t ? bi[KM - 1 - i] : il[i];
    }
#pragma unroll
    for (int h = KM / 2; h > 0; h >>= 1)
#pragma unroll
        for (int i = 0; i < KM; i++)
            if ((i & h) == 0) {
                const bool t = cand_less(dl[i + h], il[i + h], dl[i], il[i]);
                const double d0 = dl[i], d1 = dl[i + h];
                const int i0 = il[i], i1 = il[i + h];
                dl[i] = t ? d1 : d0;
                il[i] = t ? i1 : i0;
                dl[i + h] = t ? d0 : d1;
                il[i + h] = t ? i0 : i1;
            }
}

// MG lanes per query (8 queries per wave): lane j of a query's group takes the splits s = j
// (mod MG), keeps its own fp32 k-th list (pass 1) and fp64 (distance, index) list (pass 2), and
// the group merges them by a lane^1 / ^2 / ^4 butterfly.  The k-th smallest of a multiset and
// the KM smallest (distance, index) pairs do not depend on how the candidates were shared, so
// the results equal one thread walking every split (round 3's knn_merge); with MG times the
// threads, a 12 500-query shard fills the chip instead of 196 waves.
#ifndef KNN_MG
#define KNN_MG 8
#endif
static constexpr int MG = KNN_MG;  // lanes per query (a power of two <= 64)
template <int KC, int KM>
__global__ __launch_bounds__(64) void knn_merge(const double *__restrict__ ref, const double *__restrict__ query,
                          int64_t Nr, int64_t Nq, int D, int k, int nsplit, int64_t self_offset,
                          const float *__restrict__ cand_d, const int *__restrict__ cand_i,
                          const unsigned int *maxnorm_bits, double err_rel, double err_abs,
                          const int32_t *__restrict__ labels, int32_t *__restrict__ idx,
                          double *__restrict__ dist, int32_t *__restrict__ pred, int *fb_count,
                          int *fb_list, const float *__restrict__ seed)
{
    const int j = threadIdx.x % MG;
    const int64_t qr = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MG;
    const bool live = qr < Nq;  // every lane takes part in the shuffles
    const int64_t q = live ? qr : Nq - 1;
    const double *qx = query + q * D;
    const QRow16 q16 = qrow16(qx, D <= 16 ? D : 0);
    double dl[KM];
    int il[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) {
        dl[i] = INFINITY;
        il[i] = 0x7fffffff;
    }
    double qn = 0.0;
    if (D <= 16) {
#pragma unroll
        for (int c = 0; c < 16; c++)
            if (c < D) qn += q16.v[c] * q16.v[c];
    } else {
        for (int c = 0; c < D; c++) qn += qx[c] * qx[c];
    }
    // |fp32 screened distance - fp64 distance| <= err(d): fp32 rounding of the inputs and of the
    // sum (direct or expanded form), coefficients from the host (knn_err_coeffs)
    const double rmax = (double)__uint_as_float(*maxnorm_bits);
    auto err = [&](double d) { return err_rel * d + err_abs * (qn + rmax) + 1e-30; };
    const int64_t self = self_offset >= 0 ? self_offset + q : -1;
    // pass 1 (fp32 only): the k-th smallest screened distance t32 and the screening cut-off of
    // every split whose candidate list is full
    float k32[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) k32[i] = INFINITY;
    // cut: every row the screen did not keep has a screened distance >= cut (a seeded screen keeps
    // only rows below min(seed, the lists' thresholds))
    float kth = INFINITY, cut = seed ? seed[q] : INFINITY;
    auto load_split = [&](int s, int (&rr)[KC], float (&dd)[KC]) {
        const size_t o = ((size_t)s * Nq + q) * KC;
#pragma unroll
        for (int i = 0; i < KC; i++) {
            rr[i] = cand_i[o + i];
            dd[i] = cand_d[o + i];
        }
    };
    auto pass1 = [&](const int (&rr)[KC], const float (&dd)[KC]) {
#pragma unroll
        for (int i = 0; i < KC; i++) {
            // a value at or past this lane's k-th is not among the group's k smallest either
            if (rr[i] < 0 || rr[i] == self || !(dd[i] < kth)) continue;
            float v = dd[i];  // sorted insert into the KM smallest
#pragma unroll
            for (int jj = 0; jj < KM; jj++) {
                const float lo = fminf(v, k32[jj]);
                v = fmaxf(v, k32[jj]);
                k32[jj] = lo;
            }
            kth = kth_of<KM>(k32, k);
        }
        if (rr[KC - 1] >= 0) cut = fminf(cut, dd[KC - 1]);
    };
    // short lists (KC <= 8): a lane's first two splits are loaded together and kept in registers
    // for pass 2 (12 500 queries take 13 splits, 100 000 take 6: every split of MG = 8 lanes)
    constexpr bool CACHE2 = KC <= 8;
    constexpr int NC = CACHE2 ? KC : 1;
    int rc0[NC], rc1[NC];
    float dc0[NC], dc1[NC];
    const bool h0 = CACHE2 && j < nsplit, h1 = CACHE2 && j + MG < nsplit;
    if constexpr (CACHE2) {
        if (h0) load_split(j, rc0, dc0);
        if (h1) load_split(j + MG, rc1, dc1);
        if (h0) pass1(rc0, dc0);
        if (h1) pass1(rc1, dc1);
    }
    for (int s = j + (CACHE2 ? 2 * MG : 0); s < nsplit; s += MG) {
        int rr[KC];
        float dd[KC];
        load_split(s, rr, dd);
        pass1(rr, dd);
    }
#pragma unroll
    for (int m = 1; m < MG; m <<= 1) {
        merge_sorted_f<KM>(k32, m);
        cut = fminf(cut, __shfl_xor(cut, m, 64));
    }
    kth = kth_of<KM>(k32, k);
    // pass 2: fp64 re-rank (sklearn's own distance) of the candidates that can still be among the
    // k nearest: a candidate with d - err(d) > t32 + err(t32) is farther (in fp64) than the k
    // candidates at or below t32
    const double t32 = (double)kth;
    const double keep = t32 < INFINITY ? t32 + err(t32) : INFINITY;
    // the candidates that pass are few (about k per query over its MG lanes): a bit mask, then ONE
    // rolled loop that picks each candidate by selects -- unrolling the row loads, the distance and
    // the list insert per candidate slot made this kernel ~15k instructions (instruction-cache
    // misses) for no gain
    auto need = [&](int r, float df) {
        const double d = (double)df;
        return !(r < 0 || r == self || d - err(d) > keep);
    };
    auto rerank = [&](int r) { topk_fixed_insert<KM>(dl, il, rdist64_q(q16, qx, ref + (int64_t)r * D, D), r); };
    if constexpr (CACHE2) {
        unsigned mask = 0;
#pragma unroll
        for (int i = 0; i < KC; i++) {
            if (h0 && need(rc0[i], dc0[i])) mask |= 1u << i;
            if (h1 && need(rc1[i], dc1[i])) mask |= 1u << (KC + i);
        }
        while (mask) {
            const int bit = __builtin_ctz(mask);
            mask &= mask - 1;
            int r = rc0[0];
#pragma unroll
            for (int i = 0; i < KC; i++) {
                r = bit == i ? rc0[i] : r;
                r = bit == KC + i ? rc1[i] : r;
            }
            rerank(r);
        }
    }
    for (int s = j + (CACHE2 ? 2 * MG : 0); s < nsplit; s += MG) {
        int rr[KC];
        float dd[KC];
        load_split(s, rr, dd);
        unsigned long long mask = 0;
#pragma unroll
        for (int i = 0; i < KC; i++)
            if (need(rr[i], dd[i])) mask |= 1ull << i;
        while (mask) {
            const int bit = __builtin_ctzll(mask);
            mask &= mask - 1;
            int r = rr[0];
#pragma unroll
            for (int i = 1; i < KC; i++) r = bit == i ? rr[i] : r;
            rerank(r);
        }
    }
#pragma unroll
    for (int m = 1; m < MG; m <<= 1) merge_sorted_pairs<KM>(dl, il, m);
    if (!live || j != 0) return;
    // certification: any row that was screened out has fp32 distance >= cut; its true fp64
    // squared distance is >= cut - tol (fp32 rounding of inputs and of the sum).
    const double tol = err((double)cut);
    const bool ok = !(cut < INFINITY) || ((double)cut - tol > kth_of<KM>(dl, k));
    if (!ok) {
        const int slot = atomicAdd(fb_count, 1);
        fb_list[slot] = (int)q;
        return;
    }
    int outi[KM];
#pragma unroll
    for (int i = 0; i < KM; i++) {
        const bool valid = dl[i] < INFINITY;
        outi[i] = valid ? il[i] : -1;
        if (i < k) {
            idx[q * k + i] = outi[i];
            dist[q * k + i] = valid ? sqrt(dl[i]) : INFINITY;
        }
    }
    if (pred && labels) {  // scipy.stats.mode of the k labels: the smallest most frequent
        int best = -1, bestc = 0;
#pragma unroll
        for (int a = 0; a < KM; a++) {
            if (a >= k || outi[a] < 0) continue;
            const int la = labels[outi[a]];
            int cnt = 0;
#pragma unroll
            for (int b2 = 0; b2 < KM; b2++) cnt += b2 < k && outi[b2] >= 0 && labels[outi[b2]] == la;
            if (cnt > bestc || (cnt == bestc && la < best)) {
                bestc = cnt;
                best = la;
            }
        }
        pred[q] = best;
    }
}


// exhaustive fp64 for the queries the screen could not certify (fb_list[0 .. cnt)), in cand_less
// order like every other stage.  Two roles in one launch (no host round trip to learn cnt):
//  * blocks [0, nbp): the first FB_C listed queries, each query's reference rows cut into P parts
//    of prow rows, ONE WAVE per part: every lane keeps the KM smallest of its rows in registers,
//    the wave takes the part's k smallest by k rounds of a butterfly minimum (the winning lane
//    pops its head), writes them to the workspace, and the wave that finishes a query's last part
//    (a per-query counter, zeroed with the fallback count) merges the P lists the same way, one
//    lane per part.  Round 5 scanned a query with one workgroup: the 3 fallback queries of the
//    100k x 100k self-query on extracted features took 0.71-1.06 ms on 3 CUs.
//  * blocks [nbp, grid): the listed queries past FB_C (only when a launch has that many), one
//    workgroup per query: per-thread lists, then a tree merge through LDS.
static constexpr int FB_T = 256;
static constexpr int FB_C = 64;      // queries on the partitioned scan
static constexpr int FB_PMAX = 64;   // parts per query (one lane per part in the final merge)
static constexpr int FB_PROWS = 1024;  // target rows per part

// the smallest (d, i) over the wave in cand_less order, on every lane
__device__ __forceinline__ void wave_min_pair(double &d, int &i)
{
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        const double od = __shfl_xor(d, m, 64);
        const int oi = __shfl_xor(i, m, 64);
        if (cand_less(od, oi, d, i)) {
            d = od;
            i = oi;
        }
    }
}
// k rounds: the wave's k smallest of the lanes' ascending KM-lists (consumed); lane j < k returns
// the j-th in (od, oi)
template <int KM>
__device__ __forceinline__ void wave_take_k(double (&dl)[KM], int (&il)[KM], int k, int lane, double &od, int &oi)
{
    od = INFINITY;
    oi = 0x7fffffff;
    for (int j = 0; j < k; j++) {
        double d = dl[0];
        int i = il[0];
        wave_min_pair(d, i);
        if (lane == j) {
            od = d;
            oi = i;
        }
        if (dl[0] == d && il[0] == i && d < INFINITY) {  // this lane's head won: pop it
#pragma unroll
            for (int t = 0; t < KM - 1; t++) {
                dl[t] = dl[t + 1];
                il[t] = il[t + 1];
            }
            dl[KM - 1] = INFINITY;
            il[KM - 1] = 0x7fffffff;
        }
    }
}
// idx / dist / pred of query q from the k results held by lanes 0 .. k-1
template <int KM>
__device__ __forceinline__ void fb_write(int64_t q, int k, int lane, double od, int oi, const int32_t *labels,
                                         int32_t *idx, double *dist, int32_t *pred)
{
    const bool valid = od < INFINITY;
    if (lane < k) {
        idx[q * k + lane] = valid ? oi : -1;
        dist[q * k + lane] = valid ? sqrt(od) : INFINITY;
    }
    if (pred && labels) {
        const int lab = (lane < k && valid) ? labels[oi] : -1;
        int best = -1, bestc = 0;
#pragma unroll
        for (int a = 0; a < KM; a++) {
            if (a >= k) break;
            const int la = __shfl(lab, a, 64);
            if (la < 0) continue;
            int cnt = 0;
#pragma unroll
            for (int b2 = 0; b2 < KM; b2++)
                if (b2 < k) cnt += __shfl(lab, b2, 64) == la;
            if (cnt > bestc || (cnt == bestc && la < best)) {
                bestc = cnt;
                best = la;
            }
        }
        if (lane == 0) pred[q] = best;
    }
}

template <int KM>
__global__ __launch_bounds__(FB_T) void knn_fallback(const double *__restrict__ ref,
                                                     const double *__restrict__ query, int64_t Nr,
                                                     int D, int k, int64_t self_offset,
                                                     const int *fb_count, const int *fb_list,
                                                     const int32_t *__restrict__ labels,
                                                     int32_t *__restrict__ idx,
                                                     double *__restrict__ dist,
                                                     int32_t *__restrict__ pred, int P, int64_t prow, int nbp,
                                                     double *part_d, int *part_i, int *part_done)
{
    const int cnt = *fb_count;
    const int tid = threadIdx.x, lane = tid & 63;
    if ((int)blockIdx.x < nbp) {  // ---- partitioned scan of the first FB_C listed queries
        const int ncnt = min(cnt, FB_C);
        const int nw = nbp * (FB_T / 64);
        for (int u = (int)blockIdx.x * (FB_T / 64) + (tid >> 6); u < ncnt * P; u += nw) {
            const int item = u / P, part = u - item * P;
            const int64_t q = fb_list[item];
            const double *qx = query + q * D;
            const int64_t self = self_offset >= 0 ? self_offset + q : -1;
            const int64_t r0 = (int64_t)part * prow, r1 = min(Nr, r0 + prow);
            double dl[KM];
            int il[KM];
#pragma unroll
            for (int i = 0; i < KM; i++) {
                dl[i] = INFINITY;
                il[i] = 0x7fffffff;
            }
            if (D <= 16) {  // two rows in flight per lane, the query in registers (four: 55.7 against
                            // 46.6 us for the 3 fallbacks of the 100k self-query)
                const QRow16 q16 = qrow16(qx, D);
                for (int64_t r = r0 + lane; r < r1; r += 128) {
                    double b[2][16];
                    row16_load(b[0], ref + r * D, D);
                    row16_load(b[1], ref + (r + 64 < r1 ? r + 64 : r) * D, D);
                    if (r != self) topk_fixed_insert<KM>(dl, il, rdist64_16(q16, b[0], D), (int)r);
                    if (r + 64 < r1 && r + 64 != self) topk_fixed_insert<KM>(dl, il, rdist64_16(q16, b[1], D), (int)(r + 64));
                }
            } else {
                for (int64_t r = r0 + lane; r < r1; r += 64)
                    if (r != self) topk_fixed_insert<KM>(dl, il, rdist64(qx, ref + r * D, D), (int)r);
            }
            double od;
            int oi;
            wave_take_k<KM>(dl, il, k, lane, od, oi);
            const int64_t o = ((int64_t)item * P + part) * KM;
            if (lane < k) {
                part_d[o + lane] = od;
                part_i[o + lane] = oi;
            }
            __threadfence();  // the part's list is visible device-wide (all XCDs) before it is counted
            int last = 0;
            if (lane == 0) last = atomicAdd(&part_done[item], 1) == P - 1;
            if (!__shfl(last, 0, 64)) continue;
            __threadfence();  // acquire: every part's list, from whichever XCD wrote it
            // the final merge: lane p holds part p's ascending list
#pragma unroll
            for (int i = 0; i < KM; i++) {
                const bool in = lane < P && i < k;
                dl[i] = in ? part_d[((int64_t)item * P + lane) * KM + i] : INFINITY;
                il[i] = in ? part_i[((int64_t)item * P + lane) * KM + i] : 0x7fffffff;
            }
            wave_take_k<KM>(dl, il, k, lane, od, oi);
            fb_write<KM>(q, k, lane, od, oi, labels, idx, dist, pred);
        }
        return;
    }
    // ---- one workgroup per listed query past FB_C
    __shared__ double sd[FB_T / 2 * KM];
    __shared__ int si[FB_T / 2 * KM];
    const int nbo = (int)gridDim.x - nbp;
    for (int item = FB_C + (int)blockIdx.x - nbp; item < cnt; item += nbo) {
        const int64_t q = fb_list[item];
        const double *qx = query + q * D;
        const int64_t self = self_offset >= 0 ? self_offset + q : -1;
        double dl[KM];
        int il[KM];
#pragma unroll
        for (int i = 0; i < KM; i++) {
            dl[i] = INFINITY;
            il[i] = 0x7fffffff;
        }
        if (D <= 16) {
            const QRow16 q16 = qrow16(qx, D);
            for (int64_t r = tid; r < Nr; r += FB_T) {
                double b[16];
                row16_load(b, ref + r * D, D);
                if (r != self) topk_fixed_insert<KM>(dl, il, rdist64_16(q16, b, D), (int)r);
            }
        } else {
            for (int64_t r = tid; r < Nr; r += FB_T)
                if (r != self) topk_fixed_insert<KM>(dl, il, rdist64(qx, ref + r * D, D), (int)r);
        }
        // pairwise tree merge of the per-thread lists through LDS
        for (int width = FB_T; width > 1; width >>= 1) {
            const int half = width >> 1;
            __syncthreads();
            if (tid >= half && tid < width)
#pragma unroll
                for (int i = 0; i < KM; i++) {
                    sd[(tid - half) * KM + i] = dl[i];
                    si[(tid - half) * KM + i] = il[i];
                }
            __syncthreads();
            if (tid < half)
#pragma unroll
                for (int i = 0; i < KM; i++)
                    if (i < k) topk_fixed_insert<KM>(dl, il, sd[tid * KM + i], si[tid * KM + i]);
        }
        if (tid < 64) {  // wave 0: thread 0 holds the k smallest; spread them over lanes 0 .. k-1
            double od = INFINITY;
            int oi = 0x7fffffff;
#pragma unroll
            for (int i = 0; i < KM; i++) {
                const double d = __shfl(dl[i], 0, 64);
                const int ii = __shfl(il[i], 0, 64);
                if (lane == i) {
                    od = d;
                    oi = ii;
                }
            }
            fb_write<KM>(q, k, lane, od, oi, labels, idx, dist, pred);
        }
        __syncthreads();
    }
}

// ---- z-score (src/feature_extraction.py:157-181), numpy axis-0 order ---------------------
#pragma clang fp contract(off)
// numpy's axis-0 sums are sequential in row order per column, so each column is one dependent
// chain of fp64 adds; the kernel's job is to keep that chain fed.  One workgroup per ZS_C columns:
// waves 1-3 stage the next ZS_R-row tile of those columns in LDS (coalesced when the row is
// narrower than ZS_C) while lane c of wave 0 adds the current tile's column c in row order from
// LDS (reads issued ahead of the adds), then a barrier swaps the buffers.  Pass 0 sums x, pass 1
// (x - mean)^2.  Round 5 ran one thread per column with a dependent global load per row (46 ms
// for 100 000 x 15); one wave per column with lane_read 7.8 ms (v_readlane latency per add).
static constexpr int ZS_T = 256, ZS_R = 256, ZS_C = 16;
__global__ __launch_bounds__(ZS_T) void zscore_fit_kernel(const double *X, int64_t N, int D, double *mean, double *std)
{
    __shared__ double tile[2][ZS_R * ZS_C];
    const int c0 = (int)blockIdx.x * ZS_C, nc = min(ZS_C, D - c0), tid = threadIdx.x;
    const int64_t ntile = (N + ZS_R - 1) / ZS_R;
    // waves 1-3: rows [t ZS_R, +ZS_R) x columns [c0, c0 + nc), every load of the tile issued
    // before the first LDS store (a store waits for its load: one at a time, a tile cost ~7 us)
    constexpr int LPT = (ZS_R * ZS_C + ZS_T - 64 - 1) / (ZS_T - 64);
    auto load = [&](int64_t t, int buf) {
        double v[LPT];
#pragma unroll
        for (int u = 0; u < LPT; u++) {
            const int e = tid - 64 + u * (ZS_T - 64);
            const int r = e / nc, c = e - r * nc;
            const int64_t row = t * ZS_R + r;
            v[u] = (e < ZS_R * nc && row < N) ? X[row * D + c0 + c] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < LPT; u++) {
            const int e = tid - 64 + u * (ZS_T - 64);
            const int r = e / nc, c = e - r * nc;
            if (e < ZS_R * nc) tile[buf][r * ZS_C + c] = v[u];
        }
    };
    double m = 0.0, acc = 0.0;
    for (int pass = 0; pass < 2; pass++) {
        acc = 0.0;
        if (tid >= 64) load(0, 0);
        __syncthreads();
        for (int64_t t = 0; t < ntile; t++) {
            const int buf = (int)(t & 1);
            if (tid >= 64) {
                if (t + 1 < ntile) load(t + 1, buf ^ 1);
            } else if (tid < nc) {
                const int rows = (int)min((int64_t)ZS_R, N - t * ZS_R);
                const double *col = tile[buf] + tid;
                // batches of 16 rows: 16 LDS reads, then 16 adds (each waits only for its own read).
                // Reading the next batch before this batch's adds measured slower: 16 ahead 4.16
                // ms, 8 ahead 4.22 ms, against 2.69 ms (100 000 x 15, profiles/r06i/j/z)
                int r = 0;
                for (; r + 16 <= rows; r += 16) {
                    double v[16];
#pragma unroll
                    for (int u = 0; u < 16; u++) v[u] = col[(r + u) * ZS_C];
#pragma unroll
                    for (int u = 0; u < 16; u++) {
                        if (pass == 0) {
                            acc = acc + v[u];
                        } else {
                            const double x = v[u] - m;
                            acc = acc + x * x;
                        }
                    }
                }
                for (; r < rows; r++) {
                    if (pass == 0) {
                        acc = acc + col[r * ZS_C];
                    } else {
                        const double x = col[r * ZS_C] - m;
                        acc = acc + x * x;
                    }
                }
            }
            __syncthreads();
        }
        if (pass == 0) m = acc / (double)N;
    }
    if (tid < nc) {
        const double sd = sqrt(acc / (double)N);
        mean[c0 + tid] = m;
        std[c0 + tid] = sd == 0.0 ? 1.0 : sd;
    }
}

__global__ void zscore_apply_kernel(const double *X, int64_t N, int D, const double *mean,
                                    const double *std, double *out)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N * D) return;
    const int c = (int)(e % D);
    out[e] = (X[e] - mean[c]) / std[c];
}
#pragma clang fp contract(on)

}  // namespace dsp

// ------------------------------------------------------------------------------------------
namespace {
struct KnnLayout {
    size_t ref32, refmx, q32, cand_d, cand_i, misc, fb_d, fb_i, pilot_d, seed0, seed, total;
    int fb_parts, fb_km;  // partitioned fallback: parts per query, list length
    int DP, KC, nsplit;
    int rstride, nsample, nsplit_p;  // seeded thresholds (rstride > 0): sample rows j * rstride
    int rstride0, nsample0, nsplit_p0;  // the pilot's own seed: a smaller sample (rows j * rstride0)
    bool exp;  // expanded-form screening (a spare padded column holds |r|^2)
    bool hd;   // D > 32: chunked direct-form screen (knn_screen_hd)
    bool mfma; // expanded form on the matrix cores (knn_screen_mfma)
};

static constexpr int KNN_DMAX = 4096;
// seeded thresholds: a pilot over ~KNN_SEED_SAMPLE strided rows when the set has >= KNN_SEED_MIN_NR.
// Round 5: the pilot keeps class minima (knn_pilot_mfma) instead of top-KC lists -- at 4 096 rows
// 84.8 -> 31.5 us at 12.5k queries, 409 -> 197 us at 100k, whole job 0.795-0.807 -> 0.738-0.757 ms
// and 4.46-4.54 -> 4.27 ms (profiles/r05k2_knn_ab.txt) -- and the cheaper pilot affords a larger
// sample: 2 048 / 4 096 / 8 192 / 16 384 rows 0.81-0.83 / 0.76 / 0.716-0.721 / 0.73-0.74 ms at 12.5k,
// 4.45-4.48 / 4.27-4.30 / 4.15-4.20 / 4.30-4.34 ms at 100k (profiles/r05k2_pilot_sweep.txt).
// A pre-pilot over ~KNN_SEED_SAMPLE0 rows can seed the list pilot (KNN_PILOT_MIN 0) itself (0:
// none).  Round 5's sweep of the list pilot (profiles/r05_knn_pilot_sweep.txt): 0:4096 0.783 /
// 4.41 ms, 256:4096 0.786-0.796 / 4.48, 512:8192 0.783-0.792 / 4.47: no gain.
#ifndef KNN_PILOT_MIN
#define KNN_PILOT_MIN 1  // the pilot keeps class minima (knn_pilot_mfma); 0: top-KC lists (A/B)
#endif
#ifndef KNN_SEED_SAMPLE
#define KNN_SEED_SAMPLE 8192
#endif
#ifndef KNN_SEED_SAMPLE0
#define KNN_SEED_SAMPLE0 0
#endif
#ifndef KNN_SEED_MIN_NR
#define KNN_SEED_MIN_NR 32768
#endif
#ifndef KNN_SEED_WARM
#define KNN_SEED_WARM 1024.0
#endif
#ifndef KNN_SEED_SAT
#define KNN_SEED_SAT 16
#endif

int pick_kc(int k)
{
    const int need = k + dsp::KNN_SLACK;
    if (need <= 8) return 8;
    if (need <= 16) return 16;
    if (need <= 24) return 24;
    return 36;
}

// MFMA screen: reference splits.  Every workgroup of the grid is resident at once, so a CU's time
// is (rows per split + a split's list warm-up W) x its waves, and a CU saturates at `sat` waves:
// T(s) = (Nr / s + W) * max(waves on the busiest CU, sat).  From a threshold at +inf, W ~ 16k rows
// and two waves per SIMD saturate (sat 8); from a seeded threshold W ~ 1k rows, and a step then
// inserts so rarely that the steps' dependency chains need four waves per SIMD to hide (sat 16):
// 12.5k x 100k forced splits 4 / 6 / 8 / 10 / 12 / 16 / 20 measured 1.08 / 1.00 / 0.97 / 0.86 /
// 0.87 / 0.91 / 0.88 ms (profiles/r04_knn_split_sweep.txt).
int pick_nsplit_mfma(int64_t Nr, int64_t Nq, int qpb, int cus, double warm = 16384.0, int sat = 8)
{
    const int64_t qblocks = (Nq + qpb - 1) / qpb;
    const int64_t maxs = std::max<int64_t>(1, std::min<int64_t>(64, (Nr + dsp::MQ_TR - 1) / dsp::MQ_TR));
    int best = 1;
    double best_t = 1e300;
    for (int64_t s = 1; s <= maxs; s++) {
        const int64_t waves = (qblocks * s + cus - 1) / cus * dsp::MQ_W;
        const double t = ((double)Nr / (double)s + warm) * (double)std::max<int64_t>(waves, sat);
        if (t < best_t * (1.0 - 1e-9)) {
            best_t = t;
            best = (int)s;
        }
    }
    return best;
}

int pick_nsplit(int64_t Nr, int64_t Nq, int qpb)
{
    const int64_t qblocks = (Nq + qpb - 1) / qpb;
    // Enough workgroups to fill the chip (two per CU), as few reference splits as that allows:
    // a longer split makes a screened distance that enters its top list rarer (~KC / rows seen),
    // and a wave pays for an insertion whenever any of its 64 lanes makes one
#ifdef DSP_KNN_DIAG  // diagnostic build only (tools/knn_split_sweep.sh): launch-shape override
    static const int target = [] {
        const char *e = getenv("DSP_KNN_TARGET_WGS");
        return e ? atoi(e) : 512;
    }();
#else
    constexpr int target = 512;
#endif
    int64_t s = (target + qblocks - 1) / qblocks;
    const int64_t maxs = (Nr + dsp::KNN_TR - 1) / dsp::KNN_TR;  // >= one tile per split
    if (s > maxs) s = maxs;
    if (s > 64) s = 64;
    if (s < 1) s = 1;
    return (int)s;
}

size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// CUs of the current device, cached
int device_cus()
{
    static int cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
        cache[dev] = cus;
    }
    return cache[dev];
}

KnnLayout knn_layout(int64_t Nr, int64_t Nq, int D, int k)
{
    KnnLayout l;
    l.hd = D > 32;
    l.DP = D <= 16 ? 16 : D <= 32 ? 32 : (D + 15) & ~15;
    l.exp = !l.hd && D < l.DP;
    l.KC = pick_kc(k);
    l.mfma = l.exp;  // every expanded-form screen runs on the matrix cores

    // seeded thresholds (matrix-core screen, reference sets of >= KNN_SEED_MIN_NR rows): a pilot
    // screen over every rstride-th row (~KNN_SEED_SAMPLE rows) seeds each query's threshold
    l.rstride = l.rstride0 = 0;
    l.nsample = l.nsample0 = 0;
    l.nsplit_p = l.nsplit_p0 = 0;
    if (l.mfma && Nr >= KNN_SEED_MIN_NR) {
        int64_t samp = KNN_SEED_SAMPLE, samp0 = KNN_SEED_SAMPLE0;
#ifdef DSP_KNN_DIAG  // diagnostic build only: pilot sample sizes (tools/r05_knn_pilot.sh)
        if (const char *e = getenv("DSP_KNN_SAMPLE")) samp = std::max(64, atoi(e));
        if (const char *e = getenv("DSP_KNN_SAMPLE0")) samp0 = std::max(0, atoi(e));
#endif
        l.rstride = (int)std::max<int64_t>(2, Nr / samp);
        l.nsample = (int)((Nr + l.rstride - 1) / l.rstride);
        if (samp0 > 0) {
            l.rstride0 = (int)std::max<int64_t>(2, Nr / samp0);
            l.nsample0 = (int)((Nr + l.rstride0 - 1) / l.rstride0);
        }
    }
#ifdef DSP_KNN_DIAG  // diagnostic build only: seeding off (DSP_KNN_SEED=0)
    if (const char *e = getenv("DSP_KNN_SEED"))
        if (atoi(e) == 0) l.rstride = l.nsample = 0;
#endif
    l.nsplit = l.mfma ? pick_nsplit_mfma(Nr, Nq, dsp::mq_qpb(l.KC), device_cus(),
                                         l.rstride ? KNN_SEED_WARM : 16384.0, l.rstride ? KNN_SEED_SAT : 8)
                      : pick_nsplit(Nr, Nq, l.hd ? dsp::KNN_TQ : dsp::KNN_TQ * dsp::KNN_QP);
#ifdef DSP_KNN_DIAG  // diagnostic build only: forced split count (tools/knn_split_sweep.sh)
    if (const char *e = getenv("DSP_KNN_NSPLIT")) l.nsplit = std::max(1, std::min(64, atoi(e)));
#endif
#if KNN_MFMA_KC6
    // matrix-core screen over short splits (<= 32k rows), k <= 5: six candidates per split
    // (slack 1 instead of 3).  A short split's cost is mostly its list warm-up, and a shorter list
    // inserts less often and more cheaply (12.5k x 100k, 5 splits of 20k rows: 1.19 -> 1.05 ms);
    // over long splits the longer list measured faster (100k x 100k, 2 splits of 50k rows: 5.58
    // against 6.06 ms) and stays.  Same tiles per wave (mq_tiles): the split count is unchanged.
    if (l.mfma && k <= 5 && (Nr + l.nsplit - 1) / l.nsplit <= 32768) l.KC = 6;
#endif
    size_t o = 0;
    // the converted reference set and its max row norm first, at offsets that depend on (Nr, D)
    // only: a workspace reused for the same reference set keeps them (DSP_KNN_REF_READY)
    l.ref32 = o; o += al((size_t)Nr * l.DP * 4);
    l.refmx = o; o += al(4);
    l.q32 = o;   o += al((size_t)Nq * l.DP * 4);
    l.cand_d = o; o += al((size_t)l.nsplit * Nq * l.KC * 4);
    l.cand_i = o; o += al((size_t)l.nsplit * Nq * l.KC * 4);
    // (unused), fallback count, 2 words (unused), the per-query part counters of the partitioned
    // fallback (FB_C words, zeroed with the count), the fallback list
    l.misc = o;  o += al(16 + 4 * (size_t)dsp::FB_C + (size_t)Nq * 4);
    l.fb_parts = (int)std::max<int64_t>(1, std::min<int64_t>(dsp::FB_PMAX, (Nr + dsp::FB_PROWS - 1) / dsp::FB_PROWS));
    l.fb_km = k <= 8 ? 8 : k <= 16 ? 16 : 32;
    {
        const size_t nfb = (size_t)std::min<int64_t>(Nq, dsp::FB_C) * l.fb_parts * l.fb_km;
        l.fb_d = o; o += al(nfb * 8);
        l.fb_i = o; o += al(nfb * 4);
    }
    l.pilot_d = l.seed0 = l.seed = 0;
    if (l.rstride) {
        // pilot splits: enough workgroups to fill the chip twice over, >= one tile of rows each
        const int64_t qblocks = (Nq + dsp::mq_qpb(l.KC) - 1) / dsp::mq_qpb(l.KC);
        l.nsplit_p = (int)std::max<int64_t>(1, std::min<int64_t>({(2 * device_cus() + qblocks - 1) / qblocks,
                                                                  (l.nsample + dsp::MQ_TR - 1) / dsp::MQ_TR, 64}));
        // the pre-pilot: splits of >= 64 sample rows, at most the pilot's count
        l.nsplit_p0 = (int)std::max<int64_t>(1, std::min<int64_t>(l.nsplit_p, l.nsample0 / 64));
        l.pilot_d = o; o += al((size_t)l.nsplit_p * Nq * std::max(l.KC, dsp::PIL_CLS) * 4);
        l.seed0 = o;   o += al((size_t)Nq * 4);
        l.seed = o;    o += al((size_t)Nq * 4);
    }
    l.total = o;
    return l;
}

template <int DP, int KC>
void launch_screen(dim3 g, hipStream_t s, const float *r, int64_t Nr, const float *q, int64_t Nq, int64_t self,
                   int nsplit, float *cd, int *ci)
{
    hipLaunchKernelGGL((dsp::knn_screen<DP, KC, dsp::KNN_QP>), g, dim3(dsp::KNN_TQ), 0, s, r, Nr, q, Nq,
                       self, nsplit, cd, ci);
}

// returns false when no merge kernel covers (KC, k): the layout broke KC >= k + KNN_SLACK
template <int KC>
bool launch_merge(hipStream_t s, const double *ref, const double *query, int64_t Nr, int64_t Nq, int D, int k,
                  int nsplit, int64_t self, const float *cd, const int *ci, const unsigned *mx, double er,
                  double ea, const int32_t *lbl, int32_t *idx, double *dist, int32_t *pred, int *fbc, int *fbl,
                  const float *seed)
{
    // 64-thread workgroups, MG lanes per query: 12 500 queries (one rank of the 8-GPU self-query)
    // are 1 563 of them
    const dim3 g((unsigned)((Nq * dsp::MG + 63) / 64)), b(64);
    // KC >= k + KNN_SLACK, so KC = 8 implies k <= 8 and KC = 16 implies k <= 16
    if (k > KC) return false;
    if (k <= 8) {
        hipLaunchKernelGGL((dsp::knn_merge<KC, 8>), g, b, 0, s, ref, query, Nr, Nq, D, k, nsplit, self, cd, ci, mx,
                           er, ea, lbl, idx, dist, pred, fbc, fbl, seed);
        return true;
    }
    const dim3 g1((unsigned)((Nq + 63) / 64));  // one thread per query (k > 8)
    if constexpr (KC >= 16) {
        if (k <= 16) {
            hipLaunchKernelGGL((dsp::knn_merge1<KC, 16>), g1, b, 0, s, ref, query, Nr, Nq, D, k, nsplit, self, cd,
                               ci, mx, er, ea, lbl, idx, dist, pred, fbc, fbl, seed);
            return true;
        }
    }
    if constexpr (KC >= 24) {
        hipLaunchKernelGGL((dsp::knn_merge1<KC, 32>), g1, b, 0, s, ref, query, Nr, Nq, D, k, nsplit, self, cd, ci,
                           mx, er, ea, lbl, idx, dist, pred, fbc, fbl, seed);
        return true;
    }
    return false;
}

// err(d) = er * d + ea * (|q|^2 + max |r|^2) bounds |fp32 screened - fp64| distance.
//  * D <= 32, expanded form |q|^2 + q'.r' (or direct form at D = 16 / 32): <= 16 FMA roundings of
//    partial sums bounded by 2 (|q|^2 + |r|^2), plus the fp32 rounding of the inputs.  The MFMA
//    form without assuming fma-chain equivalence: each of the DP / 4 blocks adds 4 products to
//    the accumulator in any order, <= 1 rounding per product and per addition (5 per block), every
//    partial sum bounded by |q|^2 + sum |q'_j r'_j| <= 2 (|q|^2 + |r|^2); over 4 blocks
//    20 u * 2 (|q|^2 + |r|^2) = 40u (...), plus 4u (...) for the inputs: 44u = 2.7e-6 < ea = 4e-6
//    at DP = 16; at DP = 32 (8 blocks) 84u = 5.0e-6 < ea = 8e-6 (u = 2^-24);
//  * D > 32, direct form: D sequential FMAs of non-negative terms, each (q - r) rounded once:
//    relative (D + 3) u on the sum, plus 4 u (|q|^2 + |r|^2) from the inputs (u = 2^-24); 2x margin.
void knn_err_coeffs(const KnnLayout &l, int D, double &er, double &ea)
{
    if (!l.hd) {
        er = 2e-6;
        ea = l.DP <= 16 ? 4e-6 : 8e-6;
    } else {
        const double u = 1.0 / 16777216.0;
        er = 2.0 * (D + 3) * u * 1.05;
        ea = 2.0 * 4.2 * u;
    }
}
}  // namespace

extern "C" size_t dsp_knn_workspace_bytes(int64_t Nr, int64_t Nq, int D, int k)
{
    if (Nr < 0 || Nq < 0 || D < 1 || D > KNN_DMAX || k < 1 || k > 32) return 0;
    return knn_layout(Nr, Nq, D, k).total;
}

extern "C" size_t dsp_knn_workspace_fallbacks_offset(int64_t Nr, int64_t Nq, int D, int k)
{
    if (Nr < 0 || Nq < 0 || D < 1 || D > KNN_DMAX || k < 1 || k > 32) return 0;
    return knn_layout(Nr, Nq, D, k).misc + 4;
}

extern "C" int dsp_knn_classify(const double *ref, const int32_t *ref_labels, int64_t Nr,
                                const double *query, int64_t Nq, int D, int k, int64_t self_offset,
                                int n_classes, int32_t *idx, double *dist, int32_t *pred,
                                void *workspace, size_t workspace_bytes, int flags, void *stream)
{
    if (D < 1 || D > KNN_DMAX || k < 1 || k > dsp::KMAX || Nr < 0 || Nq < 0) return DSP_ERR_ARGS;
    if (Nr > 0x7fffffff || (Nq > 0 && (!query || !idx || !dist)) || (Nr > 0 && !ref))
        return DSP_ERR_ARGS;
    if (Nq == 0) return DSP_OK;
    (void)n_classes;
    const KnnLayout l = knn_layout(Nr, Nq, D, k);
    if (!workspace || workspace_bytes < l.total) return DSP_ERR_WORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    char *ws = (char *)workspace;
    float *ref32 = (float *)(ws + l.ref32);
    float *q32 = (float *)(ws + l.q32);
    float *cd = (float *)(ws + l.cand_d);
    int *ci = (int *)(ws + l.cand_i);
    unsigned *mx = (unsigned *)(ws + l.refmx);
    int *fbc = (int *)(ws + l.misc + 4);
    int *fbdone = (int *)(ws + l.misc + 16);
    int *fbl = (int *)(ws + l.misc + 16 + 4 * dsp::FB_C);
    float *seedp = l.rstride ? (float *)(ws + l.seed) : nullptr;
    if (hipMemsetAsync(ws + l.misc, 0, 16 + 4 * dsp::FB_C, s) != hipSuccess) return DSP_ERR_HIP;
    const int cb = 256;
    if (Nr > 0 && !(flags & DSP_KNN_REF_READY)) {  // (fit: the reference set in fp32 + its max norm)
        if (hipMemsetAsync(mx, 0, 4, s) != hipSuccess) return DSP_ERR_HIP;
        hipLaunchKernelGGL(dsp::knn_convert, dim3((unsigned)((Nr + cb - 1) / cb)), dim3(cb), 0, s,
                           ref, Nr, D, l.DP, l.exp ? 1 : 0, ref32, mx);
    }
    hipLaunchKernelGGL(dsp::knn_convert, dim3((unsigned)((Nq + cb - 1) / cb)), dim3(cb), 0, s,
                       query, Nq, D, l.DP, l.exp ? 2 : 0, q32, (unsigned *)nullptr);
    if (l.hd) {
        const dim3 g((unsigned)((Nq + dsp::KNN_TQ - 1) / dsp::KNN_TQ), (unsigned)l.nsplit);
        switch (l.KC) {
#define DSP_SCREEN_HD(KCV)                                                                        \
    case KCV:                                                                                     \
        hipLaunchKernelGGL((dsp::knn_screen_hd<KCV>), g, dim3(dsp::KNN_TQ), 0, s, ref32, Nr, q32, Nq, \
                           l.DP, self_offset, l.nsplit, cd, ci);                                  \
        break
            DSP_SCREEN_HD(8); DSP_SCREEN_HD(16); DSP_SCREEN_HD(24); DSP_SCREEN_HD(36);
#undef DSP_SCREEN_HD
        }
    } else if (l.mfma) {
        const int qpb = dsp::mq_qpb(l.KC);
        const unsigned qb = (unsigned)((Nq + qpb - 1) / qpb);
        const dim3 b(64 * dsp::MQ_W);
#define DSP_SCREEN_MQ(DPV, KCV, PIL, G, NR, NS, CD, CI, RSTR, SEED)                                \
    if (l.DP == DPV && l.KC == KCV)                                                               \
    hipLaunchKernelGGL((dsp::knn_screen_mfma<DPV, KCV, PIL>), G, b, 0, s, ref32, NR, q32, Nq, self_offset, NS, \
                       CD, CI, RSTR, SEED)
#define DSP_SCREEN_MQ_ALL(...)                                                                    \
        DSP_SCREEN_MQ(16, 8, __VA_ARGS__); DSP_SCREEN_MQ(16, 16, __VA_ARGS__); DSP_SCREEN_MQ(16, 24, __VA_ARGS__); \
        DSP_SCREEN_MQ(16, 36, __VA_ARGS__); DSP_SCREEN_MQ(32, 8, __VA_ARGS__); DSP_SCREEN_MQ(32, 16, __VA_ARGS__); \
        DSP_SCREEN_MQ(32, 24, __VA_ARGS__); DSP_SCREEN_MQ(32, 36, __VA_ARGS__); DSP_SCREEN_MQ(16, 6, __VA_ARGS__); \
        DSP_SCREEN_MQ(32, 6, __VA_ARGS__)
        if (l.rstride) {
            float seed_scale = 1.f;
#ifdef DSP_KNN_DIAG  // diagnostic build only: an adversarially tight seed (fallback tests)
            if (const char *e = getenv("DSP_KNN_SEED_SCALE")) seed_scale = (float)atof(e);
#endif
            // pilots over the sampled rows (same kernel, same fp32 arithmetic): a pre-pilot over
            // nsample0 rows from +inf thresholds seeds the pilot over nsample rows, whose seeds
            // start the main screen
            float *pd = (float *)(ws + l.pilot_d);
            float *seed0 = (float *)(ws + l.seed0);
            const dim3 gs((unsigned)((Nq + 255) / 256));
            auto seeds = [&](int nsp, const float *prev, float *out, float scale) {
                switch (l.KC) {
                case 6: hipLaunchKernelGGL((dsp::knn_seed<6>), gs, dim3(256), 0, s, pd, nsp, Nq, prev, out, scale); break;
                case 8: hipLaunchKernelGGL((dsp::knn_seed<8>), gs, dim3(256), 0, s, pd, nsp, Nq, prev, out, scale); break;
                case 16: hipLaunchKernelGGL((dsp::knn_seed<16>), gs, dim3(256), 0, s, pd, nsp, Nq, prev, out, scale); break;
                case 24: hipLaunchKernelGGL((dsp::knn_seed<24>), gs, dim3(256), 0, s, pd, nsp, Nq, prev, out, scale); break;
                default: hipLaunchKernelGGL((dsp::knn_seed<36>), gs, dim3(256), 0, s, pd, nsp, Nq, prev, out, scale); break;
                }
            };
            const dim3 gp0(qb, (unsigned)l.nsplit_p0), gp(qb, (unsigned)l.nsplit_p);
            if (KNN_PILOT_MIN) {
                constexpr int pqpb = 16 * KNN_MQ_T * dsp::MQ_W;
                const dim3 gpm((unsigned)((Nq + pqpb - 1) / pqpb), (unsigned)l.nsplit_p);
                if (l.DP == 16)
                    hipLaunchKernelGGL((dsp::knn_pilot_mfma<16>), gpm, b, 0, s, ref32, (int64_t)l.nsample, q32, Nq,
                                       self_offset, l.nsplit_p, pd, l.rstride);
                else
                    hipLaunchKernelGGL((dsp::knn_pilot_mfma<32>), gpm, b, 0, s, ref32, (int64_t)l.nsample, q32, Nq,
                                       self_offset, l.nsplit_p, pd, l.rstride);
                switch (l.KC) {
#define DSP_SEED_MIN(KCV)                                                                                   \
    case KCV:                                                                                               \
        hipLaunchKernelGGL((dsp::knn_seed<KCV, dsp::PIL_CLS>), gs, dim3(256), 0, s, pd, l.nsplit_p, Nq,       \
                           (const float *)nullptr, seedp, seed_scale);                                        \
        break
                    DSP_SEED_MIN(6); DSP_SEED_MIN(8); DSP_SEED_MIN(16); DSP_SEED_MIN(24); DSP_SEED_MIN(36);
#undef DSP_SEED_MIN
                }
            } else {
            if (l.rstride0) {
                DSP_SCREEN_MQ_ALL(true, gp0, (int64_t)l.nsample0, l.nsplit_p0, pd, (int *)nullptr, l.rstride0,
                                  (const float *)nullptr);
                seeds(l.nsplit_p0, nullptr, seed0, 1.f);
            }
            DSP_SCREEN_MQ_ALL(true, gp, (int64_t)l.nsample, l.nsplit_p, pd, (int *)nullptr, l.rstride,
                              (const float *)(l.rstride0 ? seed0 : nullptr));
            seeds(l.nsplit_p, l.rstride0 ? seed0 : nullptr, seedp, seed_scale);
            }
        }
        const dim3 g(qb, (unsigned)l.nsplit);
        DSP_SCREEN_MQ_ALL(false, g, Nr, l.nsplit, cd, ci, 1, (const float *)seedp);
#undef DSP_SCREEN_MQ_ALL
#undef DSP_SCREEN_MQ
    } else {
        const dim3 g((unsigned)((Nq + dsp::KNN_TQ * dsp::KNN_QP - 1) / (dsp::KNN_TQ * dsp::KNN_QP)), (unsigned)l.nsplit);
#define DSP_SCREEN(DPV, KCV)                                                                  \
    if (l.DP == DPV && l.KC == KCV) launch_screen<DPV, KCV>(g, s, ref32, Nr, q32, Nq, self_offset, \
                                                            l.nsplit, cd, ci)
        DSP_SCREEN(16, 8); DSP_SCREEN(16, 16); DSP_SCREEN(16, 24); DSP_SCREEN(16, 36);
        DSP_SCREEN(32, 8); DSP_SCREEN(32, 16); DSP_SCREEN(32, 24); DSP_SCREEN(32, 36);
#undef DSP_SCREEN
    }
    double er, ea;
    knn_err_coeffs(l, D, er, ea);
    const int32_t *lbl = pred ? ref_labels : nullptr;
    bool merged = false;
    switch (l.KC) {
#if KNN_MFMA_KC6
    case 6: merged = launch_merge<6>(s, ref, query, Nr, Nq, D, k, l.nsplit, self_offset, cd, ci, mx, er, ea, lbl, idx, dist, pred, fbc, fbl, seedp); break;
#endif
    case 8: merged = launch_merge<8>(s, ref, query, Nr, Nq, D, k, l.nsplit, self_offset, cd, ci, mx, er, ea, lbl, idx, dist, pred, fbc, fbl, seedp); break;
    case 16: merged = launch_merge<16>(s, ref, query, Nr, Nq, D, k, l.nsplit, self_offset, cd, ci, mx, er, ea, lbl, idx, dist, pred, fbc, fbl, seedp); break;
    case 24: merged = launch_merge<24>(s, ref, query, Nr, Nq, D, k, l.nsplit, self_offset, cd, ci, mx, er, ea, lbl, idx, dist, pred, fbc, fbl, seedp); break;
    default: merged = launch_merge<36>(s, ref, query, Nr, Nq, D, k, l.nsplit, self_offset, cd, ci, mx, er, ea, lbl, idx, dist, pred, fbc, fbl, seedp); break;
    }
    if (!merged) return DSP_ERR_ARGS;  // unreachable while KC >= k + KNN_SLACK (knn_layout)
    {
        // partitioned role: enough waves for every part of FB_C queries, at most 1 024 (most
        // launches list no query and these workgroups return at once); the per-workgroup role only
        // when this launch can list more than FB_C queries
        const int P = l.fb_parts;
        const int64_t prow = (Nr + P - 1) / P;
        const int nbp = (int)std::min<int64_t>(256, ((int64_t)std::min<int64_t>(Nq, dsp::FB_C) * P + 3) / 4);
        const int nbo = Nq > dsp::FB_C ? (int)std::min<int64_t>(512, Nq - dsp::FB_C) : 0;
        double *fbd = (double *)(ws + l.fb_d);
        int *fbi = (int *)(ws + l.fb_i);
#define DSP_FB(KMV)                                                                                              \
    hipLaunchKernelGGL((dsp::knn_fallback<KMV>), dim3((unsigned)(nbp + nbo)), dim3(dsp::FB_T), 0, s, ref, query, Nr, \
                       D, k, self_offset, fbc, fbl, lbl, idx, dist, pred, P, prow, nbp, fbd, fbi, fbdone)
        if (l.fb_km == 8) DSP_FB(8); else if (l.fb_km == 16) DSP_FB(16); else DSP_FB(32);
#undef DSP_FB
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? DSP_OK : DSP_ERR_HIP + (int)e;
}

extern "C" int dsp_zscore_fit(const double *X, int64_t N, int D, double *mean, double *std,
                              void *stream)
{
    if (!X || !mean || !std || N < 1 || D < 1) return DSP_ERR_ARGS;
    hipLaunchKernelGGL(dsp::zscore_fit_kernel, dim3((unsigned)((D + dsp::ZS_C - 1) / dsp::ZS_C)), dim3(dsp::ZS_T), 0,
                       (hipStream_t)stream, X, N, D, mean, std);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? DSP_OK : DSP_ERR_HIP + (int)e;
}

extern "C" int dsp_zscore_apply(const double *X, int64_t N, int D, const double *mean,
                                const double *std, double *out, void *stream)
{
    if (!X || !mean || !std || !out || N < 0 || D < 1) return DSP_ERR_ARGS;
    if (N == 0) return DSP_OK;
    const int64_t tot = N * D;
    hipLaunchKernelGGL(dsp::zscore_apply_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, X, N, D, mean, std, out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? DSP_OK : DSP_ERR_HIP + (int)e;
}

extern "C" int dsp_abi_version(void) { return DSP_ABI_VERSION; }
