// extract.hip -- fused per-clip feature extraction for gfx950 (CDNA4).
//
// One 1024-thread workgroup owns one clip.  The clip (int16) is streamed from HBM once
// with 16-byte loads into LDS; every later pass (clip statistics, sign bits, endpoint
// energies, windowed frames, per-frame statistics) runs out of LDS, so the algorithmic
// HBM traffic is 2 B/sample in + 72 B/clip out.
//
// Reference functions restated (Hypersonic-cpu/DSP-AudioRecLabs):
//   preprocess            src/audio_processing.py:78-90
//   endpoint_detection    src/audio_processing.py:135-275
//   frame_signal          src/audio_processing.py:299-333
//   extract_frame_features src/feature_extraction.py:12-43
//   compute_statistics / extract_statistical_features src/feature_extraction.py:46-88
//
// Exactness plan:
//   * mean / peak: exact from integer sums (the reference's float64 mean of k/32768 is exact,
//     so mq = fl(K/n) and M' = max(fl(kmax-mq), fl(mq-kmin)) reproduce it bit for bit).
//   * signs and every ZCR: pure integer (k >= floor(mq)+1), bit-exact.
//   * endpoint energies: exact integer moments per frame -> fp64 (rel. err ~1e-15); every
//     threshold decision is certified against a 1e-11 margin and, if any is a near tie, the
//     energies are recomputed in numpy's exact float64 order (pairwise_sum) -- so start/end
//     are always the reference's.
//   * windowed E/M: fp32 on VALU (tolerance 1e-5 rel., measured ~2e-7); stats in fp64.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dsp_audiorec.h"
#include "extract_layout.h"

namespace dsp {

static constexpr int NT = EXTRACT_THREADS;
static constexpr int NWAVE = NT / 64;

struct ExtractParams {
    const int16_t *pcm;
    const int64_t *offsets;
    int B, ncap, L, S;
    const double *window;
    int do_vad;
    double hi, lo, zr;
    float *feat;
    int32_t *start_end, *n_frames, *status;
    double *vad_energy;
    int32_t *vad_zcr;
    int ld_vad;
    float *seq;
    int ld_seq;
};

typedef short short8 __attribute__((ext_vector_type(8)));

template <typename T>
__device__ __forceinline__ T wave_sum(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int wave_min(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_maxd(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_mind(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}

// ------------------------------------------------------------------------------------------
// numpy float64 summation order (pairwise_sum, 8192-element buffered chunks) -- used only on
// the certified-exact endpoint path.  Value i of the summed array is x_i^2 with
// x_i = fl(fl(k_i - mq) / M') (or k_i - mq when M' == 0), i.e. the reference's
// frame ** 2 (src/audio_processing.py:103) on preprocess()'s output.
// ------------------------------------------------------------------------------------------
#pragma clang fp contract(off)
__device__ __noinline__ double xsq(const int16_t *clip, int i, double mq, double Mp)
{
    double d = (double)clip[i] - mq;
    double x = Mp > 0.0 ? d / Mp : d;
    return x * x;
}

__device__ __noinline__ double pw_leaf(const int16_t *clip, int lo, int n, double mq, double Mp)
{
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; i++) res += xsq(clip, lo + i, mq, Mp);
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = xsq(clip, lo + j, mq, Mp);
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += xsq(clip, lo + i + j, mq, Mp);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += xsq(clip, lo + i, mq, Mp);
    return res;
}

// iterative restatement of numpy's recursive pairwise_sum over [lo, lo+n), n <= 8192
__device__ __noinline__ double pw_block(const int16_t *clip, int lo, int n, double mq, double Mp)
{
    int s_lo[16], s_n[16], s_stage[16];
    double s_left[16];
    int sp = 0;
    s_lo[0] = lo;
    s_n[0] = n;
    s_stage[0] = 0;
    double ret = 0.0;
    bool have = false;
    for (;;) {
        if (!have) {
            int cl = s_lo[sp], cn = s_n[sp];
            if (cn <= 128) {
                ret = pw_leaf(clip, cl, cn, mq, Mp);
                have = true;
            } else {
                int n2 = cn / 2;
                n2 -= n2 % 8;
                s_stage[sp] = 1;
                sp++;
                s_lo[sp] = cl;
                s_n[sp] = n2;
                s_stage[sp] = 0;
                continue;
            }
        }
        if (sp == 0) return ret;
        sp--;
        int pl = s_lo[sp], pn = s_n[sp];
        int n2 = pn / 2;
        n2 -= n2 % 8;
        if (s_stage[sp] == 1) {
            s_left[sp] = ret;
            s_stage[sp] = 2;
            sp++;
            s_lo[sp] = pl + n2;
            s_n[sp] = pn - n2;
            s_stage[sp] = 0;
            have = false;
        } else {
            ret = s_left[sp] + ret;
        }
    }
}

__device__ __noinline__ double np_energy_exact(const int16_t *clip, int lo, int n, double mq, double Mp)
{
    double total = 0.0;
    for (int c = 0; c < n; c += 8192) total += pw_block(clip, lo + c, min(8192, n - c), mq, Mp);
    return total;
}

// numpy pairwise sum of a small contiguous double array (n <= 128): noise means
__device__ double np_small_sum(const double *v, int n)
{
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; i++) res += v[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = v[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += v[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += v[i];
    return res;
}
#pragma clang fp contract(on)

// ------------------------------------------------------------------------------------------
struct Shared {
    long long red_l[NWAVE];
    int red_a[NWAVE], red_b[NWAVE];
    double mq, Mp, delta, p90, noise_e, t1, t2, tz;
    long long K;
    float deltaf, invMf;
    int kmin, kmax, t, t0, nv, st, en, F, flags, exact, n3, n4, n2, n5, n1, n6, j0, j1;
    double noise_buf[16];
};
static_assert(sizeof(Shared) <= EXTRACT_SHARED_BYTES, "grow EXTRACT_SHARED_BYTES");

// number of set change-bits with index in [0, x)
__device__ __forceinline__ int chg_prefix(const uint32_t *chg, const uint32_t *pref, int x)
{
    int w = x >> 5, b = x & 31;
    uint32_t m = b ? (chg[w] & ((1u << b) - 1u)) : 0u;
    return (int)pref[w] + __popc(m);
}

// Endpoint scan (src/audio_processing.py:186-273) by wave 0 with ballots.  Returns the
// near-tie flag (only meaningful when certify != 0).  All lanes return the same values.
__device__ int vad_scan(Shared *sh, const double *E, const int32_t *Z, const double *sortedE, int nv,
                        double hi, double lo, double zr, int certify, int lane)
{
    const int nf = min(5, nv / 10);  // :188
    double noise_e, noise_z;
    if (nf > 0) {                    // :189-193
        if (lane == 0) {
            for (int i = 0; i < nf; i++) {
                sh->noise_buf[i] = E[i];
                sh->noise_buf[nf + i] = E[nv - nf + i];
            }
        }
        __builtin_amdgcn_wave_barrier();
        noise_e = np_small_sum(sh->noise_buf, 2 * nf) / (double)(2 * nf);
        __builtin_amdgcn_wave_barrier();
        long long zs = 0;
        for (int i = 0; i < nf; i++) zs += Z[i] + Z[nv - nf + i];
        noise_z = (double)zs / (double)(2 * nf);  // integer sum is exact in any order
    } else {                          // :194-195, :244-245
        double me = INFINITY;
        int mz = 0x7fffffff;
        for (int i = lane; i < nv; i += 64) {
            me = fmin(me, E[i]);
            mz = min(mz, Z[i]);
        }
        noise_e = wave_mind(me);
        noise_z = (double)wave_min(mz);
    }
    // np.percentile(E, 90), method 'linear' (:198)
    const double vi = (double)(nv - 1) * 0.9;
    double pa, pb, g;
    if (vi >= (double)(nv - 1)) {
        pa = pb = sortedE[nv - 1];
        g = vi + 1.0;
    } else {
        double pv = floor(vi);
        int pi = (int)pv;
        pa = sortedE[pi];
        pb = sortedE[pi + 1];
        g = vi - pv;
    }
    double p90;
    {
#pragma clang fp contract(off)
        double d = pb - pa;
        p90 = (g >= 0.5) ? pb - d * (1.0 - g) : pa + d * g;
    }
    double t1, t2, tz;
    {
#pragma clang fp contract(off)
        t1 = p90 * hi;                          // :202
        t2 = noise_e + (p90 - noise_e) * lo;    // :217
        tz = noise_z * zr;                      // :247
    }
    // N3 / N4: first / last frame with E > T1 (:205-213)
    int n3 = -1, n4 = -1;
    for (int c = 0; c < nv; c += 64) {
        int f = c + lane;
        unsigned long long m = __ballot(f < nv && E[f] > t1);
        if (m) {
            if (n3 < 0) n3 = c + __ffsll((long long)m) - 1;
            n4 = c + 63 - __clzll((long long)m);
        }
    }
    int flag = 0;
    auto near = [&](double e, double t) {
        double d = fabs(e - t);
        double tol = 1e-11 * fmax(fabs(e), fabs(t));
        return d <= tol && !(e == 0.0 && t == 0.0);
    };
    if (certify) {
        for (int c = 0; c < nv; c += 64) {
            int f = c + lane;
            bool chk = f < nv && (n3 < 0 || f <= n3 || f >= n4);
            if (__ballot(chk && near(E[f], t1))) flag = 1;
        }
    }
    if (n3 < 0) {  // :207-209
        sh->n3 = -1;
        return flag;
    }
    // N2: scan left from N3-1 for E <= T2 (:219-226)
    int n2 = 0;
    for (int c = ((n3 - 1) >> 6) << 6; c >= 0 && n3 > 0; c -= 64) {
        int i = c + lane;
        unsigned long long m = __ballot(i < n3 && E[i] <= t2);
        if (m) {
            n2 = c + 63 - __clzll((long long)m) + 1;
            break;
        }
    }
    // N5: scan right from N4+1 (:229-235)
    int n5 = nv - 1;
    for (int c = ((n4 + 1) >> 6) << 6; c < nv; c += 64) {
        int i = c + lane;
        unsigned long long m = __ballot(i > n4 && i < nv && E[i] <= t2);
        if (m) {
            n5 = c + __ffsll((long long)m) - 1 - 1;
            break;
        }
    }
    if (certify) {  // frames the two scans actually compared against T2
        for (int c = 0; c < nv; c += 64) {
            int i = c + lane;
            bool chk = i < nv && ((i >= n2 - 1 && i < n3) || (i > n4 && i <= n5 + 1));
            if (__ballot(chk && near(E[i], t2))) flag = 1;
        }
    }
    // N1 / N6: same scans on ZCR from N2 / N5 (:249-265) -- integer compares, exact
    int n1 = 0;
    for (int c = ((n2 - 1) >> 6) << 6; c >= 0 && n2 > 0; c -= 64) {
        int i = c + lane;
        unsigned long long m = __ballot(i < n2 && (double)Z[i] <= tz);
        if (m) {
            n1 = c + 63 - __clzll((long long)m) + 1;
            break;
        }
    }
    int n6 = nv - 1;
    for (int c = ((n5 + 1) >> 6) << 6; c < nv; c += 64) {
        int i = c + lane;
        unsigned long long m = __ballot(i > n5 && i < nv && (double)Z[i] <= tz);
        if (m) {
            n6 = c + __ffsll((long long)m) - 1 - 1;
            break;
        }
    }
    if (lane == 0) {
        sh->n3 = n3;
        sh->n4 = n4;
        sh->n2 = n2;
        sh->n5 = n5;
        sh->n1 = n1;
        sh->n6 = n6;
        sh->p90 = p90;
        sh->noise_e = noise_e;
        sh->t1 = t1;
        sh->t2 = t2;
        sh->tz = tz;
    }
    return flag;
}

// rank-sort E[0..nv) into sortedE (stable ranks; all threads)
__device__ void rank_sort(const double *E, double *sortedE, int nv, int tid)
{
    for (int i = tid; i < nv; i += NT) {
        double e = E[i];
        int r = 0;
        for (int j = 0; j < nv; j++) {
            double o = E[j];
            r += (o < e) || (o == e && j < i);
        }
        sortedE[r] = e;
    }
}

// mean/std/max/min/median of v[0..F) by one wave (src/feature_extraction.py:46-62)
template <typename T>
__device__ void seq_stats(const T *v, int F, int lane, float *out5)
{
    double s = 0.0, mx = -INFINITY, mn = INFINITY;
    for (int i = lane; i < F; i += 64) {
        double x = (double)v[i];
        s += x;
        mx = fmax(mx, x);
        mn = fmin(mn, x);
    }
    s = wave_sum(s);
    mx = wave_maxd(mx);
    mn = wave_mind(mn);
    const double mean = s / (double)F;
    double q = 0.0;
    for (int i = lane; i < F; i += 64) {
        double d = (double)v[i] - mean;
        q += d * d;
    }
    q = wave_sum(q);
    // order statistics (F-1)/2 and F/2 by rank
    const int rlo = (F - 1) / 2, rhi = F / 2;
    double vlo = -INFINITY, vhi = -INFINITY;
    for (int i = lane; i < F; i += 64) {
        T e = v[i];
        int r = 0;
        for (int j = 0; j < F; j++) {
            T o = v[j];
            r += (o < e) || (o == e && j < i);
        }
        if (r == rlo) vlo = (double)e;
        if (r == rhi) vhi = (double)e;
    }
    vlo = wave_maxd(vlo);
    vhi = wave_maxd(vhi);
    double med;
    {
#pragma clang fp contract(off)
        med = (F & 1) ? vhi : (vlo + vhi) / 2.0;
    }
    if (lane == 0) {
        out5[0] = (float)mean;
        out5[1] = (float)sqrt(q / (double)F);
        out5[2] = (float)mx;
        out5[3] = (float)mn;
        out5[4] = (float)med;
    }
}

__global__ __launch_bounds__(NT) void extract_kernel(ExtractParams p)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const ExtractCarve c = extract_carve(p.ncap, p.L, p.S);
    Shared *sh = reinterpret_cast<Shared *>(lds + c.sh);
    int16_t *clip = reinterpret_cast<int16_t *>(lds + c.clip);
    float *win = reinterpret_cast<float *>(lds + c.win);
    uint32_t *chg = reinterpret_cast<uint32_t *>(lds + c.chg);
    uint32_t *pref = reinterpret_cast<uint32_t *>(lds + c.pref);
    long long *seg1 = reinterpret_cast<long long *>(lds + c.seg1);
    double *seg2 = reinterpret_cast<double *>(lds + c.seg2);
    double *vE = reinterpret_cast<double *>(lds + c.vE);
    int32_t *vZ = reinterpret_cast<int32_t *>(lds + c.vZ);
    double *vS = reinterpret_cast<double *>(lds + c.vS);
    float *fE = reinterpret_cast<float *>(lds + c.fE);
    float *fM = reinterpret_cast<float *>(lds + c.fM);
    int32_t *fZ = reinterpret_cast<int32_t *>(lds + c.fZ);

    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int L = p.L, S = p.S;
    const int64_t o0 = p.offsets[b];
    const int64_t nn = p.offsets[b + 1] - o0;
    float *featb = p.feat + (size_t)b * 15;

    if (nn <= 0 || nn > p.ncap) {
        if (tid < 15) featb[tid] = __builtin_nanf("");
        if (tid == 0) {
            p.status[b] = nn <= 0 ? DSP_CLIP_EMPTY : DSP_CLIP_TOO_LONG;
            p.start_end[2 * b] = 0;
            p.start_end[2 * b + 1] = 0;
            p.n_frames[b] = 0;
        }
        return;
    }
    const int n = (int)nn;
    const int64_t total = p.offsets[p.B];  // samples readable in pcm
    if (tid == 0) {
        sh->j0 = L;
        sh->j1 = -1;
    }
    __syncthreads();

    // ---- P0/P1: window + clip -> LDS; integer clip statistics -------------------------
    for (int j = tid; j < L; j += NT) {
        const double w = p.window[j];
        win[j] = (float)w;
        if (w > 0.0) {  // the window is positive exactly on [j0, j1] (zeros only at its ends)
            atomicMin(&sh->j0, j);
            atomicMax(&sh->j1, j);
        }
    }
    const int64_t base = o0 & ~(int64_t)7;
    const int lead = (int)(o0 - base);
    const int nvec = (lead + n + 7) >> 3;
    const int16_t *src = p.pcm + base;
    long long ksum = 0;
    int kmin = 0x7fffffff, kmax = -0x7fffffff - 1;
    for (int v = tid; v < nvec; v += NT) {
        short8 val;
        if (base + 8 * (int64_t)v + 8 <= total) {
            val = *reinterpret_cast<const short8 *>(src + 8 * v);
        } else {
#pragma unroll
            for (int e = 0; e < 8; e++) val[e] = (base + 8 * (int64_t)v + e < total) ? src[8 * v + e] : 0;
        }
        *reinterpret_cast<short8 *>(clip + 8 * v) = val;
        const int i0 = 8 * v - lead;
        if (i0 >= 0 && i0 + 8 <= n) {
            int s = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                int k = val[e];
                s += k;
                kmin = min(kmin, k);
                kmax = max(kmax, k);
            }
            ksum += s;
        } else {
#pragma unroll
            for (int e = 0; e < 8; e++) {
                int i = i0 + e;
                if (i >= 0 && i < n) {
                    int k = val[e];
                    ksum += k;
                    kmin = min(kmin, k);
                    kmax = max(kmax, k);
                }
            }
        }
    }
    ksum = wave_sum(ksum);
    kmin = wave_min(kmin);
    kmax = wave_max(kmax);
    if (lane == 0) {
        sh->red_l[wid] = ksum;
        sh->red_a[wid] = kmin;
        sh->red_b[wid] = kmax;
    }
    __syncthreads();
    if (tid == 0) {
        long long K = 0;
        int a = 0x7fffffff, z = -0x7fffffff - 1;
        for (int w = 0; w < NWAVE; w++) {
            K += sh->red_l[w];
            a = min(a, sh->red_a[w]);
            z = max(z, sh->red_b[w]);
        }
        // remove_dc / normalize_audio (:49-75) in sample units: the reference's float64 mean of
        // k/32768 is exact, so m = fl(K/n) and the peak is max(fl(kmax-m), fl(m-kmin)).
        const double mq = (double)K / (double)n;
        const double Mp = fmax((double)z - mq, mq - (double)a);
        const int t0 = (int)floor(mq + 0.5);
        sh->K = K;
        sh->kmin = a;
        sh->kmax = z;
        sh->mq = mq;
        sh->Mp = Mp;
        sh->t = (int)floor(mq) + 1;  // sample is positive after preprocess  <=>  k >= t
        sh->t0 = t0;
        sh->delta = mq - (double)t0;  // exact (Sterbenz), |delta| <= 0.5
        sh->deltaf = (float)(mq - (double)t0);
        sh->invMf = Mp > 0.0 ? (float)(1.0 / Mp) : 0.0f;
        sh->flags = 0;
    }
    __syncthreads();
    const int tpos = sh->t;
    const int16_t *cl = clip + lead;  // cl[i], i in [0, n)

    // ---- P2: change bits chg[i] = pos[i] ^ pos[i+1] (i < n-1), prefix popcounts ---------
    const int nwords = (n + 31) >> 5;
    for (int w = tid; w < nwords; w += NT) {
        const int i0 = w << 5;
        uint32_t pos = 0;
        if (i0 + 32 <= n) {
#pragma unroll
            for (int e = 0; e < 32; e++) pos |= (uint32_t)(cl[i0 + e] >= tpos) << e;
        } else {
            for (int e = 0; e < 32; e++)
                if (i0 + e < n) pos |= (uint32_t)(cl[i0 + e] >= tpos) << e;
        }
        const uint32_t nxt = (i0 + 32 < n) ? (uint32_t)(cl[i0 + 32] >= tpos) : 0u;
        uint32_t ch = pos ^ ((pos >> 1) | (nxt << 31));
        const int valid = n - 1 - i0;  // bits [0, valid) are real pairs
        if (valid < 32) ch &= valid > 0 ? ((1u << valid) - 1u) : 0u;
        chg[w] = ch;
    }
    if (tid == 0) chg[nwords] = 0;
    __syncthreads();
    // exclusive scan of popc(chg[w]) -> pref[0..nwords] (two words per thread)
    {
        const int w0 = 2 * tid;
        int a0 = w0 < nwords ? __popc(chg[w0]) : 0;
        int a1 = w0 + 1 < nwords ? __popc(chg[w0 + 1]) : 0;
        int tsum = a0 + a1;
        int inc = tsum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) sh->red_a[wid] = inc;
        __syncthreads();
        int wofs = 0;
        for (int w = 0; w < wid; w++) wofs += sh->red_a[w];
        int excl = wofs + inc - tsum;
        // handles nwords <= 2*NT words; larger clips loop below
        if (w0 <= nwords) pref[w0] = excl;
        if (w0 + 1 <= nwords) pref[w0 + 1] = excl + a0;
        __syncthreads();
        // carry for clips with more than 2*NT words (n > 65536 samples)
        for (int base_w = 2 * NT; base_w <= nwords; base_w += 2 * NT) {
            const int carry = pref[base_w - 1] + __popc(chg[base_w - 1]);
            __syncthreads();
            const int w = base_w + 2 * tid;
            int b0 = w < nwords ? __popc(chg[w]) : 0;
            int b1 = w + 1 < nwords ? __popc(chg[w + 1]) : 0;
            int ts = b0 + b1, ic = ts;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                int y = __shfl_up(ic, o, 64);
                if (lane >= o) ic += y;
            }
            if (lane == 63) sh->red_a[wid] = ic;
            __syncthreads();
            int wo = carry;
            for (int q = 0; q < wid; q++) wo += sh->red_a[q];
            int ex = wo + ic - ts;
            if (w <= nwords) pref[w] = ex;
            if (w + 1 <= nwords) pref[w + 1] = ex + b0;
            __syncthreads();
        }
    }

    // ---- P3: endpoint energies / ZCR (src/audio_processing.py:166-184) -----------------
    int st = 0, en = n;
    const int nv = (p.do_vad && n >= L) ? (n - L) / S + 1 : 0;
    if (nv > 0) {
        const int a = L / S, r = L % S;
        const int nq = nv + a;
        const int nseg = 2 * nq;
        const int t0 = sh->t0;
        // integer moments of d = k - t0 per segment [qS, qS+r) and [qS+r, (q+1)S)
        for (int sgb = 0; sgb < nseg; sgb += NT / 8) {
            const int sg = sgb + (tid >> 3), u = tid & 7;
            long long s1 = 0;
            double s2 = 0.0;
            int lo = 0, hi = 0;
            if (sg < nseg) {
                const int q = sg >> 1, h = sg & 1;
                if (r > 0) {
                    lo = q * S + (h ? r : 0);
                    hi = h ? (q + 1) * S : q * S + r;
                } else if (!h) {
                    lo = q * S;
                    hi = (q + 1) * S;
                }
                hi = min(hi, n);
                for (int i = lo + u; i < hi; i += 8) {
                    const int d = cl[i] - t0;
                    s1 += d;
                    const double dd = (double)d;
                    s2 = fma(dd, dd, s2);  // exact: integers < 2^53
                }
            }
            s1 += __shfl_xor(s1, 1, 64);
            s2 += __shfl_xor(s2, 1, 64);
            s1 += __shfl_xor(s1, 2, 64);
            s2 += __shfl_xor(s2, 2, 64);
            s1 += __shfl_xor(s1, 4, 64);
            s2 += __shfl_xor(s2, 4, 64);
            if (sg < nseg && u == 0) {
                seg1[sg] = s1;
                seg2[sg] = s2;
            }
        }
        __syncthreads();
        const double delta = sh->delta, Mp = sh->Mp;
        for (int f = tid; f < nv; f += NT) {
            long long T1 = 0;
            double T2 = 0.0;
            for (int q = f; q < f + a; q++) {
                T1 += seg1[2 * q] + seg1[2 * q + 1];
                T2 += seg2[2 * q] + seg2[2 * q + 1];
            }
            if (r > 0) {
                T1 += seg1[2 * (f + a)];
                T2 += seg2[2 * (f + a)];
            }
            double e = 0.0;
            if (Mp > 0.0) {
                // sum (k - mq)^2 = T2 - 2*delta*T1 + L*delta^2, every term exact or within a few ulp
                const double num = T2 - (2.0 * delta) * (double)T1 + (double)L * (delta * delta);
                e = num / (Mp * Mp);
            }
            vE[f] = e;
            vZ[f] = chg_prefix(chg, pref, f * S + L - 1) - chg_prefix(chg, pref, f * S);
        }
        __syncthreads();
        rank_sort(vE, vS, nv, tid);
        __syncthreads();
        // ---- P4: double-threshold scan, certified; exact numpy-order fallback -----------
        if (wid == 0) {
            int flag = vad_scan(sh, vE, vZ, vS, nv, p.hi, p.lo, p.zr, sh->Mp > 0.0, lane);
            if (lane == 0) sh->exact = flag;
        }
        __syncthreads();
        if (sh->exact) {
            const double mq = sh->mq;
            for (int f = tid; f < nv; f += NT) vE[f] = np_energy_exact(cl, f * S, L, mq, Mp);
            __syncthreads();
            rank_sort(vE, vS, nv, tid);
            __syncthreads();
            if (wid == 0) vad_scan(sh, vE, vZ, vS, nv, p.hi, p.lo, p.zr, 0, lane);
            if (tid == 0) sh->flags |= DSP_CLIP_FLAG_VAD_EXACT;
            __syncthreads();
        }
        if (sh->n3 >= 0) {
            st = sh->n1 * S;                   // :272
            en = min(sh->n6 * S + L, n);       // :273
        }
        if (p.vad_energy) {
            for (int f = tid; f < nv && f < p.ld_vad; f += NT) {
                p.vad_energy[(size_t)b * p.ld_vad + f] = vE[f];
                p.vad_zcr[(size_t)b * p.ld_vad + f] = vZ[f];
            }
        }
    }

    // ---- P5: windowed frames over the crop [st, en) (:378, :299-333; fe.py:12-43) ------
    const int m = en - st;  // > 0 always (start < end by construction)
    const int F = (m <= L) ? 1 : (m - L + S - 1) / S + 1;
    const float deltaf = sh->deltaf, invMf = sh->invMf;
    const int t0 = sh->t0;
    for (int g = wid; g < F; g += NWAVE) {
        const int fs = st + g * S;
        const int lim = min(L, en - fs);  // samples beyond the crop are zero padding
        float ae = 0.f, am = 0.f;
        for (int j = lane; j < lim; j += 64) {
            const float x = ((float)(cl[fs + j] - t0) - deltaf) * invMf;
            const float y = x * win[j];
            ae = fmaf(y, y, ae);
            am += fabsf(y);
        }
        ae = wave_sum(ae);
        am = wave_sum(am);
        if (lane == 0) {
            // ZCR of the windowed, padded frame from the change bits: signs of y_j are
            // pos[i] && w_j > 0 && i < en; the window is positive exactly on [j0, j1].
            int zc = 0;
            const int ia = fs + sh->j0;
            const int ib = min(fs + sh->j1, en - 1);
            if (ia <= ib) {
                zc = chg_prefix(chg, pref, ib) - chg_prefix(chg, pref, ia);
                if (sh->j0 > 0) zc += cl[ia] >= tpos;
                if (ib < fs + L - 1) zc += cl[ib] >= tpos;
            }
            fE[g] = ae;
            fM[g] = am;
            fZ[g] = zc;
        }
    }
    __syncthreads();

    // ---- P6: 15-d statistics (compute_statistics x 3) --------------------------------
    if (wid == 0) seq_stats(fE, F, lane, featb + 0);
    if (wid == 1) seq_stats(fM, F, lane, featb + 5);
    if (wid == 2) seq_stats(fZ, F, lane, featb + 10);
    if (p.seq) {
        for (int g = tid; g < F && g < p.ld_seq; g += NT) {
            float *o = p.seq + ((size_t)b * p.ld_seq + g) * 3;
            o[0] = fE[g];
            o[1] = fM[g];
            o[2] = (float)fZ[g];
        }
    }
    if (tid == 0) {
        p.start_end[2 * b] = st;
        p.start_end[2 * b + 1] = en;
        p.n_frames[b] = F;
        p.status[b] = DSP_CLIP_OK | sh->flags;
    }
}

}  // namespace dsp

extern "C" size_t dsp_extract_lds_bytes(int64_t max_len, int frame_length, int frame_shift)
{
    if (max_len < 1 || frame_length < 1 || frame_shift < 1 || max_len > (1 << 24)) return 0;
    ExtractCarve c = extract_carve((int)max_len, frame_length, frame_shift);
    return c.total <= EXTRACT_LDS_LIMIT ? (size_t)c.total : 0;
}

extern "C" int dsp_extract_features(const int16_t *pcm, const int64_t *offsets, int B,
                                    int64_t max_len, int frame_length, int frame_shift,
                                    const double *window, int do_vad, double hi, double lo,
                                    double zr, float *feat, int32_t *start_end, int32_t *n_frames,
                                    int32_t *status, double *vad_energy, int32_t *vad_zcr,
                                    int ld_vad, float *seq, int ld_seq, void *stream)
{
    if (B < 0 || !offsets || !window || !feat || !start_end || !n_frames || !status)
        return DSP_ERR_ARGS;
    if (frame_length < 1 || frame_shift < 1 || max_len < 1) return DSP_ERR_ARGS;
    if (((uintptr_t)pcm & 15) != 0) return DSP_ERR_ARGS;
    if ((vad_energy == nullptr) != (vad_zcr == nullptr)) return DSP_ERR_ARGS;
    if (vad_energy && ld_vad < 1) return DSP_ERR_ARGS;
    if (seq && ld_seq < 1) return DSP_ERR_ARGS;
    if (B == 0) return DSP_OK;
    const size_t lds = dsp_extract_lds_bytes(max_len, frame_length, frame_shift);
    if (lds == 0) return DSP_ERR_TOO_LONG;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void *)dsp::extract_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, EXTRACT_LDS_LIMIT);
        attr_set = true;
    }
    dsp::ExtractParams p;
    p.pcm = pcm;
    p.offsets = offsets;
    p.B = B;
    p.ncap = (int)max_len;
    p.L = frame_length;
    p.S = frame_shift;
    p.window = window;
    p.do_vad = do_vad;
    p.hi = hi;
    p.lo = lo;
    p.zr = zr;
    p.feat = feat;
    p.start_end = start_end;
    p.n_frames = n_frames;
    p.status = status;
    p.vad_energy = vad_energy;
    p.vad_zcr = vad_zcr;
    p.ld_vad = ld_vad;
    p.seq = seq;
    p.ld_seq = ld_seq;
    hipLaunchKernelGGL(dsp::extract_kernel, dim3(B), dim3(dsp::NT), lds, (hipStream_t)stream, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? DSP_OK : DSP_ERR_HIP + (int)e;
}
