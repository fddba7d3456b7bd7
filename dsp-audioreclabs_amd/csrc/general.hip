// general.hip -- the per-clip pipeline for clips outside the fused kernel's on-chip plan: any
// length (the reference has no limit, src/audio_processing.py:336-396) and samples wider than
// int16 (16-bit stereo: load_wav averages the two channels, :35-44, so the exact sample is the
// 17-bit sum l + r in units of 2^-16).
//
// One 256-thread workgroup per clip, everything read straight from global memory (L2): the
// sample passes are frame-parallel (one wave per frame), the order statistics are radix
// selections over order-preserving keys, and the per-frame values live in a workspace of
// dsp_extract_general_workspace_bytes().  Same arithmetic as the fused kernel (extract.hip):
//   * mean / peak from exact integer sums (the reference's float64 values bit for bit);
//   * endpoint energies from exact integer moments in float64, every threshold decision
//     certified against a 1e-11 margin, near ties redone in numpy's pairwise float64 order;
//   * positive samples k >= floor(mq) + 1 (integer), every ZCR exact;
//   * windowed E / M in fp32 in the canonical order of dsp_device.h (the fused kernel's bits);
//     statistics in fp64.
// Reference functions restated: preprocess :78-90, endpoint_detection :135-275, frame_signal
// :299-333, extract_frame_features fe.py:12-43, compute_statistics fe.py:46-62.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dsp_audiorec.h"
#include "dsp_device.h"

namespace dsp {
namespace gen {

constexpr int NT = 256;
constexpr int NWAVE = NT / 64;

struct Params {
    const void *pcm;
    const int64_t *offsets;
    const int32_t *index;  // clips to process (NULL: 0 .. nclip-1)
    int nclip;
    int64_t min_len, max_len;  // clips with min_len < n <= max_len (others untouched)
    int L, S;
    const double *window;
    int do_vad;
    double hi, lo, zr;
    float *feat;
    int32_t *start_end, *n_frames, *status;
    int ostride;  // 0: per-array rows; > 0: row i of each output at i * ostride (ABI 6)
    double *vad_energy;
    int32_t *vad_zcr;
    int ld_vad;
    float *seq;
    int ld_seq;
    unsigned char *ws;
    int64_t ws_stride;  // bytes per processed clip
    int64_t nvcap, fcap;
};

__device__ __forceinline__ float *out_feat(const Params &p, int i) { return p.feat + (int64_t)i * (p.ostride ? p.ostride : 15); }
__device__ __forceinline__ int32_t *out_se(const Params &p, int i) { return p.start_end + (int64_t)i * (p.ostride ? p.ostride : 2); }
__device__ __forceinline__ int32_t *out_nf(const Params &p, int i) { return p.n_frames + (int64_t)i * (p.ostride ? p.ostride : 1); }
__device__ __forceinline__ int32_t *out_st(const Params &p, int i) { return p.status + (int64_t)i * (p.ostride ? p.ostride : 1); }

// workspace of one clip: vE f64[nvcap], vZ i32[nvcap], fE f32[fcap], fM f32[fcap], fZ i32[fcap],
// keys u64[max(nvcap, fcap)]
struct Ws {
    double *vE;
    int32_t *vZ;
    float *fE, *fM;
    int32_t *fZ;
    unsigned long long *key;
};
__host__ __device__ inline int64_t ws_stride(int64_t nvcap, int64_t fcap)
{
    const int64_t kc = nvcap > fcap ? nvcap : fcap;
    return ((8 * nvcap + 4 * nvcap + 12 * fcap + 8 * kc + 16 * 8) + 255) & ~(int64_t)255;
}
__device__ inline Ws ws_at(const Params &p, int j)
{
    unsigned char *b = p.ws + (int64_t)j * p.ws_stride;
    Ws w;
    int64_t o = 0;
    auto take = [&](int64_t bytes) {
        unsigned char *r = b + o;
        o = (o + bytes + 15) & ~(int64_t)15;
        return r;
    };
    w.vE = reinterpret_cast<double *>(take(8 * p.nvcap));
    w.vZ = reinterpret_cast<int32_t *>(take(4 * p.nvcap));
    w.fE = reinterpret_cast<float *>(take(4 * p.fcap));
    w.fM = reinterpret_cast<float *>(take(4 * p.fcap));
    w.fZ = reinterpret_cast<int32_t *>(take(4 * p.fcap));
    w.key = reinterpret_cast<unsigned long long *>(take(8 * (p.nvcap > p.fcap ? p.nvcap : p.fcap)));
    return w;
}

struct Sh {
    long long red_l[NWAVE];
    unsigned long long red_u[NWAVE];
    int red_a[NWAVE], red_b[NWAVE];
    double red_d[NWAVE], red_e[NWAVE];
    unsigned hist[256];
    unsigned long long prefix;
    int rank;
    int n1, n6, n3, near;
};

template <typename T> __device__ __forceinline__ int sample(const T *x, int64_t i) { return (int)x[i]; }

// the rare exact endpoint energy, out of line (its pairwise-sum stack stays off the common path)
template <typename T>
__device__ __attribute__((noinline)) double exact_energy(const T *x, int64_t lo, int L, double mq, double Mp)
{
    return np_energy_exact(x, lo, L, mq, Mp);
}

// block reductions (every thread gets the result)
__device__ long long block_sum_ll(Sh &s, long long v)
{
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.red_l[threadIdx.x >> 6] = v;
    __syncthreads();
    long long t = 0;
    for (int w = 0; w < NWAVE; w++) t += s.red_l[w];
    return t;
}
__device__ unsigned long long block_sum_ull(Sh &s, unsigned long long v)
{
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.red_u[threadIdx.x >> 6] = v;
    __syncthreads();
    unsigned long long t = 0;
    for (int w = 0; w < NWAVE; w++) t += s.red_u[w];
    return t;
}
__device__ double block_sum_d(Sh &s, double v)  // fixed order: waves 0..3 (deterministic)
{
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s.red_d[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < NWAVE; w++) t += s.red_d[w];
    return t;
}
__device__ void block_minmax(Sh &s, int &mn, int &mx)
{
    mn = wave_min(mn);
    mx = wave_max(mx);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        s.red_a[threadIdx.x >> 6] = mn;
        s.red_b[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    mn = s.red_a[0];
    mx = s.red_b[0];
    for (int w = 1; w < NWAVE; w++) {
        mn = min(mn, s.red_a[w]);
        mx = max(mx, s.red_b[w]);
    }
}
__device__ void block_minmax_f(Sh &s, float &mn, float &mx)
{
    mn = wave_reduce(mn, OpMin());
    mx = wave_reduce(mx, OpMax());
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        s.red_d[threadIdx.x >> 6] = mn;
        s.red_e[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    mn = (float)s.red_d[0];
    mx = (float)s.red_e[0];
    for (int w = 1; w < NWAVE; w++) {
        mn = fminf(mn, (float)s.red_d[w]);
        mx = fmaxf(mx, (float)s.red_e[w]);
    }
}

// the r-th smallest (0-based) of n order-preserving keys, 8-bit digits from the top, KB bytes
template <int KB>
__device__ unsigned long long radix_select(Sh &s, const unsigned long long *key, int64_t n, int64_t r)
{
    unsigned long long prefix = 0, mask = 0;
    int64_t rr = r;
    for (int shift = 8 * (KB - 1); shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += NT) s.hist[b] = 0;
        __syncthreads();
        for (int64_t i = threadIdx.x; i < n; i += NT) {
            const unsigned long long k = key[i];
            if ((k & mask) == prefix) atomicAdd(&s.hist[(k >> shift) & 255], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t c = 0;
            int d = 0;
            for (; d < 255; d++) {
                if (c + s.hist[d] > rr) break;
                c += s.hist[d];
            }
            s.rank = (int)(rr - c);
            s.prefix = prefix | ((unsigned long long)d << shift);
        }
        __syncthreads();
        rr = s.rank;
        prefix = s.prefix;
        mask |= 255ull << shift;
        __syncthreads();
    }
    return prefix;
}

// one clip (number i), start to finish, by the whole workgroup; w is the workgroup's workspace
template <typename T>
__device__ __forceinline__ void general_clip(const Params &p, Sh &s, const Ws &w, int i)
{
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t o0 = p.offsets[i], nn = p.offsets[i + 1] - o0;
    // min_len == 0: this launch owns every clip, so an empty one (np.max of an empty array raises,
    // :72) and one longer than max_len are reported here; otherwise they belong to another launch
    if (p.min_len == 0 && (nn <= 0 || nn > p.max_len)) {
        if (tid < 15) out_feat(p, i)[tid] = __builtin_nanf("");
        if (tid == 0) {
            *out_st(p, i) = nn <= 0 ? DSP_CLIP_EMPTY : DSP_CLIP_TOO_LONG;
            out_se(p, i)[0] = out_se(p, i)[1] = 0;
            *out_nf(p, i) = 0;
        }
        return;
    }
    if (nn <= p.min_len || nn > p.max_len) return;  // another launch's clip
    const T *x = reinterpret_cast<const T *>(p.pcm) + o0;
    const int64_t n = nn;
    const int L = p.L, S = p.S;

    // ---- preprocess (:49-75): exact integer sum / min / max ---------------------------------
    long long ks = 0;
    int kmin = 0x7fffffff, kmax = -0x7fffffff - 1;
    for (int64_t j = tid; j < n; j += NT) {
        const int k = sample(x, j);
        ks += k;
        kmin = min(kmin, k);
        kmax = max(kmax, k);
    }
    const long long K = block_sum_ll(s, ks);
    block_minmax(s, kmin, kmax);
    const double mq = (double)K / (double)n;
    const double Mp = fmax((double)kmax - mq, mq - (double)kmin);
    const int tpos = (int)floor(mq) + 1;
    const int t0 = (int)floor(mq + 0.5);
    const double delta = mq - (double)t0;
    const double invM2 = Mp > 0.0 ? 1.0 / (Mp * Mp) : 0.0;
    const float invMf = Mp > 0.0 ? (float)(1.0 / Mp) : 0.f;
    const int64_t nv = (p.do_vad && n >= L) ? (n - L) / S + 1 : 0;
    const int64_t Fmax = n <= L ? 1 : (n - L + S - 1) / S + 1;

    // ---- endpoint frames (:166-184): one wave per frame, exact moments, sign changes --------
    for (int64_t f = wid; f < nv; f += NWAVE) {
        const int64_t a = f * S;
        long long s1 = 0, s2 = 0;
        int zc = 0;
        for (int j = lane; j < L; j += 64) {
            const int k = sample(x, a + j);
            s1 += k;
            s2 += (long long)k * k;
            if (j + 1 < L) zc += (k >= tpos) != (sample(x, a + j + 1) >= tpos);
        }
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        zc = wave_sum(zc);
        if (lane == 0) {
            const long long D1 = s1 - (long long)L * t0;
            const long long D2 = s2 - 2LL * t0 * s1 + (long long)L * t0 * t0;
            const double r = fma(-2.0 * delta, (double)D1, (double)D2) + (double)L * delta * delta;
            w.vE[f] = r * invM2;
            w.vZ[f] = zc;
        }
    }
    __syncthreads();

    // ---- endpoint decisions (:186-273) ------------------------------------------------------
    int64_t st = 0, en = n, F = Fmax;
    int flags = 0;
    if (nv > 0) {
        for (int pass = 0; pass < 2; pass++) {
            const bool certify = pass == 0;
            // p90 (:198): order statistics of the energies by radix selection
            for (int64_t f = tid; f < nv; f += NT) w.key[f] = dkey(w.vE[f]);
            __syncthreads();
            const double vi = (double)(nv - 1) * 0.9;
            int64_t r0, r1;
            if (vi >= (double)(nv - 1)) {
                r0 = r1 = nv - 1;
            } else {
                r0 = (int64_t)floor(vi);
                r1 = r0 + 1;
            }
            const double pa = dkey_value(radix_select<8>(s, w.key, nv, r0));
            const double pb = dkey_value(radix_select<8>(s, w.key, nv, r1));
            const double g = (vi >= (double)(nv - 1)) ? vi + 1.0 : vi - floor(vi);
            const double p90 = np_lerp(pa, pb, g);
            if (tid == 0) {
                // noise estimates (:188-195, :239-245), numpy order for the small sums
                const int64_t nfr = min((int64_t)5, nv / 10);
                double noise_e, noise_z;
                if (nfr > 0) {
                    long long zs = 0;
                    for (int64_t q = 0; q < nfr; q++) zs += w.vZ[q] + w.vZ[nv - nfr + q];
                    auto cat = [&](int q) { return q < nfr ? w.vE[q] : w.vE[nv - 2 * nfr + q]; };
                    noise_e = np_small_sum(cat, (int)(2 * nfr)) / (double)(2 * nfr);
                    noise_z = (double)zs / (double)(2 * nfr);
                } else {
                    noise_e = INFINITY;
                    int mz = 0x7fffffff;
                    for (int64_t q = 0; q < nv; q++) {
                        noise_e = fmin(noise_e, w.vE[q]);
                        mz = min(mz, w.vZ[q]);
                    }
                    noise_z = (double)mz;
                }
                double t1, t2, tz;
                {
#pragma clang fp contract(off)
                    t1 = p90 * p.hi;                        // :202
                    t2 = noise_e + (p90 - noise_e) * p.lo;  // :217
                    tz = noise_z * p.zr;                    // :247
                }
                auto near = [&](double e, double t) {
                    const double d = fabs(e - t);
                    return d <= 1e-11 * fmax(fabs(e), fabs(t)) && !(e == 0.0 && t == 0.0);
                };
                int nr = 0;
                int64_t n3 = -1, n4 = -1;
                for (int64_t q = 0; q < nv; q++)  // :205-213
                    if (w.vE[q] > t1) {
                        if (n3 < 0) n3 = q;
                        n4 = q;
                    }
                if (certify) {  // the decisions of N3 / N4 depend on frames <= N3 and >= N4
                    for (int64_t q = 0; q < nv; q++)
                        if ((n3 < 0 || q <= n3 || q >= n4) && near(w.vE[q], t1)) nr = 1;
                }
                int64_t n1 = 0, n6 = nv - 1;
                if (n3 >= 0) {
                    int64_t n2 = 0, n5 = nv - 1;
                    for (int64_t q = n3 - 1; q >= 0; q--)  // :219-226
                        if (w.vE[q] <= t2) {
                            n2 = q + 1;
                            break;
                        }
                    for (int64_t q = n4 + 1; q < nv; q++)  // :229-235
                        if (w.vE[q] <= t2) {
                            n5 = q - 1;
                            break;
                        }
                    if (certify)
                        for (int64_t q = 0; q < nv; q++)
                            if (((q >= n2 - 1 && q < n3) || (q > n4 && q <= n5 + 1)) && near(w.vE[q], t2)) nr = 1;
                    for (int64_t q = n2 - 1; q >= 0; q--)  // :249-256
                        if ((double)w.vZ[q] <= tz) {
                            n1 = q + 1;
                            break;
                        }
                    for (int64_t q = n5 + 1; q < nv; q++)  // :258-265
                        if ((double)w.vZ[q] <= tz) {
                            n6 = q - 1;
                            break;
                        }
                }
                s.n3 = (int)n3;
                s.n1 = (int)n1;
                s.n6 = (int)n6;
                s.near = certify && nr && Mp > 0.0;
            }
            __syncthreads();
            if (!s.near) break;
            // near tie: endpoint energies in numpy's exact float64 order, then decide again
            flags = DSP_CLIP_FLAG_VAD_EXACT;
            for (int64_t f = tid; f < nv; f += NT) w.vE[f] = exact_energy(x, f * S, L, mq, Mp);
            __syncthreads();
        }
        if (s.n3 >= 0) {
            st = (int64_t)s.n1 * S;                            // :272
            en = min((int64_t)s.n6 * S + L, n);                // :273
            F = s.n6 - s.n1 + 1;
        }
        if (p.vad_energy)
            for (int64_t f = tid; f < nv && f < p.ld_vad; f += NT) {
                p.vad_energy[(int64_t)i * p.ld_vad + f] = w.vE[f];
                p.vad_zcr[(int64_t)i * p.ld_vad + f] = w.vZ[f];
            }
    }

    // ---- windowed frames of the crop [st, en) (:378, :299-333; fe.py:12-43) ---------------
    // frame g covers crop samples [g S, g S + L), zero-padded past the crop.  One 16-lane row per
    // frame, E / M in the canonical order of dsp_device.h (the fused kernel's, same bits); the
    // ZCR is exact either way.
    const CanonX cx = canon_x(mq, t0);
    const int rl = lane & 15, row = lane >> 4;
    for (int64_t gi = wid; 4 * gi < F; gi += NWAVE) {
        const int64_t g = 4 * gi + row;
        const bool act = g < F;
        const int64_t fs = st + (act ? g : F - 1) * S;
        const int64_t lim = min((int64_t)L, en - fs);
        const int64_t va = fs >> 3, vb = (fs + lim - 1) >> 3;
        float2v ea = {0.f, 0.f};
        float m0 = 0.f, m1 = 0.f;
        for (int64_t v = va + rl; v <= vb; v += 16)
            for (int h = 0; h < 4; h++) {
                float2v wv, xv;
                for (int t = 0; t < 2; t++) {
                    const int64_t sj = 8 * v + 2 * h + t, j = sj - fs;
                    wv[t] = (j >= 0 && j < lim) ? (float)p.window[j] : 0.f;
                    xv[t] = sj < n ? canon_xval(sample(x, sj), cx) : 0.f;
                }
                canon_pair(wv, xv, ea, m0, m1);
            }
        const float es = dpp_row_reduce(ea.x + ea.y, OpAdd()), ms = dpp_row_reduce(m0 + m1, OpAdd());
        int zc = 0;
        for (int j = rl; j + 1 < L; j += 16) {
            const bool p0 = j < lim && p.window[j] > 0.0 && sample(x, fs + j) >= tpos;
            const bool p1 = j + 1 < lim && p.window[j + 1] > 0.0 && sample(x, fs + j + 1) >= tpos;
            zc += p0 != p1;
        }
        zc = dpp_row_reduce(zc, OpAdd());
        if (act && rl == 0) {
            w.fE[g] = es * (invMf * invMf);
            w.fM[g] = ms * invMf;
            w.fZ[g] = zc;
        }
    }
    __syncthreads();

    // ---- statistics (fe.py:46-62): mean, population std, max, min, median -----------------
    float *featb = out_feat(p, i);
    for (int q = 0; q < 3; q++) {
        auto get = [&](int64_t g) -> float { return q == 0 ? w.fE[g] : q == 1 ? w.fM[g] : (float)w.fZ[g]; };
        double sm = 0.0;
        float mn = INFINITY, mx = -INFINITY;
        for (int64_t g = tid; g < F; g += NT) {
            const float v = get(g);
            sm += (double)v;
            mn = fminf(mn, v);
            mx = fmaxf(mx, v);
            w.key[g] = fkey(v);
        }
        const double mean = block_sum_d(s, sm) / (double)F;
        block_minmax_f(s, mn, mx);
        double sq = 0.0;
        for (int64_t g = tid; g < F; g += NT) {
            const double d = (double)get(g) - mean;
            sq = fma(d, d, sq);
        }
        const double var = block_sum_d(s, sq) / (double)F;
        const float v0 = fkey_value((unsigned)radix_select<4>(s, w.key, F, (F - 1) / 2));
        const float v1 = fkey_value((unsigned)radix_select<4>(s, w.key, F, F / 2));
        double med;
        {
#pragma clang fp contract(off)
            med = (F & 1) ? (double)v1 : ((double)v0 + (double)v1) / 2.0;
        }
        if (tid == 0) {
            featb[5 * q + 0] = (float)mean;
            featb[5 * q + 1] = (float)sqrt(var);
            featb[5 * q + 2] = mx;
            featb[5 * q + 3] = mn;
            featb[5 * q + 4] = (float)med;
        }
        __syncthreads();
    }
    if (p.seq)
        for (int64_t g = tid; g < F && g < p.ld_seq; g += NT) {
            float *o = p.seq + ((int64_t)i * p.ld_seq + g) * 3;
            o[0] = w.fE[g];
            o[1] = w.fM[g];
            o[2] = (float)w.fZ[g];
        }
    if (tid == 0) {
        out_se(p, i)[0] = (int32_t)st;
        out_se(p, i)[1] = (int32_t)en;
        *out_nf(p, i) = (int32_t)F;
        *out_st(p, i) = DSP_CLIP_OK | flags;
    }
}

// Persistent grid: workgroup b takes list entries b, b + G, ... and keeps its workspace slot b,
// so the workspace is min(nclip, GEN_GRID) slots and a launch over a whole batch (clip_index
// NULL, the length window selecting the clips) needs no host-side selection.
constexpr int GEN_GRID = 1024;
template <typename T>
__global__ __launch_bounds__(NT) void general_kernel(Params p)
{
    __shared__ Sh s;
    const Ws w = ws_at(p, blockIdx.x);
    for (int j = blockIdx.x; j < p.nclip; j += gridDim.x) {
        general_clip<T>(p, s, w, p.index ? p.index[j] : j);
        __syncthreads();  // shared state and the workspace slot are the next clip's
    }
}

}  // namespace gen
}  // namespace dsp

extern "C" size_t dsp_extract_general_workspace_bytes(int64_t nclip, int64_t max_len, int frame_length,
                                                      int frame_shift)
{
    if (nclip < 1 || max_len < 1 || frame_length < 1 || frame_shift < 1) return 0;
    const int64_t nv = max_len >= frame_length ? (max_len - frame_length) / frame_shift + 1 : 1;
    const int64_t F = max_len <= frame_length ? 1 : (max_len - frame_length + frame_shift - 1) / frame_shift + 1;
    return (size_t)(std::min<int64_t>(nclip, dsp::gen::GEN_GRID) * dsp::gen::ws_stride(nv, F));
}

extern "C" int dsp_extract_general(const void *pcm, int sample_bytes, const int64_t *offsets,
                                   const int32_t *clip_index, int nclip, int64_t min_len, int64_t max_len,
                                   int frame_length, int frame_shift, const double *window, int do_vad,
                                   double hi, double lo, double zr, float *feat, int32_t *start_end,
                                   int32_t *n_frames, int32_t *status, int out_stride, double *vad_energy,
                                   int32_t *vad_zcr, int ld_vad, float *seq, int ld_seq,
                                   void *workspace, size_t workspace_bytes, void *stream)
{
    if (nclip < 0 || !pcm || !offsets || !window || !feat || !start_end || !n_frames || !status)
        return DSP_ERR_ARGS;
    if (out_stride != 0 && out_stride < DSP_OUT_ROW_WORDS) return DSP_ERR_ARGS;
    if (sample_bytes != 2 && sample_bytes != 4) return DSP_ERR_ARGS;
    if (frame_length < 1 || frame_shift < 1 || max_len < 1 || min_len < 0) return DSP_ERR_ARGS;
    if (frame_length > (1 << 16) || max_len > ((int64_t)1 << 31)) return DSP_ERR_ARGS;
    if ((vad_energy == nullptr) != (vad_zcr == nullptr)) return DSP_ERR_ARGS;
    if (vad_energy && ld_vad < 1) return DSP_ERR_ARGS;
    if (seq && ld_seq < 1) return DSP_ERR_ARGS;
    if (nclip == 0 || min_len >= max_len) return DSP_OK;
    const size_t need = dsp_extract_general_workspace_bytes(nclip, max_len, frame_length, frame_shift);
    if (!workspace || workspace_bytes < need) return DSP_ERR_WORKSPACE;
    dsp::gen::Params p;
    p.pcm = pcm;
    p.offsets = offsets;
    p.index = clip_index;
    p.nclip = nclip;
    p.min_len = min_len;
    p.max_len = max_len;
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
    p.ostride = out_stride;
    p.vad_energy = vad_energy;
    p.vad_zcr = vad_zcr;
    p.ld_vad = ld_vad;
    p.seq = seq;
    p.ld_seq = ld_seq;
    p.ws = (unsigned char *)workspace;
    p.nvcap = max_len >= frame_length ? (max_len - frame_length) / frame_shift + 1 : 1;
    p.fcap = max_len <= frame_length ? 1 : (max_len - frame_length + frame_shift - 1) / frame_shift + 1;
    p.ws_stride = dsp::gen::ws_stride(p.nvcap, p.fcap);
    const unsigned grid = (unsigned)std::min(nclip, dsp::gen::GEN_GRID);
    if (sample_bytes == 2)
        hipLaunchKernelGGL(dsp::gen::general_kernel<int16_t>, dim3(grid), dim3(dsp::gen::NT), 0, (hipStream_t)stream, p);
    else
        hipLaunchKernelGGL(dsp::gen::general_kernel<int32_t>, dim3(grid), dim3(dsp::gen::NT), 0, (hipStream_t)stream, p);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DSP_OK : DSP_ERR_HIP + (int)e;
}
