// extract.hip -- fused per-clip feature extraction for gfx950 (CDNA4).
//
// Persistent workgroups (1024 threads, one per CU: the clip lives in LDS) walk the batch.  While
// a workgroup computes clip i out of LDS, the 16-byte loads of clip i+grid are already in flight
// into registers, so the HBM stream never waits for the compute.  The clip is read from HBM exactly
// once: algorithmic traffic is 2 B/sample in + 76 B/clip out.
//
// Reference functions restated (Hypersonic-cpu/DSP-AudioRecLabs):
//   preprocess              src/audio_processing.py:78-90
//   endpoint_detection      src/audio_processing.py:135-275
//   frame_signal            src/audio_processing.py:299-333
//   extract_frame_features  src/feature_extraction.py:12-43
//   compute_statistics / extract_statistical_features  src/feature_extraction.py:46-88
//
// Exactness plan:
//   * mean / peak: exact integer sums -> mq = fl(K/n), M' = max(fl(kmax-mq), fl(mq-kmin)) are the
//     reference's float64 values bit for bit (its mean of k/32768 is exact).
//   * signs and every ZCR: pure integer (sample positive <=> k >= floor(mq)+1): bit-exact.
//   * endpoint energies: exact int64 moments per frame (sum k, sum k^2) combined with mq in
//     double-double -> relative error ~1e-16; every threshold decision is certified against a
//     1e-11 margin and, on a near tie, the energies are recomputed in numpy's exact float64 order
//     (pairwise_sum), so start/end are always the reference's.
//   * windowed E/M: fp32 on VALU (tolerance 1e-5 rel., measured ~2e-7); statistics in fp64.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dsp_audiorec.h"
#include "extract_layout.h"

namespace dsp {

static constexpr int NT = EXTRACT_THREADS;
static constexpr int NWAVE = NT / 64;
static constexpr int NR = EXTRACT_MAX_ROUNDS;  // 16-B vectors per thread per clip (max)
static constexpr int NPF = EXTRACT_PREFETCH;   // of which prefetched into registers

#ifdef DSP_STAMPS
// diagnostic build only (make stamps): per-phase shader-clock stamps of each clip
__device__ unsigned long long *g_stamps;
__device__ uint32_t *g_dump;  // chg words of each clip after R2a (4096 words per clip)
#define STAMP(clip, k)                                                                           \
    do {                                                                                         \
        if (threadIdx.x == 0 && g_stamps) g_stamps[(size_t)(clip) * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define STAMP(clip, k) \
    do {               \
    } while (0)
#endif

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

typedef short short2v __attribute__((ext_vector_type(2)));

// ---- wave reductions on DPP (VALU lane permutes, no LDS crossbar) + 4 readlanes -------------
// Every lane must be active.  Results are wave-uniform.
#define DPP_QXOR1 0xB1   // quad_perm [1,0,3,2]
#define DPP_QXOR2 0x4E   // quad_perm [2,3,0,1]
#define DPP_HMIRROR 0x141
#define DPP_MIRROR 0x140
__device__ __forceinline__ int dpp_i(int v, int ctrl)
{
    switch (ctrl) {
    case DPP_QXOR1: return __builtin_amdgcn_update_dpp(0, v, DPP_QXOR1, 0xF, 0xF, false);
    case DPP_QXOR2: return __builtin_amdgcn_update_dpp(0, v, DPP_QXOR2, 0xF, 0xF, false);
    case DPP_HMIRROR: return __builtin_amdgcn_update_dpp(0, v, DPP_HMIRROR, 0xF, 0xF, false);
    default: return __builtin_amdgcn_update_dpp(0, v, DPP_MIRROR, 0xF, 0xF, false);
    }
}
template <typename T, typename Op>
__device__ __forceinline__ T dpp_row_reduce(T v, Op op)
{
    constexpr int ctl[4] = {DPP_QXOR1, DPP_QXOR2, DPP_HMIRROR, DPP_MIRROR};
#pragma unroll
    for (int s = 0; s < 4; s++) {
        T o;
        if constexpr (sizeof(T) == 4) {
            o = __builtin_bit_cast(T, dpp_i(__builtin_bit_cast(int, v), ctl[s]));
        } else {
            const long long x = __builtin_bit_cast(long long, v);
            const int lo = dpp_i((int)x, ctl[s]), hi = dpp_i((int)(x >> 32), ctl[s]);
            o = __builtin_bit_cast(T, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
        }
        v = op(v, o);
    }
    return v;
}
// quad (4-lane) reduction: lanes 4q..4q+3 all get the quad's result
template <typename Op>
__device__ __forceinline__ int dpp_quad_reduce(int v, Op op)
{
    v = op(v, dpp_i(v, DPP_QXOR1));
    return op(v, dpp_i(v, DPP_QXOR2));
}
template <typename T>
__device__ __forceinline__ T lane_read(T v, int lane)
{
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
    } else {
        const long long x = __builtin_bit_cast(long long, v);
        const unsigned lo = __builtin_amdgcn_readlane((int)x, lane);
        const unsigned hi = __builtin_amdgcn_readlane((int)(x >> 32), lane);
        return __builtin_bit_cast(T, (long long)(((unsigned long long)hi << 32) | lo));
    }
}
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op)
{
    v = dpp_row_reduce(v, op);
    return op(op(lane_read(v, 0), lane_read(v, 16)), op(lane_read(v, 32), lane_read(v, 48)));
}
struct OpAdd {
    template <typename T> __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpMin {
    template <typename T> __device__ T operator()(T a, T b) const { return a < b ? a : b; }
};
struct OpMax {
    template <typename T> __device__ T operator()(T a, T b) const { return a > b ? a : b; }
};
template <typename T> __device__ __forceinline__ T wave_sum(T v) { return wave_reduce(v, OpAdd()); }
__device__ __forceinline__ int wave_min(int v) { return wave_reduce(v, OpMin()); }
__device__ __forceinline__ int wave_max(int v) { return wave_reduce(v, OpMax()); }
__device__ __forceinline__ double wave_maxd(double v) { return wave_reduce(v, OpMax()); }
__device__ __forceinline__ double wave_mind(double v) { return wave_reduce(v, OpMin()); }

// ------------------------------------------------------------------------------------------
// exact float64 helpers (no contraction: error-free transformations and numpy's own order)
// ------------------------------------------------------------------------------------------
#pragma clang fp contract(off)
__device__ __forceinline__ void two_sum(double a, double b, double &s, double &e)
{
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}
__device__ __forceinline__ void two_prod(double a, double b, double &p, double &e)
{
    p = a * b;
    e = __fma_rn(a, b, -p);
}

// sum_{frame} (k - mq)^2 / M'^2 from the exact moments S1 = sum k, S2 = sum k^2 (L samples):
// S2 - 2 mq S1 + L mq^2 evaluated in double-double (cancellation-free), then one division.
__device__ double energy_from_moments(unsigned long long S2, long long S1, int L, double mq, double Mp)
{
    if (!(Mp > 0.0)) return 0.0;  // constant clip: preprocess leaves zeros (:73-75)
    const double s2 = (double)S2, s1 = (double)S1;
    double p, pe, q, qe, r, re;
    two_prod(mq, s1, p, pe);
    p *= 2.0;
    pe *= 2.0;
    two_prod(mq, mq, q, qe);
    two_prod((double)L, q, r, re);
    re += (double)L * qe;
    double a, ae, b, be;
    two_sum(s2, -p, a, ae);
    two_sum(a, r, b, be);
    const double A = b + (((ae + be) - pe) + re);
    return A / (Mp * Mp);
}

// numpy float64 summation order (pairwise_sum in 8192-element buffered chunks): the certified
// fallback of the endpoint energies.  Element i is x_i^2, x_i = fl(fl(k_i - mq) / M').
__device__ __forceinline__ double xsq(const int16_t *clip, int i, double mq, double Mp)
{
    const double d = (double)clip[i] - mq;
    const double x = Mp > 0.0 ? d / Mp : d;
    return x * x;
}

__device__ __forceinline__ double pw_leaf(const int16_t *clip, int lo, int n, double mq, double Mp)
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
__device__ __forceinline__ double pw_block(const int16_t *clip, int lo, int n, double mq, double Mp)
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
            const int cl = s_lo[sp], cn = s_n[sp];
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
        const int pl = s_lo[sp], pn = s_n[sp];
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

__device__ __forceinline__ double np_energy_exact(const int16_t *clip, int lo, int n, double mq, double Mp)
{
    double total = 0.0;
    for (int c = 0; c < n; c += 8192) total += pw_block(clip, lo + c, min(8192, n - c), mq, Mp);
    return total;
}

// numpy pairwise sum of a small array (n <= 128) given by an accessor: noise means (:190-193)
template <typename Acc>
__device__ __forceinline__ double np_small_sum(Acc v, int n)
{
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; i++) res += v(i);
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = v(j);
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] += v(i + j);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += v(i);
    return res;
}

// numpy _lerp for the 'linear' percentile (numpy/lib/_function_base_impl.py)
__device__ double np_lerp(double a, double b, double g)
{
    const double d = b - a;
    return (g >= 0.5) ? b - d * (1.0 - g) : a + d * g;
}
#pragma clang fp contract(on)

// ------------------------------------------------------------------------------------------
struct Shared {
    int red_s[NWAVE], red_a[NWAVE], red_b[NWAVE];
    double pa, pb;            // the two order statistics of the VAD energies around p90
    double oslo[3], oshi[3];  // order statistics (F-1)/2 and F/2 of E, M, ZCR (medians)
    double noise_buf[16];
    int n3, n1, n6, exact, j0, j1, ndefer;
};
static_assert(sizeof(Shared) <= EXTRACT_SHARED_BYTES, "grow EXTRACT_SHARED_BYTES");

// set change-bits in buffer-bit range [x0, x1) (bit u = sign change between samples u, u+1)
__device__ __forceinline__ int popc_range(const uint32_t *chg, int x0, int x1)
{
    if (x1 <= x0) return 0;
    const int w0 = x0 >> 5, w1 = (x1 - 1) >> 5;
    int c = 0;
    for (int w = w0; w <= w1; w++) {
        uint32_t m = chg[w];
        if (w == w0) m &= ~0u << (x0 & 31);
        if (w == w1 && ((x1 & 31) != 0)) m &= (1u << (x1 & 31)) - 1u;
        c += __popc(m);
    }
    return c;
}

struct ClipRef {
    int64_t base;  // 8-aligned first sample index of the clip's vectors
    int lead, n, nvec, lim;
    bool ok;
};

__device__ __forceinline__ ClipRef clip_ref(const ExtractParams &p, int i, int64_t total)
{
    ClipRef c;
    const int64_t o0 = p.offsets[i], nn = p.offsets[i + 1] - o0;
    c.ok = nn > 0 && nn <= p.ncap;
    c.n = c.ok ? (int)nn : 0;
    c.base = o0 & ~(int64_t)7;
    c.lead = (int)(o0 - c.base);
    c.nvec = (c.lead + c.n + 7) >> 3;
    c.lim = c.ok ? (int)min((int64_t)c.nvec, (total - c.base) >> 3) : 0;
    return c;
}

// 16-B loads of rounds [R0, R1) of a clip (unconditional, clamped addresses: no per-load branch,
// so no vmcnt(0) between them).  The prefetch of the next clip is issued in slices spread over the
// phases of the current one, so the issue never blocks on a full memory queue.
template <int R0, int R1>
__device__ __forceinline__ void issue_rounds(short8 (&regs)[NPF], const int16_t *pcm, const ClipRef &c,
                                             int tid)
{
    if (c.lim <= 0) return;
    const short8 *src = reinterpret_cast<const short8 *>(pcm + c.base);
#pragma unroll
    for (int r = R0; r < R1; r++) regs[r] = __builtin_nontemporal_load(src + min(tid + r * NT, c.lim - 1));
}
__device__ __forceinline__ void issue_loads(short8 (&regs)[NPF], const int16_t *pcm, const ClipRef &c,
                                            int tid)
{
    issue_rounds<0, NPF>(regs, pcm, c, tid);
}
static_assert(NPF % 4 == 0, "prefetch issued in four slices");
#define PREFETCH_SLICE(k)                                                                     \
    do {                                                                                      \
        if (!EXACT && prefetch) issue_rounds<(k) * (NPF / 4), ((k) + 1) * (NPF / 4)>(regs, p.pcm, nxt, tid); \
    } while (0)

struct Ctx {
    Shared *sh;
    int16_t *buf;  // clip samples, buffer coordinates u = i + lead
    uint32_t *chg;
    uint32_t *pos;                     // positive-sample bits
    int *sgS, *sgZ;                    // per-segment sum k, sign changes
    unsigned long long *sgQ;           // per-segment sum k^2
    float2 *wtab;                      // (window, window^2)
    double *vE;
    int32_t *vZ;
    float *fE, *fM;
    int32_t *fZ;
    int *defer;
    int64_t total;
};

__device__ __forceinline__ short2v half_pair(const short8 &x, int i)
{
    switch (i) {
    case 0: return __builtin_shufflevector(x, x, 0, 1);
    case 1: return __builtin_shufflevector(x, x, 2, 3);
    case 2: return __builtin_shufflevector(x, x, 4, 5);
    default: return __builtin_shufflevector(x, x, 6, 7);
    }
}

// exact moments of 8 samples: sum k (packed dot with ones) and sum k^2 (packed dot of each pair,
// <= 2^31 read as unsigned, accumulated in 64 bits)
__device__ __forceinline__ void moments8(const short8 &x, int &s1, unsigned long long &s2)
{
    const short2v ones = {1, 1};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const short2v d = half_pair(x, i);
        s1 = __builtin_amdgcn_sdot2(d, ones, s1, false);
        s2 += (unsigned)__builtin_amdgcn_sdot2(d, d, 0, false);
    }
}
__device__ __forceinline__ unsigned long long dpp_quad_sum64(unsigned long long v)
{
    const auto add = [](unsigned long long a, unsigned long long b) { return a + b; };
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const int ctl = s == 0 ? DPP_QXOR1 : DPP_QXOR2;
        const unsigned lo = dpp_i((int)(unsigned)v, ctl), hi = dpp_i((int)(unsigned)(v >> 32), ctl);
        v = add(v, ((unsigned long long)hi << 32) | lo);
    }
    return v;
}

// ---- 256-frame bit sets (wave-uniform: four ballots) ------------------------------------------
struct Bits256 {
    unsigned long long w[4];
};
__device__ __forceinline__ int bits_first_ge(const Bits256 &m, int from)  // lowest set >= from, or -1
{
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int sh = from - 64 * k;
        unsigned long long x = m.w[k];
        if (sh >= 64) x = 0;
        else if (sh > 0) x &= ~0ull << sh;
        if (x) return 64 * k + __ffsll((long long)x) - 1;
    }
    return -1;
}
__device__ __forceinline__ int bits_last_lt(const Bits256 &m, int below)  // highest set < below, or -1
{
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        const int sh = below - 64 * k;
        unsigned long long x = m.w[k];
        if (sh <= 0) x = 0;
        else if (sh < 64) x &= (1ull << sh) - 1ull;
        if (x) return 64 * k + 63 - __clzll((long long)x);
    }
    return -1;
}
__device__ __forceinline__ bool bits_any_in(const Bits256 &m, int lo, int hi)  // any set in [lo, hi)
{
    const int f = bits_first_ge(m, lo);
    return f >= 0 && f < hi;
}

// Double-threshold endpoint scan (src/audio_processing.py:186-273) by wave 0 on vE/vZ with the
// p90 order statistics in sh->pa / sh->pb.  Writes sh->n3 (-1: no high-energy frame), n1, n6;
// returns the near-tie flag.
template <bool CERTIFY>
__device__ __forceinline__ int vad_scan(const ExtractParams &p, const Ctx &c, int nv, int lane)
{
    const double *vE = c.vE;
    const int32_t *vZ = c.vZ;
    Shared *sh = c.sh;
    const int nfr = min(5, nv / 10);  // :188
    double noise_e, noise_z;
    if (nfr > 0) {  // :189-193, :239-243 (every lane computes the same numpy-order sum)
        long long zs = 0;
        for (int q = 0; q < nfr; q++) zs += vZ[q] + vZ[nv - nfr + q];
        // np.concatenate([E[:nfr], E[-nfr:]]) read in place
        auto cat = [&](int q) { return q < nfr ? vE[q] : vE[nv - 2 * nfr + q]; };
        noise_e = np_small_sum(cat, 2 * nfr) / (double)(2 * nfr);
        noise_z = (double)zs / (double)(2 * nfr);  // exact integer sum
    } else {  // :194-195, :244-245
        double me = INFINITY;
        int mz = 0x7fffffff;
        for (int q = lane; q < nv; q += 64) {
            me = fmin(me, vE[q]);
            mz = min(mz, vZ[q]);
        }
        noise_e = wave_mind(me);
        noise_z = (double)wave_min(mz);
    }
    // np.percentile(E, 90) (:198): lerp of the two order statistics found by the workgroup
    const double vi = (double)(nv - 1) * 0.9;
    const double g = (vi >= (double)(nv - 1)) ? vi + 1.0 : vi - floor(vi);
    const double p90 = np_lerp(sh->pa, sh->pb, g);
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
    int flag = 0, n3 = -1, n1 = 0, n6 = nv - 1;
    if (nv <= 256) {
        Bits256 hiE, loE, loZ, nr1, nr2;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int q = 64 * k + lane;
            const bool in = q < nv;
            const double e = in ? vE[q] : 0.0;
            const int z = in ? vZ[q] : 0;
            hiE.w[k] = __ballot(in && e > t1);
            loE.w[k] = __ballot(in && e <= t2);
            loZ.w[k] = __ballot(in && (double)z <= tz);
            nr1.w[k] = CERTIFY ? __ballot(in && near(e, t1)) : 0ull;
            nr2.w[k] = CERTIFY ? __ballot(in && near(e, t2)) : 0ull;
        }
        n3 = bits_first_ge(hiE, 0);  // :205-213
        const int n4 = bits_last_lt(hiE, nv);
        if (CERTIFY) {  // decisions of N3 / N4 depend on frames <= N3 and >= N4
            if (n3 < 0) flag |= bits_any_in(nr1, 0, nv);
            else flag |= bits_any_in(nr1, 0, n3 + 1) || bits_any_in(nr1, n4, nv);
        }
        if (n3 >= 0) {
            const int b2 = bits_last_lt(loE, n3);  // :219-226
            const int n2 = b2 >= 0 ? b2 + 1 : 0;
            const int b5 = bits_first_ge(loE, n4 + 1);  // :229-235
            const int n5 = b5 >= 0 ? b5 - 1 : nv - 1;
            if (CERTIFY)  // only the frames the two scans compared against T2
                flag |= bits_any_in(nr2, max(n2 - 1, 0), n3) || bits_any_in(nr2, n4 + 1, min(n5 + 2, nv));
            const int b1 = bits_last_lt(loZ, n2);  // :249-256
            n1 = b1 >= 0 ? b1 + 1 : 0;
            const int b6 = bits_first_ge(loZ, n5 + 1);  // :258-265
            n6 = b6 >= 0 ? b6 - 1 : nv - 1;
        }
    } else {  // long sequences: chunked ballots straight from LDS
        int n4 = -1;
        for (int q0 = 0; q0 < nv; q0 += 64) {
            const int f = q0 + lane;
            const unsigned long long m = __ballot(f < nv && vE[f] > t1);
            if (m) {
                if (n3 < 0) n3 = q0 + __ffsll((long long)m) - 1;
                n4 = q0 + 63 - __clzll((long long)m);
            }
        }
        if (CERTIFY)
            for (int q0 = 0; q0 < nv; q0 += 64) {
                const int f = q0 + lane;
                const bool chk = f < nv && (n3 < 0 || f <= n3 || f >= n4);
                if (__ballot(chk && near(vE[f], t1))) flag = 1;
            }
        if (n3 >= 0) {
            int n2 = 0, n5 = nv - 1;
            for (int q0 = ((n3 - 1) >> 6) << 6; q0 >= 0 && n3 > 0; q0 -= 64) {
                const int q = q0 + lane;
                const unsigned long long m = __ballot(q < n3 && vE[q] <= t2);
                if (m) {
                    n2 = q0 + 63 - __clzll((long long)m) + 1;
                    break;
                }
            }
            for (int q0 = ((n4 + 1) >> 6) << 6; q0 < nv; q0 += 64) {
                const int q = q0 + lane;
                const unsigned long long m = __ballot(q > n4 && q < nv && vE[q] <= t2);
                if (m) {
                    n5 = q0 + __ffsll((long long)m) - 2;
                    break;
                }
            }
            if (CERTIFY)
                for (int q0 = 0; q0 < nv; q0 += 64) {
                    const int q = q0 + lane;
                    const bool chk = q < nv && ((q >= n2 - 1 && q < n3) || (q > n4 && q <= n5 + 1));
                    if (__ballot(chk && near(vE[q], t2))) flag = 1;
                }
            for (int q0 = ((n2 - 1) >> 6) << 6; q0 >= 0 && n2 > 0; q0 -= 64) {
                const int q = q0 + lane;
                const unsigned long long m = __ballot(q < n2 && (double)vZ[q] <= tz);
                if (m) {
                    n1 = q0 + 63 - __clzll((long long)m) + 1;
                    break;
                }
            }
            for (int q0 = ((n5 + 1) >> 6) << 6; q0 < nv; q0 += 64) {
                const int q = q0 + lane;
                const unsigned long long m = __ballot(q > n5 && q < nv && (double)vZ[q] <= tz);
                if (m) {
                    n6 = q0 + __ffsll((long long)m) - 2;
                    break;
                }
            }
        }
    }
    if (lane == 0) {
        sh->n3 = n3;
        sh->n1 = n1;
        sh->n6 = n6;
    }
    return flag;
}

// rank (ties by index) of every element of v[0..n) -> the elements of ranks r0 / r1 (all threads)
template <typename T>
__device__ __forceinline__ void rank_select(const T *v, int n, int r0, int r1, double *o0, double *o1,
                                            int tid)
{
    for (int i = tid; i < n; i += NT) {
        const T e = v[i];
        int r = 0;
#pragma unroll 8
        for (int j = 0; j < n; j++) {
            const T o = v[j];
            r += (o < e) || (o == e && j < i);
        }
        if (r == r0) *o0 = (double)e;
        if (r == r1) *o1 = (double)e;
    }
}

// One clip, start to finish.  EXACT = false: the streaming path (registers prefetched, endpoint
// energies from exact moments, decisions certified); returns false when a decision is a near tie
// (the clip is then redone with EXACT = true after the persistent loop).
template <bool EXACT>
__device__ __forceinline__ bool clip_body(const ExtractParams &p, const Ctx &c, int i,
                                          const ClipRef &cur, short8 (&regs)[NPF], bool prefetch,
                                          const ClipRef &nxt)
{
    Shared *sh = c.sh;
    int16_t *buf = c.buf;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int L = p.L, S = p.S;
    const int n = cur.n, lead = cur.lead, nvec = cur.nvec;
    const int16_t *cl = buf + lead;  // cl[i], sample coords
    const int64_t total = c.total;
    float *featb = p.feat + (size_t)i * 15;
    STAMP(i, 0);

    // ---- R1: clip -> LDS; integer sum / min / max (packed 16-bit) ---------------------------
    int s1 = 0, kmin_s = 0x7fffffff, kmax_s = -0x7fffffff - 1;
    short2v pmin = {32767, 32767}, pmax = {-32768, -32768};
    auto consume = [&](short8 val, int v) {
        if (v >= cur.lim && v < nvec) {  // last vector of the pcm buffer: partial
            const int16_t *src = p.pcm + cur.base + 8 * v;
            for (int e = 0; e < 8; e++) val[e] = (cur.base + 8 * v + e < total) ? src[e] : 0;
        }
        if (v < nvec) {
            *reinterpret_cast<short8 *>(buf + 8 * v) = val;
            const int u0 = 8 * v;
            if (u0 >= lead && u0 + 8 <= lead + n) {
                const short2v ones = {1, 1};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const short2v d = half_pair(val, q);
                    pmin = __builtin_elementwise_min(pmin, d);
                    pmax = __builtin_elementwise_max(pmax, d);
                    s1 = __builtin_amdgcn_sdot2(d, ones, s1, false);
                }
            } else {  // first / last vector of the clip
                for (int e = 0; e < 8; e++) {
                    const int u = u0 + e;
                    if (u >= lead && u < lead + n) {
                        const int k = val[e];
                        s1 += k;
                        kmin_s = min(kmin_s, k);
                        kmax_s = max(kmax_s, k);
                    }
                }
            }
        }
    };
    const short8 *gsrc = reinterpret_cast<const short8 *>(p.pcm + cur.base);
    if (!EXACT) {
#pragma unroll
        for (int r = 0; r < NPF; r++) consume(regs[r], tid + r * NT);
    }
#pragma unroll 1
    for (int v = tid + (EXACT ? 0 : NPF * NT); v - tid < nvec; v += NT) {  // long clips / exact redo
        short8 val = {};
        if (v < cur.lim) val = gsrc[v];
        consume(val, v);
    }
    {
        const int kmn = min(kmin_s, min((int)pmin.x, (int)pmin.y));
        const int kmx = max(kmax_s, max((int)pmax.x, (int)pmax.y));
        const int ws = wave_sum(s1), wmn = wave_min(kmn), wmx = wave_max(kmx);
        if (lane == 0) {
            sh->red_s[wid] = ws;
            sh->red_a[wid] = wmn;
            sh->red_b[wid] = wmx;
        }
    }
    __syncthreads();
    // remove_dc / normalize_audio (:49-75) in sample units, computed redundantly by every thread:
    // the reference's float64 mean of k/32768 is exact, so m = fl(K/n) and the peak is
    // max(fl(kmax - m), fl(m - kmin)); a sample is positive after preprocess <=> k >= t.
    long long K = 0;
    int kmin = 0x7fffffff, kmax = -0x7fffffff - 1;
#pragma unroll
    for (int w = 0; w < NWAVE; w++) {
        K += sh->red_s[w];
        kmin = min(kmin, sh->red_a[w]);
        kmax = max(kmax, sh->red_b[w]);
    }
    const double mq = (double)K / (double)n;
    const double Mp = fmax((double)kmax - mq, mq - (double)kmin);
    const int tpos = (int)floor(mq) + 1;
    const int t0 = (int)floor(mq + 0.5);
    const float deltaf = (float)(mq - (double)t0);  // mq - t0 is exact (Sterbenz)
    const float invMf = Mp > 0.0 ? (float)(1.0 / Mp) : 0.0f;
    const int nv = (p.do_vad && n >= L) ? (n - L) / S + 1 : 0;
    STAMP(i, 1);

    // ---- R2a: positive-sample bits (pos byte v = buffer samples 8v..8v+7; pos(u): sample u is
    //      real and positive after preprocess), then sign-change bits at word level:
    //      chg bit u = pos(u) ^ pos(u+1) for real pairs ---------------------------------------
    unsigned char *posb = reinterpret_cast<unsigned char *>(c.pos);
    const bool tbig = tpos > 32767;  // no int16 sample can be positive
    const short2v tt = {(short)(tbig ? 32767 : tpos), (short)(tbig ? 32767 : tpos)};
    auto pos_of = [&](const short8 &val, int v) {
        if (v >= nvec) return;
        unsigned P = 0u;
        if (!tbig) {
            const unsigned a0 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 0), tt));
            const unsigned a1 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 1), tt));
            const unsigned a2 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 2), tt));
            const unsigned a3 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 3), tt));
            // the four sign bytes of each pair of dwords, then their top bits (k < t)
            const unsigned x01 = __builtin_amdgcn_perm(a1, a0, 0x07050301u) & 0x80808080u;
            const unsigned x23 = __builtin_amdgcn_perm(a3, a2, 0x07050301u) & 0x80808080u;
            P = ~(((x01 * 0x00204081u) >> 28) | (((x23 * 0x00204081u) >> 28) << 4)) & 0xFFu;
        }
        const int u0 = 8 * v;
        if (u0 < lead || u0 + 8 > lead + n) {  // first / last vector: real samples only
            const int lo_ = min(max(lead - u0, 0), 8), hi_ = min(max(lead + n - u0, 0), 8);
            P &= ((1u << hi_) - 1u) & ~((1u << lo_) - 1u);
        }
        posb[v] = (unsigned char)P;
    };
    const short8 *bv = reinterpret_cast<const short8 *>(buf);
    if (!EXACT) {
#pragma unroll
        for (int r = 0; r < NPF; r++) {  // the buffer's partial last vector was patched in LDS only
            const int v = tid + r * NT;
            pos_of(v < cur.lim ? regs[r] : bv[min(v, nvec)], v);
        }
    }
#pragma unroll 1
    for (int v = tid + (EXACT ? 0 : NPF * NT); v - tid < nvec; v += NT) pos_of(v < nvec ? bv[v] : short8{}, v);
    if (tid < 8) posb[nvec + tid] = 0;
    PREFETCH_SLICE(0);
    __syncthreads();
    {
        // in place: every thread reads its words (and the next word's first bit), then, after a
        // barrier, writes the change bits over them
        const int nw = (nvec + 3) >> 2;
        const int rlo = lead, rhi = lead + n - 1;  // real pairs start in [rlo, rhi)
        constexpr int MW = (EXTRACT_MAX_ROUNDS * NT * 8 / 32 + NT - 1) / NT;  // words per thread
        uint32_t chw[MW];
#pragma unroll
        for (int k = 0; k < MW; k++) {
            const int w = tid + k * NT;
            uint32_t ch = 0;
            if (w < nw) {
                const uint32_t p0 = c.pos[w], p1 = c.pos[w + 1];
                ch = p0 ^ ((p0 >> 1) | (p1 << 31));
                const int b0 = 32 * w;
                if (b0 < rlo || b0 + 32 > rhi) {
                    const int lo_ = min(max(rlo - b0, 0), 32), hi_ = min(max(rhi - b0, 0), 32);
                    const uint32_t mhi = hi_ >= 32 ? ~0u : ((1u << hi_) - 1u);
                    const uint32_t mlo = lo_ >= 32 ? 0u : ~((1u << lo_) - 1u);
                    ch &= mhi & mlo;
                }
            }
            chw[k] = ch;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < MW; k++) {
            const int w = tid + k * NT;
            if (w < nw) c.chg[w] = chw[k];
        }
        if (tid < 2) c.chg[nw + tid] = 0;
    }
    __syncthreads();
#ifdef DSP_STAMPS
    if (g_dump)
        for (int w = tid; w < 4096; w += NT) g_dump[(size_t)i * 4096 + w] = w < (nvec + 3) / 4 + 2 ? c.chg[w] : 0xdeadbeefu;
#endif
    STAMP(i, 2);

    // ---- R2b: exact moments + sign changes per segment [qS, qS+r), [qS+r, (q+1)S), L = aS + r:
    //      frame f = segments of hops f..f+a-1 + the head segment of hop f+a ------------------
    const int a_ = L / S, r_ = L % S;
    if (!EXACT && nv > 0) {
        const int nseg = 2 * (nv + a_);
        const int jj = tid & 3;
        for (int sg = tid >> 2; sg < nseg; sg += NT / 4) {
            const int q = sg >> 1, h = sg & 1;
            int lo, hi;
            if (r_ > 0) {
                lo = q * S + (h ? r_ : 0);
                hi = h ? (q + 1) * S : q * S + r_;
            } else {
                lo = q * S;
                hi = h ? lo : (q + 1) * S;
            }
            hi = min(hi, n);
            lo = min(lo, hi);
            const int ulo = lo + lead, uhi = hi + lead;
            int a1 = 0, zc = 0;
            unsigned long long q2 = 0;
            if (uhi > ulo) {
                for (int v = (ulo >> 3) + jj; v <= ((uhi - 1) >> 3); v += 4) {
                    short8 x = bv[v];
                    const int u0 = 8 * v;
                    const int mlo = max(ulo - u0, 0), mhi = min(uhi - u0, 8);
                    if (mlo > 0 || mhi < 8)
                        for (int e = 0; e < 8; e++)
                            if (e < mlo || e >= mhi) x[e] = 0;
                    moments8(x, a1, q2);
                }
                const int w0 = ulo >> 5, w1 = (uhi - 1) >> 5;
                for (int w = w0 + jj; w <= w1; w += 4) {
                    uint32_t m = c.chg[w];
                    if (w == w0) m &= ~0u << (ulo & 31);
                    if (w == w1 && (uhi & 31)) m &= (1u << (uhi & 31)) - 1u;
                    zc += __popc(m);
                }
            }
            a1 = dpp_quad_reduce(a1, OpAdd());
            q2 = dpp_quad_sum64(q2);
            zc = dpp_quad_reduce(zc, OpAdd());
            if (jj == 0) {
                c.sgS[sg] = a1;
                c.sgQ[sg] = q2;
                c.sgZ[sg] = zc;
            }
        }
        __syncthreads();
        STAMP(i, 7);
    }

    PREFETCH_SLICE(1);

    // ---- R3: endpoint detection (:161-273) ------------------------------------------------
    int st = 0, en = n;
    if (nv > 0) {
        for (int f = tid; f < nv; f += NT) {
            const int ua = lead + f * S;  // buffer coords of the frame start
            if (EXACT) {
                c.vE[f] = np_energy_exact(cl, f * S, L, mq, Mp);
                c.vZ[f] = popc_range(c.chg, ua, ua + L - 1);
            } else {
                long long S1 = 0;
                unsigned long long S2 = 0;
                int zc = 0;
                auto add = [&](int sg) {
                    S1 += c.sgS[sg];
                    S2 += c.sgQ[sg];
                    zc += c.sgZ[sg];
                };
                for (int q = f; q < f + a_; q++) {
                    add(2 * q);
                    if (r_ > 0) add(2 * q + 1);
                }
                if (r_ > 0) add(2 * (f + a_));
                c.vE[f] = energy_from_moments(S2, S1, L, mq, Mp);
                // the last segment also counted the pair leaving the frame
                const int ub = ua + L - 1;
                c.vZ[f] = zc - (int)((c.chg[ub >> 5] >> (ub & 31)) & 1u);
            }
        }
        __syncthreads();
        STAMP(i, 8);
        // p90 order statistics (:198) by parallel ranks
        {
            const double vi = (double)(nv - 1) * 0.9;
            int r0, r1;
            if (vi >= (double)(nv - 1)) {
                r0 = r1 = nv - 1;
            } else {
                r0 = (int)floor(vi);
                r1 = r0 + 1;
            }
            rank_select<double>(c.vE, nv, r0, r1, &sh->pa, &sh->pb, tid);
        }
        __syncthreads();
        STAMP(i, 3);
        if (wid == 0) {
            const int flag = vad_scan<!EXACT>(p, c, nv, lane);
            if (lane == 0) sh->exact = (!EXACT && Mp > 0.0) ? flag : 0;
        }
        __syncthreads();
        if (!EXACT && sh->exact) {  // near tie: redo in numpy's exact order after the loop
            PREFETCH_SLICE(2);
            PREFETCH_SLICE(3);
            return false;
        }
        if (sh->n3 >= 0) {
            st = sh->n1 * S;              // :272
            en = min(sh->n6 * S + L, n);  // :273
        }
        if (p.vad_energy)
            for (int f = tid; f < nv && f < p.ld_vad; f += NT) {
                p.vad_energy[(size_t)i * p.ld_vad + f] = c.vE[f];
                p.vad_zcr[(size_t)i * p.ld_vad + f] = c.vZ[f];
            }
    }
    PREFETCH_SLICE(2);
    STAMP(i, 4);

    // ---- R4: windowed frames over the crop [st, en) (:378, :299-333; fe.py:12-43) ---------
    const int m = en - st;  // > 0 always (start < end)
    const int F = (m <= L) ? 1 : (m - L + S - 1) / S + 1;
    const int j0 = sh->j0, j1 = sh->j1;
    const float2 *wtab = c.wtab;
    auto zcr_words = [&](int fs) {  // this lane's share of the frame's sign changes
        const int ia = fs + j0, ib = min(fs + j1, en - 1);
        int cnt = 0;
        if (ia < ib) {
            const int x0 = ia + lead, x1 = ib + lead;
            const int w0 = x0 >> 5, w1 = (x1 - 1) >> 5;
            for (int w = w0 + lane; w <= w1; w += 64) {
                uint32_t mm = c.chg[w];
                if (w == w0) mm &= ~0u << (x0 & 31);
                if (w == w1 && (x1 & 31)) mm &= (1u << (x1 & 31)) - 1u;
                cnt += __popc(mm);
            }
        }
        return cnt;
    };
    auto zcr_edges = [&](int fs) {  // transitions into / out of the window's zero ends or padding
        const int ia = fs + j0, ib = min(fs + j1, en - 1);
        int z = 0;
        if (ia <= ib) {
            if (j0 > 0) z += (int)cl[ia] >= tpos;
            if (ib < fs + L - 1) z += (int)cl[ib] >= tpos;
        }
        return z;
    };
    const float sE = invMf * invMf, sM = invMf;
    for (int g = wid; g < F; g += 2 * NWAVE) {  // two frames per wave: g and g + NWAVE
        const int g2 = g + NWAVE;
        const bool two = g2 < F;
        const int fs = st + g * S, fs2 = st + g2 * S;
        const int lim = min(L, en - fs);  // samples beyond the crop are zero padding
        const int lim2 = two ? min(L, en - fs2) : 0;
        const int16_t *X = cl + fs, *X2 = two ? cl + fs2 : cl + fs;
        const int lim2c = two ? lim2 : lim;
        // E = sum w^2 x^2, M = sum w |x| with x = (k - t0) - delta (scaled by 1/M' at the end);
        // wave-uniform trip count, 4 window positions x 2 frames per lane and iteration
        float e0 = 0.f, m0 = 0.f, e1 = 0.f, m1 = 0.f, f0 = 0.f, n0 = 0.f, f1 = 0.f, n1 = 0.f;
        const int nit = (max(lim, lim2) + 255) >> 8;
        for (int it = 0; it < nit; it++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int j = it * 256 + u * 64 + lane;
                const float2 w = wtab[min(j, L - 1)];
                const int ka = X[min(j, lim - 1)], kb = X2[min(j, lim2c - 1)];
                const float xa = j < lim ? (float)(ka - t0) - deltaf : 0.f;
                const float xb = j < lim2 ? (float)(kb - t0) - deltaf : 0.f;
                if (u & 1) {
                    e1 = fmaf(w.y, xa * xa, e1);
                    m1 = fmaf(w.x, fabsf(xa), m1);
                    f1 = fmaf(w.y, xb * xb, f1);
                    n1 = fmaf(w.x, fabsf(xb), n1);
                } else {
                    e0 = fmaf(w.y, xa * xa, e0);
                    m0 = fmaf(w.x, fabsf(xa), m0);
                    f0 = fmaf(w.y, xb * xb, f0);
                    n0 = fmaf(w.x, fabsf(xb), n0);
                }
            }
        }
        const float E1 = wave_sum(e0 + e1) * sE, M1 = wave_sum(m0 + m1) * sM;
        const int z1 = wave_sum(zcr_words(fs)) + zcr_edges(fs);
        if (lane == 0) {
            c.fE[g] = E1;
            c.fM[g] = M1;
            c.fZ[g] = z1;
        }
        if (two) {
            const float E2 = wave_sum(f0 + f1) * sE, M2 = wave_sum(n0 + n1) * sM;
            const int z2 = wave_sum(zcr_words(fs2)) + zcr_edges(fs2);
            if (lane == 0) {
                c.fE[g2] = E2;
                c.fM[g2] = M2;
                c.fZ[g2] = z2;
            }
        }
    }
    PREFETCH_SLICE(3);
    __syncthreads();
    STAMP(i, 5);

    // ---- R5: 15-d statistics (compute_statistics x 3, fe.py:46-62) ------------------------
    {
        // np.median: the middle order statistic (odd F) or the mean of the two middle ones;
        // ranks of the three sequences in parallel, thread t -> (sequence t / F, element t % F)
        const int r0 = (F - 1) / 2, r1 = F / 2;
        for (int t = tid; t < 3 * F; t += NT) {
            const int sq = t / F, e = t - sq * F;
            int r = 0;
            double val;
            if (sq == 2) {
                const int x = c.fZ[e];
#pragma unroll 8
                for (int q = 0; q < F; q++) {
                    const int o = c.fZ[q];
                    r += (o < x) || (o == x && q < e);
                }
                val = (double)x;
            } else {
                const float *v = sq == 0 ? c.fE : c.fM;
                const float x = v[e];
#pragma unroll 8
                for (int q = 0; q < F; q++) {
                    const float o = v[q];
                    r += (o < x) || (o == x && q < e);
                }
                val = (double)x;
            }
            if (r == r0) sh->oslo[sq] = val;
            if (r == r1) sh->oshi[sq] = val;
        }
    }
    __syncthreads();
    STAMP(i, 9);
    if (wid < 3) {
        double s = 0.0, mx = -INFINITY, mn = INFINITY;
        for (int q = lane; q < F; q += 64) {
            const double x = wid == 0 ? (double)c.fE[q] : wid == 1 ? (double)c.fM[q] : (double)c.fZ[q];
            s += x;
            mx = fmax(mx, x);
            mn = fmin(mn, x);
        }
        s = wave_sum(s);
        mx = wave_maxd(mx);
        mn = wave_mind(mn);
        const double mean = s / (double)F;
        double qq = 0.0;
        for (int q = lane; q < F; q += 64) {
            const double x = wid == 0 ? (double)c.fE[q] : wid == 1 ? (double)c.fM[q] : (double)c.fZ[q];
            const double d = x - mean;
            qq = fma(d, d, qq);
        }
        qq = wave_sum(qq);
        double med;
        {
#pragma clang fp contract(off)
            med = (F & 1) ? sh->oshi[wid] : (sh->oslo[wid] + sh->oshi[wid]) / 2.0;
        }
        if (lane < 5) {
            const double o = lane == 0 ? mean : lane == 1 ? sqrt(qq / (double)F) : lane == 2 ? mx
                             : lane == 3 ? mn : med;
            featb[5 * wid + lane] = (float)o;
        }
    }
    if (p.seq)
        for (int g = tid; g < F && g < p.ld_seq; g += NT) {
            float *o = p.seq + ((size_t)i * p.ld_seq + g) * 3;
            o[0] = c.fE[g];
            o[1] = c.fM[g];
            o[2] = (float)c.fZ[g];
        }
    if (tid == 0) {
        p.start_end[2 * i] = st;
        p.start_end[2 * i + 1] = en;
        p.n_frames[i] = F;
        p.status[i] = DSP_CLIP_OK | (EXACT ? DSP_CLIP_FLAG_VAD_EXACT : 0);
    }
    STAMP(i, 6);
    return true;
}

__device__ __forceinline__ void write_bad_clip(const ExtractParams &p, int i, int tid)
{
    if (tid < 15) p.feat[(size_t)i * 15 + tid] = __builtin_nanf("");
    if (tid == 0) {
        const int64_t nn = p.offsets[i + 1] - p.offsets[i];
        p.status[i] = nn <= 0 ? DSP_CLIP_EMPTY : DSP_CLIP_TOO_LONG;
        p.start_end[2 * i] = 0;
        p.start_end[2 * i + 1] = 0;
        p.n_frames[i] = 0;
    }
}

__global__ __launch_bounds__(NT) void extract_kernel(ExtractParams p)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const ExtractCarve cv = extract_carve(p.ncap, p.L, p.S, EXTRACT_DEFER_CAP);
    Ctx c;
    c.sh = reinterpret_cast<Shared *>(lds + cv.sh);
    c.buf = reinterpret_cast<int16_t *>(lds + cv.clip);
    c.chg = reinterpret_cast<uint32_t *>(lds + cv.chg);
    c.pos = c.chg;  // positive bits are turned into change bits in place
    c.sgQ = reinterpret_cast<unsigned long long *>(lds + cv.seg);
    c.sgS = reinterpret_cast<int *>(c.sgQ + cv.nseg);
    c.sgZ = c.sgS + cv.nseg;
    c.wtab = reinterpret_cast<float2 *>(lds + cv.wtab);
    c.vE = reinterpret_cast<double *>(lds + cv.vE);
    c.vZ = reinterpret_cast<int32_t *>(lds + cv.vZ);
    c.fE = reinterpret_cast<float *>(lds + cv.fE);
    c.fM = reinterpret_cast<float *>(lds + cv.fM);
    c.fZ = reinterpret_cast<int32_t *>(lds + cv.fZ);
    c.defer = reinterpret_cast<int *>(lds + cv.defer);
    c.total = p.offsets[p.B];
    Shared *sh = c.sh;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int L = p.L, G = gridDim.x;

    // window (create_window, :278-296) -> LDS once; its support [j0, j1] via ballots
    if (tid == 0) {
        sh->j0 = L;
        sh->j1 = -1;
        sh->ndefer = 0;
    }
    __syncthreads();
    for (int q0 = wid * 64; q0 < L; q0 += NT) {
        const int j = q0 + lane;
        const double w = j < L ? p.window[j] : 0.0;
        if (j < L) {
            c.wtab[j] = make_float2((float)w, (float)(w * w));
        }
        const unsigned long long m = __ballot(j < L && w > 0.0);
        if (lane == 0 && m) {
            atomicMin(&sh->j0, q0 + __ffsll((long long)m) - 1);
            atomicMax(&sh->j1, q0 + 63 - __clzll((long long)m));
        }
    }

    short8 regs[NPF];
    int i = blockIdx.x;
    ClipRef cur;
    if (i < p.B) {
        cur = clip_ref(p, i, c.total);
        issue_loads(regs, p.pcm, cur, tid);
    }
    for (; i < p.B; i += G) {
        const bool has_next = i + G < p.B;
        const ClipRef nxt = has_next ? clip_ref(p, i + G, c.total) : ClipRef{0, 0, 0, 0, 0, false};
        if (!cur.ok) {
            write_bad_clip(p, i, tid);
            if (has_next) issue_loads(regs, p.pcm, nxt, tid);
        } else {
            const bool done = clip_body<false>(p, c, i, cur, regs, has_next, nxt);
            if (!done && tid == 0) {
                if (sh->ndefer < EXTRACT_DEFER_CAP) {
                    c.defer[sh->ndefer++] = i;
                } else {  // list full (> EXTRACT_DEFER_CAP near ties in one workgroup)
                    p.status[i] = DSP_CLIP_UNCERTIFIED;
                }
            }
            __syncthreads();  // LDS is rewritten by the next clip
        }
        cur = nxt;
    }
    // near ties (rare): endpoint energies in numpy's exact float64 order, no prefetch live
    __syncthreads();
    const int nd = sh->ndefer;
    for (int d = 0; d < nd; d++) {
        const int j = c.defer[d];
        const ClipRef cr = clip_ref(p, j, c.total);
        clip_body<true>(p, c, j, cr, regs, false, cr);
        __syncthreads();
    }
}

}  // namespace dsp

#ifdef DSP_STAMPS
extern "C" int dsp_debug_set_stamp_buffer(void *buf)
{
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(dsp::g_stamps), &buf, sizeof(buf));
}
extern "C" int dsp_debug_set_dump_buffer(void *buf)
{
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(dsp::g_dump), &buf, sizeof(buf));
}
#endif

extern "C" size_t dsp_extract_lds_bytes(int64_t max_len, int frame_length, int frame_shift)
{
    if (max_len < 1 || frame_length < 1 || frame_shift < 1) return 0;
    if (max_len + 16 > (int64_t)8 * EXTRACT_MAX_ROUNDS * EXTRACT_THREADS) return 0;
    const ExtractCarve c = extract_carve((int)max_len, frame_length, frame_shift, EXTRACT_DEFER_CAP);
    return c.total <= EXTRACT_LDS_LIMIT ? (size_t)c.total : 0;
}

static int g_num_cus = 0;

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
    if (g_num_cus == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
            return DSP_ERR_HIP;
        g_num_cus = prop.multiProcessorCount;
        (void)hipFuncSetAttribute((const void *)dsp::extract_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, EXTRACT_LDS_LIMIT);
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
    // persistent grid: one workgroup per CU (the LDS footprint admits one), each walks clips
    // blockIdx, blockIdx + grid, ...
    const int grid = B < g_num_cus ? B : g_num_cus;
    hipLaunchKernelGGL(dsp::extract_kernel, dim3(grid), dim3(dsp::NT), lds, (hipStream_t)stream, p);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DSP_OK : DSP_ERR_HIP + (int)e;
}
