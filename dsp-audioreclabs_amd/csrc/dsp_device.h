// dsp_device.h -- device helpers shared by the extraction kernels (csrc/extract.hip,
// csrc/stream.hip): wave reductions on DPP, numpy-order float64 summation (the exact endpoint
// path), positive-bit / sign-change arithmetic, bit sets of ballots and in-wave bitonic sorts.
#ifndef DSP_DEVICE_H
#define DSP_DEVICE_H
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsp {
typedef short short8 __attribute__((ext_vector_type(8)));
template <bool B> struct BoolT {
    static constexpr bool value = B;
};
template <int K> struct IntT {
    static constexpr int value = K;
};
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

// sum_{frame} (k - mq)^2 / M'^2 from the exact moments S1 = sum k, S2 = sum k^2 (L samples).
// With d = k - t0 (t0 = round(mq), delta = mq - t0 exact, |delta| <= 1/2) the moments of d are
// exact integers D1, D2 (< 2^53), and sum (d - delta)^2 = D2 - 2 delta D1 + L delta^2 >= D2 / 4
// (every |d - delta| >= |d| / 2 for d != 0): no cancellation, so plain double evaluation is within
// a few ulp -- far inside the 1e-11 certification margin of the endpoint decisions.
__device__ __forceinline__ double energy_from_moments(unsigned long long S2, long long S1, int L, int t0,
                                                      double delta, double invM2)
{
    const long long D1 = S1 - (long long)L * t0;
    const long long D2 = (long long)S2 - 2LL * t0 * S1 + (long long)L * t0 * t0;
    const double r = fma(-2.0 * delta, (double)D1, (double)D2) + (double)L * delta * delta;
    return r * invM2;  // invM2 = 0 for a constant clip: preprocess leaves zeros (:73-75)
}

// numpy float64 summation order (pairwise_sum in 8192-element buffered chunks): the certified
// fallback of the endpoint energies.  Element i is x_i^2, x_i = fl(fl(k_i - mq) / M').
template <typename T>
__device__ __forceinline__ double xsq(const T *clip, int64_t i, double mq, double Mp)
{
    const double d = (double)clip[i] - mq;
    const double x = Mp > 0.0 ? d / Mp : d;
    return x * x;
}

template <typename T>
__device__ __forceinline__ double pw_leaf(const T *clip, int64_t lo, int n, double mq, double Mp)
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
template <typename T>
__device__ __forceinline__ double pw_block(const T *clip, int64_t lo, int n, double mq, double Mp)
{
    int64_t s_lo[16];
    int s_n[16], s_stage[16];
    double s_left[16];
    int sp = 0;
    s_lo[0] = lo;
    s_n[0] = n;
    s_stage[0] = 0;
    double ret = 0.0;
    bool have = false;
    for (;;) {
        if (!have) {
            const int64_t cl = s_lo[sp];
            const int cn = s_n[sp];
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
        const int64_t pl = s_lo[sp];
        const int pn = s_n[sp];
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

template <typename T>
__device__ __forceinline__ double np_energy_exact(const T *clip, int64_t lo, int n, double mq, double Mp)
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
__device__ __forceinline__ double np_lerp(double a, double b, double g)
{
    const double d = b - a;
    return (g >= 0.5) ? b - d * (1.0 - g) : a + d * g;
}
#pragma clang fp contract(on)

// ---- canonical windowed frame sums (both extraction kernels, so that a clip's features do not
// depend on where it sits in the packed buffer nor on which kernel ran it) ------------------------
// A feature frame at clip sample fs with lim real samples (frame_signal :322-331) is summed over
// the clip's 8-sample vectors v = va .. vb (va = fs >> 3, vb = (fs + lim - 1) >> 3; vector v =
// clip samples 8v .. 8v + 7) by 16 lanes: lane l takes v = va + l + 16k in increasing k, and each
// vector's pairs h = 0..3 in order, with j = 8v + 2h (+1) - fs, w = w_j for 0 <= j < lim (else 0),
//   x = (float)k + xa            (near0: |round(mq)| <= 2; xa = fl(-mq), one rounding of k - mq)
//   x = ((float)k + xa) + xb     (otherwise: xa = -t0, xb = -(mq - t0); k - t0 exact)
//   y = w x,  e_t = fma(y_t, y_t, e_t),  m_t = m_t + |y_t|   (t = the pair's first / second sample)
// Lane value (e_0 + e_1, m_0 + m_1); the frame's sum is dpp_row_reduce over the 16 lanes.
struct CanonX {
    float xa, xb;
    bool near0;
};
__device__ __forceinline__ CanonX canon_x(double mq, int t0)
{
    CanonX c;
    c.near0 = t0 >= -2 && t0 <= 2;
    c.xa = c.near0 ? (float)-mq : (float)-t0;
    c.xb = c.near0 ? 0.f : -(float)(mq - (double)t0);  // mq - t0 exact (Sterbenz)
    return c;
}
typedef float float2v __attribute__((ext_vector_type(2)));
#pragma clang fp contract(off)
__device__ __forceinline__ float canon_xval(int k, const CanonX &c)
{
    return c.near0 ? (float)k + c.xa : ((float)k + c.xa) + c.xb;
}
// x of a sample pair, packed (v_pk_add_f32): the same bits as canon_xval per sample (with
// NEAR0 = false on a near0 clip, xb = +0 and fl(k + xa) + 0 = fl(k + xa): a zero sum is +0 in
// round-to-nearest, so the bits are those of NEAR0 = true)
template <bool NEAR0>
__device__ __forceinline__ float2v canon_x2(int k0, int k1, const CanonX &c)
{
    const float2v k = {(float)k0, (float)k1};
    const float2v a = {c.xa, c.xa}, b = {c.xb, c.xb};
    return NEAR0 ? k + a : (k + a) + b;
}
#pragma clang fp contract(on)
// one pair: weights w, x values x; y = w x (v_pk_mul_f32), e = fma(y, y, e) (v_pk_fma_f32),
// m_t += |y_t| (v_add_f32 with the abs source modifier) -- per component exactly the scalar ops
__device__ __forceinline__ float add_abs_f(float acc, float v)
{
    float r;
    asm("v_add_f32_e64 %0, |%1|, %2" : "=v"(r) : "v"(v), "v"(acc));
    return r;
}
__device__ __forceinline__ void canon_pair(float2v w, float2v x, float2v &e, float &m0, float &m1)
{
    const float2v y = w * x;
    e = __builtin_elementwise_fma(y, y, e);
    m0 = add_abs_f(m0, y.x);
    m1 = add_abs_f(m1, y.y);
}

// acc + |v| in one VOP3 add with the abs source modifier
__device__ __forceinline__ float add_abs(float acc, float v)
{
    float r;
    asm("v_add_f32_e64 %0, |%1|, %2" : "=v"(r) : "v"(v), "v"(acc));
    return r;
}
// k0^2 + k1^2 of a sample pair in one VOP3 v_dot2 with an inline-zero accumulator (the builtin
// becomes v_mov 0 + v_dot2c)
__device__ __forceinline__ int sq2(short2v d)
{
    int r;
    asm("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(r) : "v"(d));
    return r;
}

// acc + k0^2 + k1^2 in one v_dot2_i32_i16 (32-bit, wrapping)
__device__ __forceinline__ int sq2acc(short2v d, int acc)
{
    int r;
    asm("v_dot2_i32_i16 %0, %1, %1, %2" : "=v"(r) : "v"(d), "v"(acc));
    return r;
}

__device__ __forceinline__ short2v half_pair(const short8 &x, int i)
{
    switch (i) {
    case 0: return __builtin_shufflevector(x, x, 0, 1);
    case 1: return __builtin_shufflevector(x, x, 2, 3);
    case 2: return __builtin_shufflevector(x, x, 4, 5);
    default: return __builtin_shufflevector(x, x, 6, 7);
    }
}

// sign-change bits of buffer word w: bit b <-> (pos(32w+b) != pos(32w+b+1))
__device__ __forceinline__ uint32_t chg_word(const uint32_t *posw, int w)
{
    const uint32_t a = posw[w], b = posw[w + 1];
    return a ^ ((a >> 1) | (b << 31));
}
// set change bits in buffer-bit range [x0, x1), words split over `nl` lanes starting at `l0`
__device__ __forceinline__ int chg_count(const uint32_t *posw, int x0, int x1, int l0, int nl)
{
    int c = 0;
    if (x1 > x0) {
        const int w0 = x0 >> 5, w1 = (x1 - 1) >> 5;
#pragma unroll 3
        for (int w = w0 + l0; w <= w1; w += nl) {
            uint32_t m = chg_word(posw, w);
            if (w == w0) m &= ~0u << (x0 & 31);
            if (w == w1 && (x1 & 31)) m &= (1u << (x1 & 31)) - 1u;
            c += __popc(m);
        }
    }
    return c;
}
// set change bits in buffer-bit range [x0, x1), one lane walking the words in order (each
// positive-bit word is read once)
__device__ __forceinline__ int chg_run(const uint32_t *posw, int x0, int x1)
{
    if (x1 <= x0) return 0;
    const int w0 = x0 >> 5, w1 = (x1 - 1) >> 5;
    uint32_t a = posw[w0];
    int cnt = 0;
#pragma unroll 4
    for (int w = w0; w <= w1; w++) {
        const uint32_t b = posw[w + 1];
        cnt += __popc(a ^ ((a >> 1) | (b << 31)));
        a = b;
    }
    // remove the bits below x0 and from x1 on
    const uint32_t c0 = chg_word(posw, w0), c1 = chg_word(posw, w1);
    cnt -= __popc(c0 & ((1u << (x0 & 31)) - 1u));
    if (x1 & 31) cnt -= __popc(c1 & (~0u << (x1 & 31)));
    return cnt;
}
__device__ __forceinline__ int pos_bit(const uint32_t *posw, int u) { return (posw[u >> 5] >> (u & 31)) & 1; }

// ---- frame bit sets of KC ballots (wave-uniform), KC * 64 frames --------------------------
template <int KC> struct BitsK {
    unsigned long long w[KC];
};
template <int KC>
__device__ __forceinline__ int bits_first_ge(const BitsK<KC> &m, int from)  // lowest set >= from, or -1
{
#pragma unroll
    for (int k = 0; k < KC; k++) {
        const int sh = from - 64 * k;
        unsigned long long x = m.w[k];
        if (sh >= 64) x = 0;
        else if (sh > 0) x &= ~0ull << sh;
        if (x) return 64 * k + __ffsll((long long)x) - 1;
    }
    return -1;
}
template <int KC>
__device__ __forceinline__ int bits_last_lt(const BitsK<KC> &m, int below)  // highest set < below, or -1
{
#pragma unroll
    for (int k = KC - 1; k >= 0; k--) {
        const int sh = below - 64 * k;
        unsigned long long x = m.w[k];
        if (sh <= 0) x = 0;
        else if (sh < 64) x &= (1ull << sh) - 1ull;
        if (x) return 64 * k + 63 - __clzll((long long)x);
    }
    return -1;
}
template <int KC>
__device__ __forceinline__ bool bits_any_in(const BitsK<KC> &m, int lo, int hi)  // any set in [lo, hi)
{
    const int f = bits_first_ge(m, lo);
    return f >= 0 && f < hi;
}

__device__ __forceinline__ unsigned long long dpp_quad_sum64(unsigned long long v)
{
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const int ctl = s == 0 ? DPP_QXOR1 : DPP_QXOR2;
        const unsigned lo = dpp_i((int)(unsigned)v, ctl), hi = dpp_i((int)(unsigned)(v >> 32), ctl);
        v += ((unsigned long long)hi << 32) | lo;
    }
    return v;
}
__device__ __forceinline__ long long dpp_quad_sum_i64(long long v)
{
    return (long long)dpp_quad_sum64((unsigned long long)v);
}

// ---- order statistics by an in-wave bitonic sort -------------------------------------------
// Keys are unsigned integers whose order is the value order (equal keys <=> equal values, so
// ties need no index), two per lane at most (element lane + 64h in a[h]); pad with the max key.
__device__ __forceinline__ unsigned long long dkey(double v)
{
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __forceinline__ double dkey_value(unsigned long long k)
{
    return __builtin_bit_cast(double, (k >> 63) ? (k & ~(1ull << 63)) : ~k);
}
__device__ __forceinline__ unsigned fkey(float v)
{
    const unsigned b = __builtin_bit_cast(unsigned, v);
    return (b >> 31) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_value(unsigned k)
{
    return __builtin_bit_cast(float, (k >> 31) ? (k & 0x7FFFFFFFu) : ~k);
}
// value of lane ^ m without the LDS crossbar: DPP for 1, 2, 8, swizzle for 4, the gfx950
// permlane swaps for 16, 32 (checked against __shfl_xor by tools/ubench/perm_check.hip)
__device__ __forceinline__ unsigned shfl_xor_k(unsigned v, int m, int lane)
{
    const int x = (int)v;
    switch (m) {
    case 1: return (unsigned)__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);
    case 2: return (unsigned)__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);
    case 4:  // i ^ 4 = (i ^ 7) ^ 3: row_half_mirror, then quad_perm [3,2,1,0] (two DPP moves, no LDS)
        return (unsigned)__builtin_amdgcn_update_dpp(0, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false),
                                                     0x1B, 0xF, 0xF, false);
    case 8: return (unsigned)__builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);
    case 16: {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (unsigned)((lane & 16) ? r[0] : r[1]);
    }
    default: {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (unsigned)((lane & 32) ? r[0] : r[1]);
    }
    }
}
__device__ __forceinline__ unsigned long long shfl_xor_k(unsigned long long v, int m, int lane)
{
    const unsigned lo = shfl_xor_k((unsigned)v, m, lane), hi = shfl_xor_k((unsigned)(v >> 32), m, lane);
    return ((unsigned long long)hi << 32) | lo;
}
// lane ^ m for m = 16 or 32 by the gfx950 permlane swaps (no LDS crossbar; tools/ubench/perm_check.hip)
__device__ __forceinline__ float lane_xor_f(float v, int m, int lane)
{
    const int x = __float_as_int(v);
    if (m == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return __int_as_float((lane & 16) ? r[0] : r[1]);
    }
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return __int_as_float((lane & 32) ? r[0] : r[1]);
}
// NMAX < 64 (NH = 1): only the stages of a sort of NMAX-element groups -- each group of NMAX lanes
// sorted on its own (keys past the real ones padded with the max key)
template <int NH, typename K, int NMAX = 64 * NH>
__device__ __forceinline__ void wave_bitonic(K (&a)[NH], int lane)
{
    static_assert(NMAX == 64 * NH || (NH == 1 && NMAX >= 2 && NMAX < 64 && (NMAX & (NMAX - 1)) == 0), "group size");
    // the lane index opaque here: the per-stage lane masks are then computed where they are used
    // instead of being hoisted out of a persistent loop and held (spilled) in SGPR pairs
    asm volatile("" : "+v"(lane));
    constexpr int N = NMAX;
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (NH == 2 && stride == 64) {  // partner in the same lane; size == 128: ascending
                const bool sw = a[NH - 1] < a[0];
                const K lo = sw ? a[NH - 1] : a[0], hi = sw ? a[0] : a[NH - 1];
                a[0] = lo;
                a[NH - 1] = hi;
            } else {
#pragma unroll
                for (int h = 0; h < NH; h++) {
                    const int i = lane + 64 * h;
                    const K q = shfl_xor_k(a[h], stride, lane);
                    const bool takemin = ((i & stride) == 0) == ((i & size) == 0);
                    const bool qless = q < a[h];
                    a[h] = (takemin == qless) ? q : a[h];
                }
            }
        }
    }
}
// the r-th and (r+1)-th smallest (0-based, wave-uniform r) of the 32-bit keys a[0..NH-1] of all 64
// lanes, by a ballot radix select from the top bit: per bit one v_bfe + compare per register, the
// candidate sets and counts in scalar registers -- 2 NH VALU per bit against bitonic's ~7 NH per
// compare-exchange stage (21 stages for 64 keys, 28 for 128).  Pads must be ~0u and r + 1 < the
// number of real keys (or r + 1 == it with r1 then read as the r-th's successor, which exists).
template <int NH>
__device__ __forceinline__ void wave_select2(const unsigned (&a)[NH], int r, unsigned &k0, unsigned &k1)
{
    unsigned long long cand[NH];
#pragma unroll
    for (int h = 0; h < NH; h++) cand[h] = ~0ull;
    unsigned pre = 0;
    int rr = r;
#pragma unroll
    for (int b = 31; b >= 0; b--) {
        unsigned long long z[NH];
        int zeros = 0;
#pragma unroll
        for (int h = 0; h < NH; h++) {
            z[h] = cand[h] & ~__ballot(__builtin_amdgcn_ubfe(a[h], b, 1) != 0u);
            zeros += __popcll(z[h]);
        }
        const bool low = rr < zeros;  // wave-uniform
#pragma unroll
        for (int h = 0; h < NH; h++) cand[h] = low ? z[h] : cand[h] & ~z[h];
        rr = low ? rr : rr - zeros;
        pre = low ? pre : pre | (1u << b);
    }
    k0 = pre;
    // the (r+1)-th: the same key when more than rr + 1 keys equal it, else the smallest key above
    int eq = 0;
#pragma unroll
    for (int h = 0; h < NH; h++) eq += __popcll(cand[h]);
    if (rr + 1 < eq) {
        k1 = pre;
    } else {
        unsigned m = ~0u;
#pragma unroll
        for (int h = 0; h < NH; h++) m = min(m, a[h] > pre ? a[h] : ~0u);
        k1 = (unsigned)wave_reduce((int)(m ^ 0x80000000u), OpMin()) ^ 0x80000000u;  // unsigned min
    }
}
template <int NH, typename K>
__device__ __forceinline__ K sorted_at(const K (&a)[NH], int r)  // wave-uniform r
{
    return lane_read((NH == 2 && r >= 64) ? a[NH - 1] : a[0], r & 63);
}

}  // namespace dsp
#endif
