// extract_hop.h -- hop-major extraction kernel for gfx950 (included by extract.hip).
//
// Same contract as dsp::extract_kernel (one fused pass per clip: preprocess, double-threshold
// VAD, windowed E/M/ZCR of the crop, 15-d statistics), laid out around the frame geometry
// instead of around 32-sample words:
//
//   * the clip is cut into hops of S samples (frame f = hops f .. f+D-1, the last one cut at
//     r = L - (D-1)S samples) and each hop into 64 chunks of C = S/64.. samples; a group of 8
//     lanes holds one hop (lane j: chunks j, j+8, .., j+56, one unaligned 16-B load each), so a
//     wave-instruction reads 8 hops x 112 contiguous bytes;
//   * 512 threads = 64 groups, two hop slots per lane: 128 hops (1.26 s at S = 441) sit in
//     registers from the load to the windowed frames -- nothing is re-read from L2;
//   * every per-frame quantity is a sum of per-hop quantities, so a frame's VAD energy (exact
//     integer moments), its ZCR (sign changes inside hops + the hop junctions) and its windowed
//     E/M are assembled from a few per-hop numbers reduced over the 8 lanes of a group, and
//     the window weights of a lane are the same for every hop (a padded per-lane table in LDS);
//   * the next clip's loads are issued as soon as the windowed frames are done, so they fly
//     while the 15-d statistics are formed.
//
// Decisions are bit-identical to extract_kernel: the VAD frame moments are the same exact
// integers and go through the same energy_from_moments / p90 / vad_scan code; a near tie
// defers the clip to the exact numpy-order redo (clip_exact) after the persistent loop.
//
// Served configurations (host check in dsp_extract_features): S = 64 * C or 63 * C with
// C in {7, 8} (S = 441, 448, 504, 512), D = ceil(L/S) in {2, 3}, clips of at most
// (128 - D + 1) hops, <= 128 VAD and feature frames, a window whose support [j0, j1] has no
// interior zeros (the three reference windows).  Everything else runs on extract_kernel.
#ifndef DSP_EXTRACT_HOP_H
#define DSP_EXTRACT_HOP_H

namespace dsp {

constexpr int HG = 8;                 // lanes per hop group
constexpr int HCH = 8;                // chunks per lane per hop
constexpr int HSLOT = 2;              // hop slots per lane
constexpr int HNG = NT / HG;          // hop groups per workgroup (64)
constexpr int HMAX = HSLOT * HNG;     // hops per clip (128)
constexpr int HWROW = HCH * 3 * 8 + 4;  // floats per lane row of the weight table (+16 B: no bank clash)

struct HopLds {
    float wt[HG][HWROW];  // lane j: [m][d][e] = w[C(8m + j) + e + dS] (0 off the window / chunk)
    int s1f[HMAX], s1a[HMAX];            // per hop: sum k over the hop / over its first r samples
    unsigned s2lf[HMAX], s2hf[HMAX];     // sum k^2 as 16-bit halves of pair sums (no carries)
    unsigned s2la[HMAX], s2ha[HMAX];
    int zf[HMAX], za[HMAX];              // sign changes of pairs inside the hop / inside [0, r)
    int b0[HMAX], bl[HMAX];              // positive bit of the hop's first / last sample
    unsigned long long bmp[HMAX][HG];    // positive bits: lane word j, bit 8m + e
    float pe[HMAX][4], pm[HMAX][4];      // windowed frame partials per (hop, d)
};
constexpr int HOP_LDS_OFF = (extract_carve_fast().total + 15) & ~15;
constexpr int HOP_LDS_TOTAL = HOP_LDS_OFF + (int)sizeof(HopLds);
static_assert(HOP_LDS_TOTAL <= EXTRACT_LDS_SHARED, "hop kernel: two workgroups per CU");

// ---- 8-lane group helpers (lane j = lane & 7) ---------------------------------------------
__device__ __forceinline__ unsigned gx(unsigned v, int m, int lane)  // lane ^ m, m in {1, 2, 4}
{
    return shfl_xor_k(v, m, lane);
}
// Transposed group sum of V <= 8 values: afterwards lane j holds the group's total of value j
// (tree order fixed: (j, j^4), then ^2, then ^1).
template <int V, typename T>
__device__ __forceinline__ T group_sum_t(const T (&a)[V], int lane)
{
    T b[8];
#pragma unroll
    for (int k = 0; k < 8; k++) b[k] = k < V ? a[k] : (T)0;
    const int j = lane & 7;
#pragma unroll
    for (int lv = 4; lv >= 1; lv >>= 1) {
        const bool hi = (j & lv) != 0;
#pragma unroll
        for (int k = 0; k < lv; k++) {
            const T keep = hi ? b[k + lv] : b[k];
            const T send = hi ? b[k] : b[k + lv];
            const T got = __builtin_bit_cast(T, gx(__builtin_bit_cast(unsigned, send), lv, lane));
            b[k] = keep + got;
        }
    }
    return b[0];
}
__device__ __forceinline__ unsigned long long dpp64(unsigned long long v, int ctrl)
{
    unsigned lo = (unsigned)v, hi = (unsigned)(v >> 32);
    if (ctrl == 0x101) {  // row_shl:1 (lane i <- i + 1)
        lo = __builtin_amdgcn_update_dpp(0, (int)lo, 0x101, 0xF, 0xF, true);
        hi = __builtin_amdgcn_update_dpp(0, (int)hi, 0x101, 0xF, 0xF, true);
    } else {  // row_shr:7 (lane i <- i - 7)
        lo = __builtin_amdgcn_update_dpp(0, (int)lo, 0x117, 0xF, 0xF, true);
        hi = __builtin_amdgcn_update_dpp(0, (int)hi, 0x117, 0xF, 0xF, true);
    }
    return ((unsigned long long)hi << 32) | lo;
}

// int16 -> "k >= t" bits of the 8 samples of a chunk (t <= 32767; all zero when t > 32767)
__device__ __forceinline__ unsigned hop_pos8(const short8 &val, short2v tt, bool tbig)
{
    if (tbig) return 0u;
    const unsigned a0 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 0), tt));
    const unsigned a1 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 1), tt));
    const unsigned a2 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 2), tt));
    const unsigned a3 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 3), tt));
    const unsigned x01 = __builtin_amdgcn_perm(a1, a0, 0x07050301u) & 0x80808080u;
    const unsigned x23 = __builtin_amdgcn_perm(a3, a2, 0x07050301u) & 0x80808080u;
    return ~(((x01 * 0x00204081u) >> 28) | (((x23 * 0x00204081u) >> 28) << 4)) & 0xFFu;
}

// wave-uniform values held in SGPRs (a value read from LDS lands in a VGPR otherwise)
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uni(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ double uni(double v)
{
    const long long b = __builtin_bit_cast(long long, v);
    const unsigned lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __builtin_bit_cast(double, (long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ long long uni(long long v)
{
    const unsigned lo = __builtin_amdgcn_readfirstlane((int)v), hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
// a clip's extent in SGPRs: its buffer descriptor must be uniform (else every load becomes a
// readfirstlane waterfall loop)
__device__ __forceinline__ ClipRef hop_ref(const ExtractParams &p, int i)
{
    ClipRef c = clip_ref(p, i);
    c.base = uni((long long)c.base);
    c.lead = uni(c.lead);
    c.n = uni(c.n);
    c.nvec = uni(c.nvec);
    c.nword = uni(c.nword);
    c.ok = uni((int)c.ok) != 0;
    return c;
}

// keep elements [0, cnt) of a chunk, zero the rest (cnt wave-varying, 0..8)
__device__ __forceinline__ short8 hop_keep(const short8 &x, int cnt)
{
    short8 y = x;
#pragma unroll
    for (int e = 0; e < 8; e++) y[e] = e < cnt ? x[e] : (short)0;
    return y;
}

// p90 order statistics (:198) of the nv <= 128 VAD energies in c.vE by wave 0: bitonic sort of
// the high halves of the order-preserving keys; the rank's element is the one holding that
// high half, or, when several do, the one of the right rank among them by the full key
__device__ __forceinline__ void hop_p90(const Ctx &c, int nv, int lane)
{
    const double vi = (double)(nv - 1) * 0.9;
    int r0, r1;
    if (vi >= (double)(nv - 1)) {
        r0 = r1 = nv - 1;
    } else {
        r0 = (int)floor(vi);
        r1 = r0 + 1;
    }
    const unsigned long long f0 = lane < nv ? dkey(c.vE[lane]) : ~0ull;
    const unsigned long long f1 = lane + 64 < nv ? dkey(c.vE[lane + 64]) : ~0ull;
    const unsigned h0 = (unsigned)(f0 >> 32), h1 = (unsigned)(f1 >> 32);
    unsigned a[2] = {h0, h1};
    wave_bitonic<2>(a, lane);
    auto full_at = [&](int r) -> double {
        const unsigned kh = sorted_at<2>(a, r);
        const unsigned long long c0 = __ballot(h0 == kh), c1 = __ballot(h1 == kh);
        if (__popcll(c0) + __popcll(c1) == 1)
            return dkey_value(c0 ? lane_read(f0, __ffsll((long long)c0) - 1) : lane_read(f1, __ffsll((long long)c1) - 1));
        const int rr = r - (__popcll(__ballot(h0 < kh)) + __popcll(__ballot(h1 < kh)));
        unsigned long long res = 0;
        for (int hh = 0; hh < 2; hh++) {
            unsigned long long cm = hh ? c1 : c0;
            while (cm) {
                const int l = __ffsll((long long)cm) - 1;
                cm &= cm - 1;
                const unsigned long long e = lane_read(hh ? f1 : f0, l);
                const int lt = __popcll(__ballot(h0 == kh && f0 < e)) + __popcll(__ballot(h1 == kh && f1 < e));
                const int eq = __popcll(__ballot(f0 == e)) + __popcll(__ballot(f1 == e));
                if (rr >= lt && rr < lt + eq) res = e;
            }
        }
        return dkey_value(res);
    };
    const double pa = full_at(r0), pb = full_at(r1);
    if (lane == 0) {
        c.sh->pa = pa;
        c.sh->pb = pb;
    }
}

// 15-d statistics (compute_statistics x 3, fe.py:46-62) of F <= 128 frames: waves 0-2 the
// medians of E / M / ZCR by an in-wave bitonic sort, waves 3-5 mean / population std (fp64
// sums) / max / min
__device__ __forceinline__ void hop_r5(const Ctx &c, int F, float *featb, int wid, int lane)
{
    if (wid >= 6) return;
    const int r0 = (F - 1) / 2, r1 = F / 2;
    const int q = wid % 3;
    auto get = [&](int j) -> float { return q == 0 ? c.fE[j] : q == 1 ? c.fM[j] : (float)c.fZ[j]; };
    const bool in0 = lane < F, in1 = lane + 64 < F;
    const float x0 = in0 ? get(lane) : 0.f, x1 = in1 ? get(lane + 64) : 0.f;
    if (wid < 3) {
        unsigned a[2] = {in0 ? fkey(x0) : ~0u, in1 ? fkey(x1) : ~0u};
        float v0, v1;
        if (F <= 64) {
            unsigned b[1] = {a[0]};
            wave_bitonic<1>(b, lane);
            v0 = fkey_value(sorted_at<1>(b, r0));
            v1 = fkey_value(sorted_at<1>(b, r1));
        } else {
            wave_bitonic<2>(a, lane);
            v0 = fkey_value(sorted_at<2>(a, r0));
            v1 = fkey_value(sorted_at<2>(a, r1));
        }
        double med;
        {
#pragma clang fp contract(off)
            med = (F & 1) ? (double)v1 : ((double)v0 + (double)v1) / 2.0;
        }
        if (lane == 0) featb[5 * q + 4] = (float)med;
    } else {
        const double s = wave_sum((in0 ? (double)x0 : 0.0) + (in1 ? (double)x1 : 0.0));
        const float mx = wave_reduce(fmaxf(in0 ? x0 : -INFINITY, in1 ? x1 : -INFINITY), OpMax());
        const float mn = wave_reduce(fminf(in0 ? x0 : INFINITY, in1 ? x1 : INFINITY), OpMin());
        const double mean = s / (double)F;
        const double d0 = in0 ? (double)x0 - mean : 0.0, d1 = in1 ? (double)x1 - mean : 0.0;
        const double qq = wave_sum(fma(d0, d0, d1 * d1));
        if (lane < 4) {
            const double o = lane == 0 ? mean : lane == 1 ? sqrt(qq / (double)F) : lane == 2 ? (double)mx : (double)mn;
            featb[5 * q + lane] = (float)o;
        }
    }
}

// Hop geometry of one launch (host-computed, kernel arguments)
struct HopGeo {
    int nch;      // chunks per hop (S / C)
    int r;        // samples of a frame's last hop, r = L - (D-1) S (<= S)
    int ciA, eA;  // [0, r) = chunks ci < ciA and elements e < eA of chunk ciA
};

// the clip's chunks in registers + its last sample (a 16-B load at a 2-B aligned offset that
// straddles the clip buffer's range check returns its last dword as zero: the last sample is
// fetched again by an aligned dword load and patched in)
struct HopRegs {
    short8 v[HSLOT][HCH];
    int last;
};

template <int C>
__device__ __forceinline__ void hop_issue(HopRegs &hr, const ExtractParams &p, const ClipRef &cr, int nhop)
{
    const int tid = threadIdx.x, g = tid >> 3, j = tid & 7, wid = uni(tid >> 6);
    const __amdgpu_buffer_rsrc_t rs = clip_rsrc(p, cr);
    hr.last = __builtin_amdgcn_raw_buffer_load_b32(rs, (2 * (cr.lead + cr.n - 1)) & ~3, 0, 0);
#pragma unroll
    for (int s = 0; s < HSLOT; s++) {
        if (64 * s + 8 * wid >= nhop) continue;  // wave-uniform: no hop of this wave's slot is needed
        const int h = 64 * s + g;
        const int base = 2 * (cr.lead + h * p.S + C * j);
#pragma unroll
        for (int m = 0; m < HCH; m++)
            hr.v[s][m] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16 * C * m, 0, 0));
    }
}

// One clip; its loads are in flight into regs.  Issues the loads of clip `nx` (if nx.ok) once
// the registers are free.  Returns false on a near-tie endpoint decision (clip redone later).
template <int C, int D, bool PA>
__device__ __forceinline__ bool hop_clip(const ExtractParams &p, const HopGeo &hg, const Ctx &c, HopLds *hl, int i,
                                         const ClipRef &cur, const ClipRef &nx, int nhop_nx, HopRegs &hr)
{
    auto &regs = hr.v;
    Shared *sh = c.sh;
    // lane-derived values are recomputed per clip (an opaque thread id): hoisted out of the
    // persistent loop they would hold dozens of registers for the whole kernel
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, g = tid >> 3, j = tid & 7;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    STAMP(i, 0);
    const int L = p.L, S = p.S, n = cur.n;
    const int nch = hg.nch;
    float *featb = p.feat + (size_t)i * 15;
    const int nv = (p.do_vad && n >= L) ? (n - L) / S + 1 : 0;
    const int Fall = n <= L ? 1 : (n - L + S - 1) / S + 1;  // frames of the whole clip (padded last)
    const int nhop = min(HMAX, (Fall - 1) + D);               // hops any frame touches
    // static element validity: elements e >= C of a chunk never belong to it
    constexpr unsigned M3 = C == 7 ? 0x0000FFFFu : 0xFFFFFFFFu;  // dword 3 (elements 6, 7)

    // ---- R1: from registers, everything that does not need the clip mean ------------------
    // integer sum / min / max of the clip; per hop sum k and sum k^2 (16-bit halves of pair
    // sums) over the hop and over its first r samples
    int K = 0;
    short2v pmin = {32767, 32767}, pmax = {-32768, -32768};
#pragma unroll
    for (int s = 0; s < HSLOT; s++) {
        const int hw = 64 * s + 8 * wid;  // first hop of this wave's slot
        if (hw >= nhop) break;
        const int h = 64 * s + g;
        // wave-uniform: every hop of the slot whole, and 8 samples to spare after it -- then the
        // elements a chunk load carries beyond its chunk are still samples of this clip, harmless
        // for min / max, and only the sums need masking
        const bool clean = (hw + 8) * S + 8 <= n;
        if (!clean) {
            // last hops: elements past the clip (or the hop, or the chunk) zeroed in place, the
            // clip's last sample patched (HopRegs), min / max over the real samples only
            const int lim = min(S, n - h * S);
            const short lv = (short)(((2 * (cur.lead + n - 1)) & 2) ? (hr.last >> 16) : (hr.last & 0xFFFF));
#pragma unroll
            for (int m = 0; m < HCH; m++) {
                const int ci = 8 * m + j;
                const int cnt = max(0, min(ci < nch ? C : 0, lim - C * ci));
                const int el = (n - 1) - h * S - C * ci;
                short8 x = regs[s][m];
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    const short v = e == el ? lv : x[e];
                    x[e] = e < cnt ? v : (short)0;
                    const short2v vv = {e < cnt ? v : (short)32767, e < cnt ? v : (short)-32768};
                    pmin.x = min(pmin.x, vv.x);
                    pmax.x = max(pmax.x, vv.y);
                }
                regs[s][m] = x;
            }
        } else if (nch < 64) {
            // the empty chunk (ci >= nch: lane j >= nch - 56 at m = 7) reads the next hop
            const short8 z8 = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 4; k++) pmin = __builtin_elementwise_min(pmin, half_pair(regs[s][HCH - 1], k));
#pragma unroll
            for (int k = 0; k < 4; k++) pmax = __builtin_elementwise_max(pmax, half_pair(regs[s][HCH - 1], k));
            if (8 * (HCH - 1) + j >= nch) regs[s][HCH - 1] = z8;
        }
        int s1 = 0, s1a = 0;
        unsigned qlo = 0, qhi = 0, qloa = 0, qhia = 0;
        const int mA = hg.ciA >> 3, jA = hg.ciA & 7;  // ci < ciA <=> m < mA, or m == mA and j < jA
#pragma unroll
        for (int m = 0; m < HCH; m++) {
            const short8 x = regs[s][m];
            if (clean && !(nch < 64 && m == HCH - 1)) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    pmin = __builtin_elementwise_min(pmin, half_pair(x, k));
                    pmax = __builtin_elementwise_max(pmax, half_pair(x, k));
                }
            }
            const short2v ones = {1, 1};
            int c1 = 0;
            unsigned cl = 0, ch = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                short2v d = half_pair(x, k);
                if (k == 3) d = __builtin_bit_cast(short2v, __builtin_bit_cast(unsigned, d) & M3);
                c1 = __builtin_amdgcn_sdot2(d, ones, c1, false);
                const unsigned q = (unsigned)sq2(d);  // <= 2^31
                cl += q & 0xFFFFu;
                ch += q >> 16;
            }
            s1 += c1;
            qlo += cl;
            qhi += ch;
            if (PA) {  // prefix [0, r) of the hop: chunks ci < ciA whole, chunk ciA in part
                if (m < mA) {
                    s1a += c1;
                    qloa += cl;
                    qhia += ch;
                } else if (m == mA) {
                    const short8 xa = hop_keep(x, j < jA ? C : j == jA ? hg.eA : 0);
                    int a1 = 0;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        short2v d = half_pair(xa, k);
                        if (k == 3) d = __builtin_bit_cast(short2v, __builtin_bit_cast(unsigned, d) & M3);
                        a1 = __builtin_amdgcn_sdot2(d, ones, a1, false);
                        const unsigned q = (unsigned)sq2(d);
                        qloa += q & 0xFFFFu;
                        qhia += q >> 16;
                    }
                    s1a += a1;
                }
            }
        }
        K += s1;
        // per-hop moments: sums over the group's 8 lanes
        if (PA) {
            const unsigned vals[6] = {(unsigned)s1, qlo, qhi, (unsigned)s1a, qloa, qhia};
            const unsigned t = group_sum_t<6>(vals, lane);
            if (h < HMAX) {
                if (j == 0) hl->s1f[h] = (int)t;
                if (j == 1) hl->s2lf[h] = t;
                if (j == 2) hl->s2hf[h] = t;
                if (j == 3) hl->s1a[h] = (int)t;
                if (j == 4) hl->s2la[h] = t;
                if (j == 5) hl->s2ha[h] = t;
            }
        } else {
            const unsigned vals[3] = {(unsigned)s1, qlo, qhi};
            const unsigned t = group_sum_t<3>(vals, lane);
            if (j == 0) hl->s1f[h] = (int)t;
            if (j == 1) hl->s2lf[h] = t;
            if (j == 2) hl->s2hf[h] = t;
        }
    }
    {
        const int kmn = min((int)pmin.x, (int)pmin.y), kmx = max((int)pmax.x, (int)pmax.y);
        const long long ks = (long long)wave_sum(K);
        const int wmn = wave_min(kmn), wmx = wave_max(kmx);
        if (lane == 0) {
            sh->red_k[wid] = ks;
            sh->red_a[wid] = 8 * wid < nhop ? wmn : 0x7fffffff;
            sh->red_b[wid] = 8 * wid < nhop ? wmx : -0x7fffffff - 1;
        }
    }
    __syncthreads();
    STAMP(i, 1);
    // remove_dc / normalize_audio (:49-75) in sample units (as extract_kernel)
    long long Kt = 0;
    int kmin = 0x7fffffff, kmax = -0x7fffffff - 1;
#pragma unroll
    for (int w = 0; w < NWAVE; w++) {
        Kt += sh->red_k[w];
        kmin = min(kmin, sh->red_a[w]);
        kmax = max(kmax, sh->red_b[w]);
    }
    const double mq = uni((double)Kt / (double)n);
    const double Mp = uni(fmax((double)kmax - mq, mq - (double)kmin));
    const int tpos = uni((int)floor(mq) + 1);
    const int t0 = uni((int)floor(mq + 0.5));
    const float deltaf = uni((float)(mq - (double)t0));
    const float invMf = uni(Mp > 0.0 ? __builtin_amdgcn_rcpf((float)Mp) : 0.0f);
    const double invM2 = uni(Mp > 0.0 ? 1.0 / (Mp * Mp) : 0.0);

    // ---- P: positive bits, sign changes per hop ----------------------------------------------
#ifndef HOP_DBG_NOP
    {
        const bool tbig = tpos > 32767;
        const short2v tt = {(short)(tbig ? 32767 : tpos), (short)(tbig ? 32767 : tpos)};
        // pair masks of a lane word (bit 8m + e = chunk ci = 8m + j, element e): pairs inside a
        // chunk, pairs into the next chunk; the same restricted to pairs (o, o+1) with o + 1 < r
        constexpr unsigned long long BYTES = 0x0101010101010101ull;
        constexpr unsigned long long INT = BYTES * ((1u << (C - 1)) - 1), BND = BYTES << (C - 1);
        const int lastc = nch - 1;  // its boundary pair leaves the hop
        const unsigned long long own = (j > (lastc & 7)) ? ~0ull >> (64 - 8 * (lastc >> 3)) : ~0ull;  // chunks < nch
        const unsigned long long nolast = (j == (lastc & 7)) ? ~(1ull << (8 * (lastc >> 3) + C - 1)) : ~0ull;
        const unsigned long long mint = INT & own, mbnd = BND & own & nolast;
        const int mA = hg.ciA >> 3, jA = hg.ciA & 7;
        const int mfull = mA + (j < jA);  // bytes of whole chunks inside [0, r)
        const unsigned long long fullA = mfull >= 8 ? ~0ull : (1ull << (8 * mfull)) - 1;
        unsigned long long mintA = INT & own & fullA, mbndA = BND & own & nolast & fullA;
        if (hg.eA == 0 && mfull > 0 && ((jA + 7) & 7) == j && hg.ciA > 0) {
            // the last whole chunk before r: its pair into chunk ciA has o + 1 = r
            const int mb = (hg.ciA - 1) >> 3;
            mbndA &= ~(1ull << (8 * mb + C - 1));
        }
        if (j == jA && hg.eA > 1 && hg.ciA < nch) mintA |= (unsigned long long)((1u << (hg.eA - 1)) - 1) << (8 * mA);
        if (j == jA && hg.eA > 0 && hg.ciA < nch && hg.eA == C) mbndA |= 0;  // (eA < C always)
#pragma unroll
        for (int s = 0; s < HSLOT; s++) {
            const int hw = 64 * s + 8 * wid;
            if (hw >= nhop) break;
            const int h = 64 * s + g;
            unsigned long long b = 0;
#pragma unroll
            for (int m = 0; m < HCH; m++) {
                // zeroed elements (invalid) read as k = 0: mask them by the chunk's valid count
                const int ci = 8 * m + j;
                int cnt = ci < nch ? C : 0;
                cnt = max(0, min(cnt, n - h * S - C * ci));
                const unsigned byte = hop_pos8(regs[s][m], tt, tbig) & ((1u << cnt) - 1u);
                b |= (unsigned long long)byte << (8 * m);
            }
            // next chunk's first bit: chunk ci + 1 is lane j + 1 (same m) or lane 0 (m + 1)
            const int src = j < 7 ? lane + 1 : lane - 7;
            const unsigned long long nw = ((unsigned long long)(unsigned)__shfl((int)(b >> 32), src) << 32) |
                                          (unsigned)__shfl((int)b, src);
            const unsigned long long nf = j < 7 ? nw : nw >> 8;
            const unsigned long long ch_in = b ^ (b >> 1);
            const unsigned long long ch_bd = b ^ (nf << (C - 1));  // bit 8m + C-1: last of chunk vs next first
            const int zf = __popcll(ch_in & mint) + __popcll(ch_bd & mbnd);
            const int za = __popcll(ch_in & mintA) + __popcll(ch_bd & mbndA);
            hl->bmp[h][j] = b;
            if (j == 0) hl->b0[h] = (int)(b & 1);
            {
                const int cl = nch - 1;  // last chunk of the hop
                if (j == (cl & 7)) hl->bl[h] = (int)((b >> (8 * (cl >> 3) + C - 1)) & 1);
            }
            const int vals[2] = {zf, za};
            const int t = group_sum_t<2>(vals, lane);
            if (j == 0) hl->zf[h] = t;
            if (j == 1) hl->za[h] = t;
        }
    }
#endif
    __syncthreads();
    STAMP(i, 2);

    // ---- VAD frames (:161-185): exact moments and sign changes from the hop sums ------------
    auto frame_z = [&](int f) -> int {
        int z = hl->za[f + D - 1];
#pragma unroll
        for (int d = 0; d < D - 1; d++) z += hl->zf[f + d] + (hl->bl[f + d] != hl->b0[f + d + 1]);
        return z;
    };
    int st = 0, en = n, fc0 = 0;
    if (nv > 0) {
        for (int f = tid; f < nv; f += NT) {
            long long s1 = PA ? hl->s1a[f + D - 1] : hl->s1f[f + D - 1];
            unsigned long long s2 = PA ? ((unsigned long long)hl->s2ha[f + D - 1] << 16) + hl->s2la[f + D - 1]
                                           : ((unsigned long long)hl->s2hf[f + D - 1] << 16) + hl->s2lf[f + D - 1];
#pragma unroll
            for (int d = 0; d < D - 1; d++) {
                s1 += hl->s1f[f + d];
                s2 += ((unsigned long long)hl->s2hf[f + d] << 16) + hl->s2lf[f + d];
            }
            c.vE[f] = energy_from_moments(s2, s1, L, t0, mq - (double)t0, invM2);
            c.vZ[f] = frame_z(f);
        }
        __syncthreads();
        STAMP(i, 3);
#ifndef HOP_DBG_NOTAIL
        if (wid == 0) hop_p90(c, nv, lane);
        if (wid == 1) vad_noise(c, nv, lane);
        __syncthreads();
        STAMP(i, 4);
        if (wid == 0) {
            const int flag = vad_scan<true, true>(p, c, nv, lane);
            if (lane == 0) sh->exact = Mp > 0.0 ? flag : 0;
        }
#else
        if (tid == 0) { sh->exact = 0; sh->n3 = 0; sh->n1 = 30; sh->n6 = 55; }
#endif
        __syncthreads();
        STAMP(i, 5);
        if (uni(sh->exact)) {  // near tie: redone in numpy's exact order after the loop
#ifndef HOP_DBG_NOPF
            if (nx.ok) hop_issue<C>(hr, p, nx, nhop_nx);
#endif
            return false;
        }
        if (uni(sh->n3) >= 0) {
            fc0 = uni(sh->n1);
            st = fc0 * S;                      // :272
            en = min(uni(sh->n6) * S + L, n);  // :273
        }
        if (p.vad_energy)
            for (int f = tid; f < nv && f < p.ld_vad; f += NT) {
                p.vad_energy[(size_t)i * p.ld_vad + f] = c.vE[f];
                p.vad_zcr[(size_t)i * p.ld_vad + f] = c.vZ[f];
            }
    }
    // crop [st, en) (:378): frames st + gS = grid frames fc0 + g (the crop ends on a VAD frame,
    // or is the whole clip with its padded last frame)
    const int m_ = en - st;
    const int F = (m_ <= L) ? 1 : (m_ - L + S - 1) / S + 1;

    // ---- R4: windowed frames (:299-333; fe.py:12-43) from registers -------------------------
    // hop h feeds frame h - d with the weights w[o + dS]; E = sum (w y)^2, M = sum |w y| with
    // y = (k - t0) - delta, scaled by 1/M' at the end
    {
        typedef float float2v __attribute__((ext_vector_type(2)));
        const float t0f = (float)t0;
        const bool near0 = t0 >= -2 && t0 <= 2;
        const float2v mt = {-t0f, -t0f}, md = {-deltaf, -deltaf};
        const float2v mqf = {(float)-mq, (float)-mq};
        const int hlo = fc0, hhi = fc0 + F - 1 + D - 1;  // hops of the crop's frames
#ifndef HOP_DBG_NOR4
#pragma unroll
        for (int s = 0; s < HSLOT; s++) {
            const int hw = 64 * s + 8 * wid;
            if (hw + 7 < hlo || hw > hhi) continue;  // wave-uniform
            const int h = 64 * s + g;
            float2v ea[D];
            float ma[D], mb[D];
#pragma unroll
            for (int d = 0; d < D; d++) {
                ea[d] = (float2v){0.f, 0.f};
                ma[d] = 0.f;
                mb[d] = 0.f;
            }
            const float *wrow = hl->wt[j];
#pragma unroll
            for (int m = 0; m < HCH; m++) {
                // one chunk at a time: scheduled across chunks, the weight reads of all of them
                // would be hoisted and push the clip's registers out
                __builtin_amdgcn_sched_barrier(0);
                const short8 x8 = regs[s][m];  // invalid elements are zero or carry zero weight
                float2v y[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    float2v x = {(float)x8[2 * k], (float)x8[2 * k + 1]};
                    y[k] = near0 ? x + mqf : (x + mt) + md;
                }
                // samples past the clip are zero padding (:322-331), not (0 - mq)
                if (hw + 8 > n / S) {
                    const int o0 = h * S + C * (8 * m + j);
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        y[k].x = o0 + 2 * k < n ? y[k].x : 0.f;
                        y[k].y = o0 + 2 * k + 1 < n ? y[k].y : 0.f;
                    }
                }
#pragma unroll
                for (int d = 0; d < D; d++) {
                    const float4 wa = *reinterpret_cast<const float4 *>(wrow + (m * 3 + d) * 8);
                    const float4 wb = *reinterpret_cast<const float4 *>(wrow + (m * 3 + d) * 8 + 4);
                    const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const float2v w = {wv[2 * k], wv[2 * k + 1]};
                        const float2v u = w * y[k];
                        ea[d] = u * u + ea[d];
                        ma[d] = add_abs(ma[d], u.x);
                        mb[d] = add_abs(mb[d], u.y);
                    }
                    // the sums of this (chunk, d) complete here (else the products are kept
                    // for a late E pass and the clip's registers spill)
                    asm volatile("" : "+v"(ea[d]), "+v"(ma[d]), "+v"(mb[d]));
                }
            }
            float vals[2 * D];
#pragma unroll
            for (int d = 0; d < D; d++) {
                vals[d] = ea[d].x + ea[d].y;
                vals[D + d] = ma[d] + mb[d];
            }
            const float t = group_sum_t<2 * D>(vals, lane);
            if (j < D) hl->pe[h][j] = t;
            else if (j < 2 * D) hl->pm[h][j - D] = t;
        }
#endif
    }
    // the clip's registers are free: the next clip's loads fly during the statistics
#ifndef HOP_DBG_NOPF
    if (nx.ok) hop_issue<C>(hr, p, nx, nhop_nx);
#endif
    __syncthreads();
    STAMP(i, 6);

    // ---- frames of the crop: E, M from the hop partials, ZCR of the windowed frames ----------
    {
        const float sE = invMf * invMf, sM = invMf;
        const int j0 = uni(sh->j0), j1 = uni(sh->j1);
        auto bit = [&](int sidx) -> int {  // positive bit of clip sample sidx (0 past the clip)
            if (sidx < 0 || sidx >= n) return 0;
            const int h = sidx / S, o = sidx - h * S;
            const int ci = o / C, e = o - ci * C;
            return (int)((hl->bmp[h][ci & 7] >> (8 * (ci >> 3) + e)) & 1);
        };
        for (int g2 = tid; g2 < F; g2 += NT) {
            const int f = fc0 + g2;
            float E = 0.f, M = 0.f;
#pragma unroll
            for (int d = 0; d < D; d++) {
                E += hl->pe[f + d][d];
                M += hl->pm[f + d][d];
            }
            int z = frame_z(f);
            // the window's zero ends (Hanning): signs survive only where w_j > 0, j in [j0, j1]
            if (j0 > 0 || j1 < L - 1) {
                const int fs = f * S;
                for (int q = 0; q < j0; q++) z -= bit(fs + q) != bit(fs + q + 1);
                for (int q = j1; q < L - 1; q++) z -= bit(fs + q) != bit(fs + q + 1);
                if (j0 > 0) z += bit(fs + j0);
                if (j1 < L - 1) z += bit(fs + j1);
            }
            c.fE[g2] = E * sE;
            c.fM[g2] = M * sM;
            c.fZ[g2] = z;
        }
    }
    __syncthreads();
    STAMP(i, 7);

    // ---- R5: 15-d statistics ------------------------------------------------------------------
#ifndef HOP_DBG_NOR5
    hop_r5(c, F, featb, wid, lane);
#endif
    if (p.seq)
        for (int g2 = tid; g2 < F && g2 < p.ld_seq; g2 += NT) {
            float *o = p.seq + ((size_t)i * p.ld_seq + g2) * 3;
            o[0] = c.fE[g2];
            o[1] = c.fM[g2];
            o[2] = (float)c.fZ[g2];
        }
    if (tid == 0) {
        p.start_end[2 * i] = st;
        p.start_end[2 * i + 1] = en;
        p.n_frames[i] = F;
        p.status[i] = DSP_CLIP_OK;
    }
    STAMP(i, 8);
    return true;
}

// hops a clip of n samples needs (its frames, with the padded last one)
__device__ __forceinline__ int hop_count(const ExtractParams &p, int n, int D)
{
    const int Fall = n <= p.L ? 1 : (n - p.L + p.S - 1) / p.S + 1;
    return min(HMAX, Fall - 1 + D);
}

// window (create_window, :278-296) -> per-lane weight rows in LDS, support [j0, j1] -> sh
template <int C, int D>
__device__ __forceinline__ void hop_window(const ExtractParams &p, const HopGeo &hg, const Ctx &c, HopLds *hl)
{
    const int tid = threadIdx.x, lane = tid & 63;
    const int L = p.L, S = p.S;
    if (tid == 0) {
        c.sh->j0 = L;
        c.sh->j1 = -1;
        c.sh->ndefer = 0;
    }
    for (int t = tid; t < HG * HCH * 3 * 8; t += NT) {
        const int jj = t / (HCH * 24), rem = t - jj * HCH * 24;
        const int m = rem / 24, d = (rem / 8) % 3, e = rem & 7;
        const int ci = 8 * m + jj;
        const int widx = C * ci + e + d * S;
        const bool in = d < D && e < C && ci < hg.nch && widx < L;
        hl->wt[jj][rem] = in ? (float)p.window[widx] : 0.f;
    }
    __syncthreads();
    for (int q0 = (tid & ~63); q0 < L; q0 += NT) {
        const int jw = q0 + lane;
        const double w = jw < L ? p.window[jw] : 0.0;
        const unsigned long long m = __ballot(jw < L && w > 0.0);
        if (lane == 0 && m) {
            atomicMin(&c.sh->j0, q0 + __ffsll((long long)m) - 1);
            atomicMax(&c.sh->j1, q0 + 63 - __clzll((long long)m));
        }
    }
    __syncthreads();
}

// workgroups per CU (HOP_WG_PER_CU = 1: 256 registers per lane; 2: 128)
#ifndef HOP_WG_PER_CU
#define HOP_WG_PER_CU 1
#endif
template <int C, int D, bool PA>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2 * HOP_WG_PER_CU))) void hop_kernel(ExtractParams p, HopGeo hg)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr ExtractCarve cv = extract_carve_fast();
    const Ctx c = ctx_from(cv, lds);
    HopLds *hl = reinterpret_cast<HopLds *>(lds + HOP_LDS_OFF);
    const int tid = threadIdx.x, G = gridDim.x;

    // the first clip's loads go out before the window setup
    HopRegs hr;
    int i = blockIdx.x;
    ClipRef cur = hop_ref(p, i < p.B ? i : 0);
    if (i < p.B && cur.ok) hop_issue<C>(hr, p, cur, hop_count(p, cur.n, D));
    hop_window<C, D>(p, hg, c, hl);

    for (; i < p.B; i += G) {
        const int inx = i + G;
        ClipRef nx = hop_ref(p, inx < p.B ? inx : i);
        if (inx >= p.B) nx.ok = false;
        const int nhop_nx = nx.ok ? hop_count(p, nx.n, D) : 0;
        if (!cur.ok) {
            write_bad_clip(p, i, tid);
#ifndef HOP_DBG_NOPF
            if (nx.ok) hop_issue<C>(hr, p, nx, nhop_nx);
#endif
        } else if (!hop_clip<C, D, PA>(p, hg, c, hl, i, cur, nx, nhop_nx, hr) && tid == 0) {
            if (c.sh->ndefer < EXTRACT_DEFER_CAP) c.defer[c.sh->ndefer++] = i;
            else p.status[i] = DSP_CLIP_UNCERTIFIED;
        }
        __syncthreads();  // LDS is rewritten by the next clip
        cur = nx;
#ifdef HOP_DBG_NOPF
        if (cur.ok) hop_issue<C>(hr, p, cur, hop_count(p, cur.n, D));
#endif
    }
    // near ties (rare): the generic kernel's exact path, with its own window table
    __syncthreads();
    const int nd = c.sh->ndefer;
#ifndef HOP_DBG_NOEXACT
    if (nd > 0) {
        extract_window_prologue<true>(p, c);
        for (int d = 0; d < nd; d++) {
            clip_exact<true>(c.defer[d]);
            __syncthreads();
        }
    }
#endif
}

}  // namespace dsp

#endif
