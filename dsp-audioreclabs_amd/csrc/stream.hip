// stream.hip -- the two-kernel extraction path for gfx950 (CDNA4): every launch whose clips fit
// the register plan (<= 49 145 samples, frame_length <= 1276, frame_shift >= 32, <= 128 frames).
//
//   frame_kernel   HBM-streaming.  Persistent 512-thread workgroups (two per CU) walk the batch;
//                  a clip is read from HBM once, straight into registers (three 32-sample words
//                  per thread, coalesced 16-B buffer loads), and EVERY per-sample quantity is
//                  computed from those registers: exact integer mean / peak (preprocess), exact
//                  per-word moments (endpoint energies), positive-sample bits (every ZCR), and
//                  the windowed E / M of every frame the clip has -- the crop is not known yet,
//                  so all candidate frames are windowed (2.5 frames per sample at 1102/441).
//                  It writes a ~2 KB frame summary per clip and nothing else.  No phase of it
//                  depends on a decision, so nothing serial sits between one clip's loads and
//                  the next: the two workgroups of a CU keep HBM busy.
//   decide_kernel  One wave per clip over the frame summary: noise estimates, p90, the
//                  double-threshold scan (certified; near ties redone in numpy's exact order from
//                  the PCM), the crop, and the 15 statistics.  Its work is ~1 k instructions per
//                  clip with no HBM stream behind it.
//
// Reference functions restated (Hypersonic-cpu/DSP-AudioRecLabs):
//   preprocess              src/audio_processing.py:78-90
//   endpoint_detection      src/audio_processing.py:135-275
//   frame_signal + crop     src/audio_processing.py:299-333, :378
//   extract_frame_features  src/feature_extraction.py:12-43
//   compute_statistics / extract_statistical_features  src/feature_extraction.py:46-88
//
// Crop frames are summary frames: with endpoint detection on and a high-energy frame found, the
// crop is [N1 S, N6 S + L) (:272-273; N6 S + L <= n always), so crop frame g is frame N1 + g with
// no zero padding; otherwise the crop is the whole clip and its frames are frames 0 .. F-1, the
// last one zero-padded past n (:322-331).  The summary therefore holds the windowed E / M / ZCR of
// frames 0 .. ceil((n-L)/S) computed over the whole clip with zero padding past n.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dsp_audiorec.h"
#include "dsp_device.h"
#include "extract_layout.h"
#include "stream.h"

namespace dsp {
namespace st {

#ifndef STREAM_NT
#define STREAM_NT 512
#define STREAM_RREG 3
#endif
#ifndef STREAM_WPE
#define STREAM_WPE 4  // waves per SIMD the register budget allows (two 512-thread workgroups per CU)
#endif
constexpr int NT = STREAM_NT;
constexpr int NWAVE = NT / 64;
constexpr int RREG = STREAM_RREG;     // 32-sample words per thread (word r * NT + tid)
constexpr int NRV = 4 * RREG;         // 16-B vectors per thread
constexpr int NWORD = NT * RREG;      // 1536 words = 49 152 buffer samples
constexpr int WPAD = STREAM_WPAD;     // zero weights on each side of every window copy
constexpr int WROWF = STREAM_WROWF;   // floats per shifted window copy (logical)
// physical layout of a copy: 4 pad floats after every 32, so that lanes reading 32 consecutive
// weights each from word-aligned positions (128 B apart) are 36 dwords apart: conflict-free
// ds_read_b128 (16 lanes per LDS cycle, bank = dword mod 64)
constexpr int WROWP = WROWF + 4 * (WROWF / 32);
__host__ __device__ constexpr int wphys(int m) { return m + 4 * (m >> 5); }
constexpr int PQ = STREAM_PQ;         // 128-sample quads one frame can overlap
constexpr int NVCAP = STREAM_FCAP, FCAP = STREAM_FCAP;

struct FrameParams {
    const int16_t *pcm;
    const int64_t *offsets;
    int B, ncap, L, S;
    const double *window;
    int do_vad;
    unsigned char *rec;
    RecLayout rl;
};

struct DecideParams {
    const int16_t *pcm;
    const int64_t *offsets;
    int B, ncap, L, S, do_vad;
    double hi, lo, zr;
    const unsigned char *rec;
    RecLayout rl;
    float *feat;
    int32_t *start_end, *n_frames, *status;
    double *vad_energy;
    int32_t *vad_zcr;
    int ld_vad;
    float *seq;
    int ld_seq;
};

// LDS of one frame_kernel workgroup (~77 KB: two workgroups per CU)
struct Lds {
    long long red_k[NWAVE];
    int red_a[NWAVE], red_b[NWAVE];
    int j0w, j1w;                        // window support: first / last strictly positive weight
#ifndef STREAM_NO_WINDOW
    alignas(16) float wtab[4][WROWP];    // copy c: w[j] at wphys(j + WPAD + c), zero elsewhere
#endif
    uint32_t posw[NWORD + 2];            // bit u: buffer sample u is real and positive
    int wS1[NWORD];                      // per word: sum k (exact)
    unsigned long long wS2[NWORD];       // per word: sum k^2 (exact)
    alignas(16) uint32_t bnd[2 * NVCAP][16];  // raw words holding an endpoint frame's start / end
    int pS1[2 * NVCAP];                  // moments of the covered part of those words
    unsigned long long pS2[2 * NVCAP];
#ifndef STREAM_NO_WINDOW
    float2 part[FCAP][PQ];               // windowed (E, M) of frame f over quad qa(f) + slot
#endif
};

struct Clip {
    int64_t base;  // 8-aligned first sample index of the clip's vectors
    int lead, n, nvec, nword;
    bool ok;
};

__device__ __forceinline__ Clip clip_from(int64_t o0, int64_t o1, int ncap)
{
    Clip c;
    const int64_t nn = o1 - o0;
    c.ok = nn > 0 && nn <= ncap;
    c.n = c.ok ? (int)nn : 0;
    c.base = o0 & ~(int64_t)7;
    c.lead = (int)(o0 - c.base);
    c.nvec = c.ok ? (c.lead + c.n + 7) >> 3 : 0;
    c.nword = (c.lead + c.n + 31) >> 5;
    return c;
}

// 16-B vectors of the clip through a buffer descriptor spanning them: a vector past the clip
// reads zeros (range check), so the loads need no clamping.  Bytes outside [lead, lead + n) are
// masked by every consumer.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const int16_t *pcm, const Clip &c)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t *>(pcm + c.base), 0, c.nvec * 16, 0x00020000);
}

__device__ __forceinline__ float quad_sumf(float v)
{
    v += __builtin_bit_cast(float, dpp_i(__builtin_bit_cast(int, v), DPP_QXOR1));
    return v + __builtin_bit_cast(float, dpp_i(__builtin_bit_cast(int, v), DPP_QXOR2));
}

// which endpoint frame end lies inside word w (owner side of vad_partial_word's rule): slot
// t = 2f (frame f starts inside the word) / 2f + 1 (ends inside it), or -1.  S >= 32: at most
// one start and one end per word.
__device__ __forceinline__ void word_boundaries(int w, int lead, int L, int S, int nv, int &ts, int &te)
{
    ts = te = -1;
    {
        const int num = 32 * w - lead;
        const int f = num <= 0 ? 0 : (num + S - 1) / S;
        const int u0 = lead + f * S;
        if (f < nv && u0 < 32 * w + 32 && (u0 & 31)) ts = 2 * f;
    }
    {
        const int num = 32 * w + 1 - lead - L;
        const int f = num <= 0 ? 0 : (num + S - 1) / S;
        const int u0 = lead + f * S, u1 = u0 + L;
        if (f < nv && u1 >= 32 * w + 1 && u1 <= 32 * w + 32 && (u1 & 31)) {
            const int wa = u0 >> 5, wb = (u1 - 1) >> 5;
            if (wb != wa || !(u0 & 31)) te = 2 * f + 1;
        }
    }
}

// element range [e0, e1) of buffer word `pw` that endpoint frame end t covers (reader side)
__device__ __forceinline__ int boundary_word(int t, int lead, int L, int S, int nv, int &e0, int &e1)
{
    e0 = e1 = 0;
    if (t >= 2 * nv) return -1;
    const int f = t >> 1;
    const int u0 = lead + f * S, u1 = u0 + L;
    const int wa = u0 >> 5, wb = (u1 - 1) >> 5;
    if (!(t & 1)) {
        if (!(u0 & 31)) return -1;
        e0 = u0 & 31;
        e1 = min(32, u1 - 32 * wa);
        return wa;
    }
    if ((u1 & 31) && (wb != wa || !(u0 & 31))) {
        e0 = max(0, u0 - 32 * wb);
        e1 = u1 & 31;
        return wb;
    }
    return -1;
}

// ------------------------------------------------------------------------------------------
// frame_kernel
// ------------------------------------------------------------------------------------------
template <int R>  // frames one 128-sample quad can overlap: (127 + L) / S + 1
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(STREAM_WPE))) void frame_kernel(FrameParams p)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    Lds &s = *reinterpret_cast<Lds *>(lds_raw);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int L = p.L, S = p.S;

    // create_window (:278-296) -> four shifted, zero-padded fp32 copies; support [j0w, j1w]
#ifndef STREAM_NO_WINDOW
    for (int t = tid; t < 4 * WROWP; t += NT) (&s.wtab[0][0])[t] = 0.f;
#endif
    if (tid == 0) {
        s.j0w = L;
        s.j1w = -1;
    }
    __syncthreads();
    for (int q0 = wid * 64; q0 < L; q0 += NT) {
        const int j = q0 + lane;
        const bool in = j < L;
        const double w = in ? p.window[j] : 0.0;
#ifndef STREAM_NO_WINDOW
        if (in) {
#pragma unroll
            for (int c = 0; c < 4; c++) s.wtab[c][wphys(j + WPAD + c)] = (float)w;
        }
#endif
        const unsigned long long m = __ballot(in && w > 0.0);
        if (lane == 0 && m) {
            atomicMin(&s.j0w, q0 + __ffsll((long long)m) - 1);
            atomicMax(&s.j1w, q0 + 63 - __clzll((long long)m));
        }
    }
    __syncthreads();
    const int j0w = s.j0w, j1w = s.j1w;
    const RecLayout rl = p.rl;

    short8 regs[NRV];
    // the clip's three words per thread straight into registers; a clip that does not fit (or
    // none) has an empty descriptor range and reads zeros
    auto issue = [&](const Clip &c) {
        const __amdgpu_buffer_rsrc_t rs = rsrc(p.pcm, c);
#pragma unroll
        for (int r = 0; r < RREG; r++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                regs[4 * r + k] = __builtin_bit_cast(
                    short8, __builtin_amdgcn_raw_buffer_load_b128(rs, 64 * (r * NT + tid) + 16 * k, 0, 0));
    };
    // the offsets of the workgroup's next clip are read one clip ahead: a scalar load issued
    // right before a clip's loads would put an L2 round trip (under full HBM load) in front of
    // every clip's HBM stream
    const int G = gridDim.x;
    int64_t on0 = 0, on1 = 0;
    if ((int)blockIdx.x < p.B) {
        on0 = p.offsets[blockIdx.x];
        on1 = p.offsets[blockIdx.x + 1];
    }
    for (int i = blockIdx.x; i < p.B; i += G) {
        const Clip cur = clip_from(on0, on1, p.ncap);
        if (i + G < p.B) {
            on0 = p.offsets[i + G];
            on1 = p.offsets[i + G + 1];
        }
        if (!cur.ok) continue;  // decide_kernel reports the clip
        issue(cur);
        const int n = cur.n, lead = cur.lead, nword = cur.nword;

        // ---- R1: exact integer sum / min / max; exact moments per word --------------------
        int K = 0;
        int kmin_s = 0x7fffffff, kmax_s = -0x7fffffff - 1;
        short2v pmin = {32767, 32767}, pmax = {-32768, -32768};
#pragma unroll
        for (int r = 0; r < RREG; r++) {
            const int w = r * NT + tid;
            if (w >= nword) continue;
            const short8 *q = &regs[4 * r];
            int s1 = 0;
            unsigned long long s2 = 0;
            if (w > 0 && w < nword - 1) {
                const short2v ones = {1, 1};
#pragma unroll
                for (int k = 0; k < 4; k++)
#pragma unroll
                    for (int h = 0; h < 4; h++) {
                        const short2v d = half_pair(q[k], h);
                        pmin = __builtin_elementwise_min(pmin, d);
                        pmax = __builtin_elementwise_max(pmax, d);
                        s1 = __builtin_amdgcn_sdot2(d, ones, s1, false);
                        s2 += (unsigned)sq2(d);
                    }
            } else {  // first / last word: real samples only
#pragma unroll 1
                for (int k = 0; k < 4; k++) {
                    const short8 v = k == 0 ? q[0] : k == 1 ? q[1] : k == 2 ? q[2] : q[3];
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const int u = 32 * w + 8 * k + e;
                        const int x = v[e];
                        if (u >= lead && u < lead + n) {
                            s1 += x;
                            s2 += (unsigned)(x * x);
                            kmin_s = min(kmin_s, x);
                            kmax_s = max(kmax_s, x);
                        }
                    }
                }
            }
            s.wS1[w] = s1;
            s.wS2[w] = s2;
            K += s1;
        }
        {
            const int kmn = min(kmin_s, min((int)pmin.x, (int)pmin.y));
            const int kmx = max(kmax_s, max((int)pmax.x, (int)pmax.y));
            const long long ks = (long long)wave_sum(K);
            const int wmn = wave_min(kmn), wmx = wave_max(kmx);
            if (lane == 0) {
                s.red_k[wid] = ks;
                s.red_a[wid] = wmn;
                s.red_b[wid] = wmx;
            }
        }
        __syncthreads();
        // remove_dc / normalize_audio (:49-75): the float64 mean of k/32768 is exact, so
        // mq = fl(K/n) and M' = max(fl(kmax - mq), fl(mq - kmin)) are the reference's values in
        // sample units; a sample is positive after preprocess <=> k >= floor(mq) + 1.
        long long Kt = 0;
        int kmin = 0x7fffffff, kmax = -0x7fffffff - 1;
#pragma unroll
        for (int w = 0; w < NWAVE; w++) {
            Kt += s.red_k[w];
            kmin = min(kmin, s.red_a[w]);
            kmax = max(kmax, s.red_b[w]);
        }
        const double mq = (double)Kt / (double)n;
        const double Mp = fmax((double)kmax - mq, mq - (double)kmin);
        const int tpos = (int)floor(mq) + 1;
        const int t0 = (int)floor(mq + 0.5);
        const float deltaf = (float)(mq - (double)t0);  // exact (Sterbenz)
        const float invMf = Mp > 0.0 ? __builtin_amdgcn_rcpf((float)Mp) : 0.0f;
        const double invM2 = Mp > 0.0 ? 1.0 / (Mp * Mp) : 0.0;
        const int nv = (p.do_vad && n >= L) ? (n - L) / S + 1 : 0;
        const int Fmax = n <= L ? 1 : (n - L + S - 1) / S + 1;
        const int nquad = (nword + 3) >> 2;

#ifdef STREAM_ABL
        if (STREAM_ABL >= 3) {
            if (tid == 0) p.rec[(size_t)i * rl.stride] = (unsigned char)(Kt + kmin + kmax);
            __syncthreads();
            continue;
        }
#endif
        // ---- R2: positive bits, endpoint boundary words, windowed frames -------------------
        const bool tbig = tpos > 32767;
        const short2v tt = {(short)(tbig ? 32767 : tpos), (short)(tbig ? 32767 : tpos)};
        // x = k - mq in fp32: |t0| <= 2: k - fl(mq) (|error| <= 2^-22 absolute, < 1e-6 of any frame
        // sum of an integer signal); otherwise (k - t0) exactly, then - delta
        const bool near0 = t0 >= -2 && t0 <= 2;
        const float xa = near0 ? (float)mq : (float)t0, xb = near0 ? 0.f : deltaf;
#pragma unroll
        for (int r = 0; r < RREG; r++) {
            const int w = r * NT + tid;
            const short8 *q = &regs[4 * r];
            if (w < nword) {
                auto pos_byte = [&](const short8 &val) -> uint32_t {
                    if (tbig) return 0u;
                    const unsigned a0 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 0), tt));
                    const unsigned a1 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 1), tt));
                    const unsigned a2 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 2), tt));
                    const unsigned a3 = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, 3), tt));
                    const unsigned x01 = __builtin_amdgcn_perm(a1, a0, 0x07050301u) & 0x80808080u;
                    const unsigned x23 = __builtin_amdgcn_perm(a3, a2, 0x07050301u) & 0x80808080u;
                    return ~(((x01 * 0x00204081u) >> 28) | (((x23 * 0x00204081u) >> 28) << 4)) & 0xFFu;
                };
                uint32_t P = pos_byte(q[0]) | (pos_byte(q[1]) << 8) | (pos_byte(q[2]) << 16) | (pos_byte(q[3]) << 24);
                if (w == 0 || w == nword - 1) {
                    const int lo_ = min(max(lead - 32 * w, 0), 32), hi_ = min(max(lead + n - 32 * w, 0), 32);
                    const uint32_t mhi = hi_ >= 32 ? ~0u : ((1u << hi_) - 1u);
                    const uint32_t mlo = lo_ >= 32 ? 0u : ~((1u << lo_) - 1u);
                    P &= mhi & mlo;
                }
                s.posw[w] = P;
                if (nv > 0) {  // raw copies of the words holding an endpoint frame's ends (pass A)
                    int ts, te;
                    word_boundaries(w, lead, L, S, nv, ts, te);
                    if (ts >= 0)
#pragma unroll
                        for (int k = 0; k < 4; k++) *reinterpret_cast<short8 *>(&s.bnd[ts][4 * k]) = q[k];
                    if (te >= 0)
#pragma unroll
                        for (int k = 0; k < 4; k++) *reinterpret_cast<short8 *>(&s.bnd[te][4 * k]) = q[k];
                }
            }
            // windowed E / M of every frame overlapping this word's quad (4 words = 128 samples,
            // lanes 4Q .. 4Q+3): per sample y = w_j x (the reference's windowed frame,
            // :329-331), E += y^2, M += |y|; the quad's four partials are summed on DPP and one
            // lane stores them at part[f][Q - qa(f)].  Waves entirely past the clip skip.
#ifdef STREAM_NO_WINDOW  // diagnostic variant: the windowed frames skipped
        }
#else
            if (r * NT + wid * 64 >= nword) continue;
            const int Q = w >> 2;
            const int qnum = 128 * Q - lead - L;
            const int fa = qnum < 0 ? 0 : qnum / S + 1;  // first frame overlapping the quad
            // per frame t: chunk k (4 weights) of the word's 32 sits at wphys(m0 + 4k) = wa + 4k,
            // or wa + 4k + 4 once the chunks cross into the next 32-float block (k >= kc)
            const float *wa[R];
            int kc[R];
#pragma unroll
            for (int t = 0; t < R; t++) {
                const int j0 = 32 * w - lead - (fa + t) * S;  // window index of the word's first sample
                const int j0c = min(max(j0, -32), L);         // past the window: zero weights
                const int c = (-j0c) & 3;
                const int m0 = j0c + WPAD + c;  // multiple of 4
                kc[t] = 8 - ((m0 & 31) >> 2);
                wa[t] = &s.wtab[c][m0 + 4 * (m0 >> 5)];
            }
            float E[R][2], M[R][2];
#pragma unroll
            for (int t = 0; t < R; t++) E[t][0] = E[t][1] = M[t][0] = M[t][1] = 0.f;
            // samples outside the clip (first / last word, words past it) are zero padding
            const bool edge = w == 0 || w >= nword - 1;
            auto run = [&](auto masked_t) {
                constexpr bool MASKED = decltype(masked_t)::value;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    float x[4];
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        x[e] = ((float)q[k >> 1][4 * (k & 1) + e] - xa) - xb;
                        if (MASKED) {
                            const int u = 32 * w + 4 * k + e;
                            x[e] = (u >= lead && u < lead + n) ? x[e] : 0.f;
                        }
                    }
#pragma unroll
                    for (int t = 0; t < R; t++) {
                        const float4 wv = *reinterpret_cast<const float4 *>(wa[t] + 4 * k + (k >= kc[t] ? 4 : 0));
                        const float y0 = wv.x * x[0], y1 = wv.y * x[1], y2 = wv.z * x[2], y3 = wv.w * x[3];
                        E[t][0] = fmaf(y0, y0, E[t][0]);
                        E[t][1] = fmaf(y1, y1, E[t][1]);
                        M[t][0] = add_abs(M[t][0], y0);
                        M[t][1] = add_abs(M[t][1], y1);
                        E[t][0] = fmaf(y2, y2, E[t][0]);
                        E[t][1] = fmaf(y3, y3, E[t][1]);
                        M[t][0] = add_abs(M[t][0], y2);
                        M[t][1] = add_abs(M[t][1], y3);
                    }
                }
            };
            if (__ballot(edge))
                run(BoolT<true>());
            else
                run(BoolT<false>());
#pragma unroll
            for (int t = 0; t < R; t++) {
                const int f = fa + t;
                const float Eq = quad_sumf(E[t][0] + E[t][1]), Mq = quad_sumf(M[t][0] + M[t][1]);
                if ((lane & 3) == 0 && f < Fmax) {
                    const int us = lead + f * S;
                    const int qa = us >> 7, qb = (us + L - 1) >> 7;
                    if (Q >= qa && Q <= qb) s.part[f][Q - qa] = make_float2(Eq, Mq);
                }
            }
        }
#endif
        if (tid < 2) s.posw[nword + tid] = 0;
        __syncthreads();

        // ---- pass A: moments of the partial words at endpoint frame ends ---------------------
#ifdef STREAM_ABL  // diagnostic ablation: 1 = no frames phase, 2 = + no pass A, 3 = + no R2
        if (STREAM_ABL >= 2) continue;
#endif
        if (tid < 2 * nv) {
            int e0, e1, t1 = 0;
            unsigned long long t2 = 0;
            if (boundary_word(tid, lead, L, S, nv, e0, e1) >= 0) {
                const short8 *q = reinterpret_cast<const short8 *>(&s.bnd[tid][0]);
#pragma unroll 1
                for (int k = 0; k < 4; k++) {
                    const short8 v = q[k];
#pragma unroll
                    for (int e = 0; e < 8; e++) {
                        const int x = v[e];
                        const int ee = 8 * k + e;
                        if (ee >= e0 && ee < e1) {
                            t1 += x;
                            t2 += (unsigned)(x * x);
                        }
                    }
                }
            }
            s.pS1[tid] = t1;
            s.pS2[tid] = t2;
        }
        __syncthreads();

#ifdef STREAM_ABL
        if (STREAM_ABL >= 1) continue;
#endif
        // ---- frames: one quad per frame -> the clip's summary record -------------------------
        unsigned char *rec = p.rec + (size_t)i * rl.stride;
        if (tid == 0) {
            reinterpret_cast<double *>(rec)[0] = mq;
            reinterpret_cast<double *>(rec)[1] = Mp;
        }
        {
            const int f = tid >> 2, lq = tid & 3;
            const int u0 = lead + f * S, u1 = u0 + L;
            // endpoint frame f (:172-181): exact moments, sign changes among its L-1 pairs
            int s1 = 0, zc = 0;
            unsigned long long s2 = 0;
            if (f < nv) {
                const int wa = u0 >> 5, wb = (u1 - 1) >> 5;
                const int wi0 = (u0 & 31) ? wa + 1 : wa, wi1 = (u1 & 31) ? wb - 1 : wb;
                const int per = (wi1 - wi0 + 4) >> 2;
                const int ws = wi0 + lq * per, we = min(ws + per - 1, wi1);
                for (int w = ws; w <= we; w++) {
                    s1 += s.wS1[w];
                    s2 += s.wS2[w];
                }
                if (lq == 0) {
                    s1 += s.pS1[2 * f] + s.pS1[2 * f + 1];
                    s2 += s.pS2[2 * f] + s.pS2[2 * f + 1];
                }
                const int np_ = L - 1, pq = (np_ + 3) >> 2;
                const int x0 = u0 + min(lq * pq, np_), x1 = u0 + min((lq + 1) * pq, np_);
                zc = chg_run(s.posw, x0, x1);
            }
            s1 = dpp_quad_reduce(s1, OpAdd());
            s2 = dpp_quad_sum64(s2);
            zc = dpp_quad_reduce(zc, OpAdd());
            // windowed frame f (frame_signal + extract_frame_features): E, M from the quad
            // partials; ZCR where the window is positive (j in [j0w, j1w]) and j < n - fs,
            // transitions into the zero ends / padding included
            float E = 0.f, M = 0.f;
            int zw = 0;
            const bool fw = f < Fmax;
            const int fs = f * S;
#ifndef STREAM_NO_WINDOW
            if (fw) {
                const int qa = u0 >> 7, qb = min((u1 - 1) >> 7, nquad - 1);
                for (int qq = qa + lq; qq <= qb; qq += 4) {
                    const float2 v = s.part[f][qq - qa];
                    E += v.x;
                    M += v.y;
                }
            }
#endif
            const int ia = fs + j0w, ib = min(fs + j1w, n - 1);
            if (fw && ia < ib) zw = chg_count(s.posw, ia + lead, ib + lead, lq, 4);
            E = quad_sumf(E);
            M = quad_sumf(M);
            zw = dpp_quad_reduce(zw, OpAdd());
            if (lq == 0) {
                if (f < nv) {
                    reinterpret_cast<double *>(rec + rl.vE)[f] =
                        energy_from_moments(s2, s1, L, t0, mq - (double)t0, invM2);
                    reinterpret_cast<uint16_t *>(rec + rl.vZ)[f] = (uint16_t)zc;
                }
                if (fw) {
                    if (ia <= ib) {
                        if (j0w > 0) zw += pos_bit(s.posw, ia + lead);
                        if (ib < fs + L - 1) zw += pos_bit(s.posw, ib + lead);
                    }
                    reinterpret_cast<float *>(rec + rl.fE)[f] = E * (invMf * invMf);
                    reinterpret_cast<float *>(rec + rl.fM)[f] = M * invMf;
                    reinterpret_cast<uint16_t *>(rec + rl.fZ)[f] = (uint16_t)zw;
                }
            }
        }
        __syncthreads();  // LDS is rewritten by the next clip
    }
}

// ------------------------------------------------------------------------------------------
// decide_kernel: one wave per clip
// ------------------------------------------------------------------------------------------
struct Decision {
    int n3, n1, n6, near;
};

// the rare exact endpoint energy (numpy's pairwise float64 order over the PCM), out of line so
// its stack of partial sums does not weigh on the register allocation of the common path
__device__ __attribute__((noinline)) double exact_energy(const int16_t *clip, int lo, int L, double mq, double Mp)
{
    return np_energy_exact(clip, lo, L, mq, Mp);
}

// endpoint decisions (:186-273) from the energies / ZCRs held as e[lane + 64h], z[lane + 64h]
template <bool CERTIFY>
__device__ __forceinline__ Decision decide(const double (&e)[2], const int (&z)[2], int nv, double hi, double lo,
                                           double zr, int lane)
{
    // p90 (:198): the two order statistics around virtual index (nv - 1) * 0.9 by a bitonic sort
    // of the high halves of order-preserving keys; ties in the high half resolved by full keys
    const double vi = (double)(nv - 1) * 0.9;
    int r0, r1;
    if (vi >= (double)(nv - 1)) {
        r0 = r1 = nv - 1;
    } else {
        r0 = (int)floor(vi);
        r1 = r0 + 1;
    }
    const unsigned long long f0 = lane < nv ? dkey(e[0]) : ~0ull;
    const unsigned long long f1 = lane + 64 < nv ? dkey(e[1]) : ~0ull;
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
                const unsigned long long ev = lane_read(hh ? f1 : f0, l);
                const int lt = __popcll(__ballot(h0 == kh && f0 < ev)) + __popcll(__ballot(h1 == kh && f1 < ev));
                const int eq = __popcll(__ballot(f0 == ev)) + __popcll(__ballot(f1 == ev));
                if (rr >= lt && rr < lt + eq) res = ev;
            }
        }
        return dkey_value(res);
    };
    const double pa = full_at(r0), pb = full_at(r1);
    const double g = (vi >= (double)(nv - 1)) ? vi + 1.0 : vi - floor(vi);
    const double p90 = np_lerp(pa, pb, g);
    // noise estimates (:188-195, :239-245)
    auto E_at = [&](int q) { return lane_read(q < 64 ? e[0] : e[1], q & 63); };
    auto Z_at = [&](int q) { return lane_read(q < 64 ? z[0] : z[1], q & 63); };
    const int nfr = min(5, nv / 10);
    double noise_e, noise_z;
    if (nfr > 0) {
        long long zs = 0;
        for (int q = 0; q < nfr; q++) zs += Z_at(q) + Z_at(nv - nfr + q);
        auto cat = [&](int q) { return q < nfr ? E_at(q) : E_at(nv - 2 * nfr + q); };
        noise_e = np_small_sum(cat, 2 * nfr) / (double)(2 * nfr);
        noise_z = (double)zs / (double)(2 * nfr);
    } else {
        const bool i0 = lane < nv, i1 = lane + 64 < nv;
        noise_e = wave_mind(fmin(i0 ? e[0] : INFINITY, i1 ? e[1] : INFINITY));
        noise_z = (double)wave_min(min(i0 ? z[0] : 0x7fffffff, i1 ? z[1] : 0x7fffffff));
    }
    double t1, t2, tz;
    {
#pragma clang fp contract(off)
        t1 = p90 * hi;                        // :202
        t2 = noise_e + (p90 - noise_e) * lo;  // :217
        tz = noise_z * zr;                    // :247
    }
    auto near = [&](double v, double t) {
        const double d = fabs(v - t);
        return d <= 1e-11 * fmax(fabs(v), fabs(t)) && !(v == 0.0 && t == 0.0);
    };
    BitsK<2> hiE, loE, loZ, nr1, nr2;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int q = 64 * k + lane;
        const bool in = q < nv;
        hiE.w[k] = __ballot(in && e[k] > t1);
        loE.w[k] = __ballot(in && e[k] <= t2);
        loZ.w[k] = __ballot(in && (double)z[k] <= tz);
        nr1.w[k] = CERTIFY ? __ballot(in && near(e[k], t1)) : 0ull;
        nr2.w[k] = CERTIFY ? __ballot(in && near(e[k], t2)) : 0ull;
    }
    Decision d{-1, 0, nv - 1, 0};
    d.n3 = bits_first_ge(hiE, 0);  // :205-213
    const int n4 = bits_last_lt(hiE, nv);
    if (CERTIFY) {  // the decisions of N3 / N4 depend on frames <= N3 and >= N4
        if (d.n3 < 0) d.near |= bits_any_in(nr1, 0, nv);
        else d.near |= bits_any_in(nr1, 0, d.n3 + 1) || bits_any_in(nr1, n4, nv);
    }
    if (d.n3 >= 0) {
        const int b2 = bits_last_lt(loE, d.n3);  // :219-226
        const int n2 = b2 >= 0 ? b2 + 1 : 0;
        const int b5 = bits_first_ge(loE, n4 + 1);  // :229-235
        const int n5 = b5 >= 0 ? b5 - 1 : nv - 1;
        if (CERTIFY) d.near |= bits_any_in(nr2, max(n2 - 1, 0), d.n3) || bits_any_in(nr2, n4 + 1, min(n5 + 2, nv));
        const int b1 = bits_last_lt(loZ, n2);  // :249-256
        d.n1 = b1 >= 0 ? b1 + 1 : 0;
        const int b6 = bits_first_ge(loZ, n5 + 1);  // :258-265
        d.n6 = b6 >= 0 ? b6 - 1 : nv - 1;
    }
    return d;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void decide_kernel(DecideParams p)
{
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= p.B) return;
    const int64_t o0 = p.offsets[i], nn = p.offsets[i + 1] - o0;
    if (nn <= 0 || nn > p.ncap) {  // np.max of an empty array raises (:72) / past the plan
        if (lane < 15) p.feat[(size_t)i * 15 + lane] = __builtin_nanf("");
        if (lane == 0) {
            p.status[i] = nn <= 0 ? DSP_CLIP_EMPTY : DSP_CLIP_TOO_LONG;
            p.start_end[2 * i] = 0;
            p.start_end[2 * i + 1] = 0;
            p.n_frames[i] = 0;
        }
        return;
    }
    const int n = (int)nn, L = p.L, S = p.S;
    const RecLayout rl = p.rl;
    const unsigned char *rec = p.rec + (size_t)i * rl.stride;
    const double mq = reinterpret_cast<const double *>(rec)[0];
    const double Mp = reinterpret_cast<const double *>(rec)[1];
    const double *vE = reinterpret_cast<const double *>(rec + rl.vE);
    const uint16_t *vZ = reinterpret_cast<const uint16_t *>(rec + rl.vZ);
    const float *fE = reinterpret_cast<const float *>(rec + rl.fE);
    const float *fM = reinterpret_cast<const float *>(rec + rl.fM);
    const uint16_t *fZ = reinterpret_cast<const uint16_t *>(rec + rl.fZ);
    const int nv = (p.do_vad && n >= L) ? (n - L) / S + 1 : 0;
    const int Fmax = n <= L ? 1 : (n - L + S - 1) / S + 1;

    int st = 0, en = n, f0 = 0, F = Fmax, flags = 0;
    if (nv > 0) {
        double e[2];
        int z[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int q = lane + 64 * h;
            e[h] = q < nv ? vE[q] : 0.0;
            z[h] = q < nv ? (int)vZ[q] : 0;
        }
        Decision d = decide<true>(e, z, nv, p.hi, p.lo, p.zr, lane);
        if (d.near && Mp > 0.0) {
            // near tie: the endpoint energies in numpy's exact float64 order from the PCM
            const int16_t *clip = p.pcm + o0;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int q = lane + 64 * h;
                if (q < nv) e[h] = exact_energy(clip, q * S, L, mq, Mp);
            }
            d = decide<false>(e, z, nv, p.hi, p.lo, p.zr, lane);
            flags = DSP_CLIP_FLAG_VAD_EXACT;
        }
        if (d.n3 >= 0) {
            st = d.n1 * S;              // :272
            en = min(d.n6 * S + L, n);  // :273
            f0 = d.n1;
            F = d.n6 - d.n1 + 1;
        }
        if (p.vad_energy)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int q = lane + 64 * h;
                if (q < nv && q < p.ld_vad) {
                    p.vad_energy[(size_t)i * p.ld_vad + q] = e[h];
                    p.vad_zcr[(size_t)i * p.ld_vad + q] = z[h];
                }
            }
    }

    // compute_statistics x 3 (fe.py:46-62) over crop frames f0 .. f0 + F - 1
    float *featb = p.feat + (size_t)i * 15;
    const int r0 = (F - 1) / 2, r1 = F / 2;
    const bool in0 = lane < F, in1 = lane + 64 < F;
#pragma unroll 1
    for (int q = 0; q < 3; q++) {
        auto get = [&](int j) -> float { return q == 0 ? fE[f0 + j] : q == 1 ? fM[f0 + j] : (float)fZ[f0 + j]; };
        const float x0 = in0 ? get(lane) : 0.f, x1 = in1 ? get(lane + 64) : 0.f;
        float v0, v1;
        if (F <= 64) {  // np.median: middle order statistic(s) by an in-wave bitonic sort
            unsigned b[1] = {in0 ? fkey(x0) : ~0u};
            wave_bitonic<1>(b, lane);
            v0 = fkey_value(sorted_at<1>(b, r0));
            v1 = fkey_value(sorted_at<1>(b, r1));
        } else {
            unsigned a[2] = {in0 ? fkey(x0) : ~0u, in1 ? fkey(x1) : ~0u};
            wave_bitonic<2>(a, lane);
            v0 = fkey_value(sorted_at<2>(a, r0));
            v1 = fkey_value(sorted_at<2>(a, r1));
        }
        double med;
        {
#pragma clang fp contract(off)
            med = (F & 1) ? (double)v1 : ((double)v0 + (double)v1) / 2.0;
        }
        // mean, population std (fp64 sums), max, min
        const double sum = wave_sum((in0 ? (double)x0 : 0.0) + (in1 ? (double)x1 : 0.0));
        const float mx = wave_reduce(fmaxf(in0 ? x0 : -INFINITY, in1 ? x1 : -INFINITY), OpMax());
        const float mn = wave_reduce(fminf(in0 ? x0 : INFINITY, in1 ? x1 : INFINITY), OpMin());
        const double mean = sum / (double)F;
        const double d0 = in0 ? (double)x0 - mean : 0.0, d1 = in1 ? (double)x1 - mean : 0.0;
        const double qq = wave_sum(fma(d0, d0, d1 * d1));
        if (lane < 5) {
            const double o = lane == 0 ? mean : lane == 1 ? sqrt(qq / (double)F) : lane == 2 ? (double)mx
                             : lane == 3 ? (double)mn : med;
            featb[5 * q + lane] = (float)o;
        }
    }
    if (p.seq)
        for (int g = lane; g < F && g < p.ld_seq; g += 64) {
            float *o = p.seq + ((size_t)i * p.ld_seq + g) * 3;
            o[0] = fE[f0 + g];
            o[1] = fM[f0 + g];
            o[2] = (float)fZ[f0 + g];
        }
    if (lane == 0) {
        p.start_end[2 * i] = st;
        p.start_end[2 * i + 1] = en;
        p.n_frames[i] = F;
        p.status[i] = DSP_CLIP_OK | flags;
    }
}

}  // namespace st
}  // namespace dsp

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// frames one 128-sample quad can overlap (frame_kernel's template parameter)
static int stream_quad_frames(int L, int S) { return (127 + L) / S + 1; }

bool dsp_stream_fits(int64_t max_len, int L, int S)
{
    if (max_len < 1 || L < 64 || S < 32) return false;
    if (stream_quad_frames(L, S) > 4) return false;
    if ((max_len + 7 + 31) / 32 > dsp::st::NWORD) return false;
    if (L + 2 * STREAM_WPAD + 4 > STREAM_WROWF) return false;
    if ((L + 126) / 128 + 1 > STREAM_PQ) return false;
    const int64_t nv = max_len >= L ? (max_len - L) / S + 1 : 0;
    const int64_t F = max_len <= L ? 1 : (max_len - L + S - 1) / S + 1;
    return nv <= STREAM_FCAP && F <= STREAM_FCAP;
}

RecLayout dsp_stream_layout(int64_t max_len, int L, int S)
{
    const int nv = max_len >= L ? (int)((max_len - L) / S + 1) : 0;
    const int F = max_len <= L ? 1 : (int)((max_len - L + S - 1) / S + 1);
    const int nvc = nv > 0 ? nv : 1;
    RecLayout r;
    int o = 16;  // mq, Mp
    r.vE = o;
    o += 8 * nvc;
    r.fE = o;
    o += 4 * F;
    r.fM = o;
    o += 4 * F;
    r.vZ = o;
    o += 2 * nvc;
    r.fZ = o;
    o += 2 * F;
    r.stride = (o + 127) & ~127;
    return r;
}

size_t dsp_stream_lds_bytes() { return sizeof(dsp::st::Lds); }
static_assert(sizeof(dsp::st::Lds) <= EXTRACT_LDS_SHARED, "two frame_kernel workgroups per CU");
static_assert(EXTRACT_LDS_LIMIT / sizeof(dsp::st::Lds) >= 4 * STREAM_WPE / dsp::st::NWAVE || STREAM_WPE == 4,
              "LDS holds the workgroups the register budget allows");

int dsp_stream_launch(const int16_t *pcm, const int64_t *offsets, int B, int64_t max_len, int L, int S,
                      const double *window, int do_vad, double hi, double lo, double zr, float *feat,
                      int32_t *start_end, int32_t *n_frames, int32_t *status, double *vad_energy,
                      int32_t *vad_zcr, int ld_vad, float *seq, int ld_seq, void *workspace,
                      size_t workspace_bytes, int num_cus, hipStream_t stream)
{
    using namespace dsp::st;
    const RecLayout rl = dsp_stream_layout(max_len, L, S);
    const int64_t chunk = (int64_t)(workspace_bytes / (size_t)rl.stride);
    if (chunk < 1) return DSP_ERR_WORKSPACE;
    const size_t lds = sizeof(Lds);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)frame_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void *)frame_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void *)frame_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    // resident workgroups per CU: LDS and the register budget (STREAM_WPE waves per SIMD)
    const int per_cu = std::max(1, std::min((int)(EXTRACT_LDS_LIMIT / lds), 4 * STREAM_WPE / NWAVE));
    const int slots = per_cu * num_cus;
    for (int64_t b0 = 0; b0 < B; b0 += chunk) {
        const int nb = (int)std::min<int64_t>(chunk, B - b0);
        FrameParams fp;
        fp.pcm = pcm;
        fp.offsets = offsets + b0;
        fp.B = nb;
        fp.ncap = (int)max_len;
        fp.L = L;
        fp.S = S;
        fp.window = window;
        fp.do_vad = do_vad;
        fp.rec = (unsigned char *)workspace;
        fp.rl = rl;
        const int grid = nb < slots ? nb : slots;
        switch (stream_quad_frames(L, S)) {
        case 2: hipLaunchKernelGGL(frame_kernel<2>, dim3(grid), dim3(NT), lds, stream, fp); break;
        case 3: hipLaunchKernelGGL(frame_kernel<3>, dim3(grid), dim3(NT), lds, stream, fp); break;
        default: hipLaunchKernelGGL(frame_kernel<4>, dim3(grid), dim3(NT), lds, stream, fp); break;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return DSP_ERR_HIP + (int)e;
        DecideParams dp;
        dp.pcm = pcm;
        dp.offsets = offsets + b0;
        dp.B = nb;
        dp.ncap = (int)max_len;
        dp.L = L;
        dp.S = S;
        dp.do_vad = do_vad;
        dp.hi = hi;
        dp.lo = lo;
        dp.zr = zr;
        dp.rec = (const unsigned char *)workspace;
        dp.rl = rl;
        dp.feat = feat + 15 * b0;
        dp.start_end = start_end + 2 * b0;
        dp.n_frames = n_frames + b0;
        dp.status = status + b0;
        dp.vad_energy = vad_energy ? vad_energy + b0 * ld_vad : nullptr;
        dp.vad_zcr = vad_zcr ? vad_zcr + b0 * ld_vad : nullptr;
        dp.ld_vad = ld_vad;
        dp.seq = seq ? seq + b0 * ld_seq * 3 : nullptr;
        dp.ld_seq = ld_seq;
        hipLaunchKernelGGL(decide_kernel, dim3((nb + 3) / 4), dim3(256), 0, stream, dp);
        e = hipGetLastError();
        if (e != hipSuccess) return DSP_ERR_HIP + (int)e;
    }
    return DSP_OK;
}
