// extract.hip -- fused per-clip feature extraction for gfx950 (CDNA4).
//
// Persistent workgroups (512 threads, three per CU on the compile-time layout, two on the generic
// one) walk the batch, one clip at a time.  The clip is read from HBM once, straight into
// registers (each thread holds EXTRACT_RREG 32-sample words):
//   R1  registers: integer sum / min / max + exact per-word moments (sum k, sum k^2) -> LDS
//   R2  registers: positive-sample bits per word -> LDS (the ZCR of any range is a popcount)
//   R3  endpoint detection from the per-word summaries (+ the two partial words of each frame;
//       sign changes from per-segment prefixes), p90 by one wave's repeated maxima, double-
//       threshold scan
//   R4  windowed frames of the crop (clip-relative vectors re-read from L2, window from LDS)
//   R5  15-d statistics
// LDS holds only summaries, the window table and the per-frame arrays (52 192 B in the
// compile-time layout), so the other workgroups on the same CU compute while one waits for HBM.
// Algorithmic traffic: 2 B/sample in + 76 B/clip out.
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
//   * endpoint energies: exact integer moments per frame (sum k, sum k^2) combined with mq in
//     double-double -> relative error ~1e-16; every threshold decision is certified against a
//     1e-11 margin and, on a near tie, the clip is redone with the energies in numpy's exact
//     float64 order (pairwise_sum), so start/end are always the reference's.
//   * windowed E/M: fp32 on VALU (tolerance 1e-5 rel., measured ~2e-7) in the canonical
//     clip-coordinate order of dsp_device.h (position independent, = dsp_extract_general);
//     statistics in fp64.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "dsp_audiorec.h"
#include "extract_layout.h"
#include "dsp_device.h"

#ifndef DSP_ABL  // the phase-ablation instrument (tools/ablate_build.sh, diagnostic builds only;
#define DSP_ABL 0 // outputs are wrong): skip 1 = R4 frames, 2 = R5 jobs, 4 = R2 sign bits,
#endif            // 8 = VAD pass-A partial moments, 64 = p90 selection -- the per-phase VALU budget of
                  // DESIGN.md §8

namespace dsp {

static constexpr int NT = EXTRACT_THREADS;
static constexpr int NWAVE = NT / 64;
static constexpr int RREG = EXTRACT_RREG;  // words per thread in registers
static constexpr int NRV = 4 * RREG;       // 16-B vectors per thread in registers

#ifdef DSP_STAMPS
// diagnostic build only (make stamps): per-phase shader-clock stamps of each clip.  The buffer
// pointer is a kernel argument (SGPRs), so a stamp never waits on a memory load.
#define STAMP(clip, k)                                                                           \
    do {                                                                                         \
        if (threadIdx.x == 0 && p.stamps) p.stamps[(size_t)(clip) * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// per workgroup (row blockIdx.x, slots 16..): real-time and shader-clock stamps (WG_STAMP, at
// entry and exit) and shader-clock stamps inside the prologue (WG_CK)
#define WG_STAMP(k)                                                                          \
    do {                                                                                     \
        if (threadIdx.x == 0 && p.stamps) {                                                  \
            p.stamps[(size_t)blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memrealtime();      \
            p.stamps[(size_t)blockIdx.x * 32 + (k) + 1] = __builtin_amdgcn_s_memtime();      \
        }                                                                                    \
    } while (0)
#define WG_CK(k)                                                                             \
    do {                                                                                     \
        if (threadIdx.x == 0 && p.stamps) p.stamps[(size_t)blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define WG_STAMP(k) \
    do {            \
    } while (0)
#define WG_CK(k) \
    do {         \
    } while (0)
#define STAMP(clip, k) \
    do {               \
    } while (0)
#endif

#ifdef DSP_MARKS  // diagnostic assembly listings only (tools/phase_insts.py): region labels
#define MARK(name) asm volatile(";@@ " #name)
#else
#define MARK(name) \
    do {           \
    } while (0)
#endif

// The kernels' only argument, a plain aggregate passed by value.
struct ExtractParams {
    const int16_t *pcm;
    const int64_t *offsets;
    int B, ncap, L, S;
    const double *window;
    int do_vad;
    double hi, lo, zr;
    float *feat;
    int32_t *start_end, *n_frames, *status;
    int ostride;  // 0: feat [B,15], start_end [B,2], n_frames / status [B]; > 0: row b of each at b * ostride
    double *vad_energy;
    int32_t *vad_zcr;
    int ld_vad;
    float *seq;
    int ld_seq;
    unsigned long long *stamps;  // diagnostic build only (else null)
    unsigned *queue;             // caller's clip-queue scratch (NULL: static split), zero at launch;
                                 // the last workgroup out zeroes it again
    int qchunk;                  // clips per queue chunk (host: 4, 2 for short batches, 0: static split)
    ExtractCarve cv;             // LDS layout, computed on the host
};

// the clip's output rows: per-array [B,15] / [B,2] / [B] / [B], or rows of p.ostride 4-byte words
// (ABI 6: one packed [B, DSP_OUT_ROW_WORDS] buffer with the four arrays as column ranges)
__device__ __forceinline__ float *out_feat(const ExtractParams &p, int i) { return p.feat + (size_t)i * (p.ostride ? p.ostride : 15); }
__device__ __forceinline__ int32_t *out_se(const ExtractParams &p, int i) { return p.start_end + (size_t)i * (p.ostride ? p.ostride : 2); }
__device__ __forceinline__ int32_t *out_nf(const ExtractParams &p, int i) { return p.n_frames + (size_t)i * (p.ostride ? p.ostride : 1); }
__device__ __forceinline__ int32_t *out_st(const ExtractParams &p, int i) { return p.status + (size_t)i * (p.ostride ? p.ostride : 1); }

static_assert(__is_standard_layout(ExtractParams) && __is_trivially_copyable(ExtractParams),
              "ExtractParams is a plain kernel argument block");
static_assert(sizeof(ExtractParams) <= 1024, "kernel argument block");

// ------------------------------------------------------------------------------------------
struct ClipStatsRaw {
    double mq, Mp, invM2;
    float invMf;
    int tpos, t0, nv, kneg;
};
struct Shared {
    long long red_k[NWAVE];
    int red_a[NWAVE], red_b[NWAVE];
    double pa, pb;            // the two order statistics of the VAD energies around p90
    ClipStatsRaw cs;          // the clip statistics, computed by wave 0
    double noise_e, noise_z;  // VAD noise estimates (:189-195, :239-245)
    double oslo[3], oshi[3];  // order statistics (F-1)/2 and F/2 of E, M, ZCR (medians)
    int n3, n1, n6, exact, j0, j1, next;
    int qnext, qend, qcursor, qrange;  // clip queue (thread 0): the current chunk's next clip and end;
                                       // static split cursor; ranges used up
    int cdir, cy;                      // the pending claim (queue_begin / queue_end)
    unsigned smask;                    // staged output slots (ost) ...
    int schunk;                        // ... of this chunk
    int sclear;                        // the staged slots were flushed: thread 0 clears smask after
                                       // the next barrier (flush_outputs reads it in every thread)
    long long noff[2];                 // offsets[noff_for], offsets[noff_for + 1]: the next clip's,
    int noff_for;                      // loaded during R5 (FAST; -1: none)
};
static_assert(sizeof(Shared) <= EXTRACT_SHARED_BYTES, "grow EXTRACT_SHARED_BYTES");
static_assert((EXTRACT_OSTAGE & (EXTRACT_OSTAGE - 1)) == 0 && EXTRACT_OSTAGE <= 32, "chunk of 2^k <= 32 clips");

struct ClipRef {
    int64_t base;  // 8-aligned first sample index of the clip's vectors
    int lead, n, nvec, nword;
    bool ok;
};

__device__ __forceinline__ ClipRef clip_ref_at(const ExtractParams &p, int64_t o0, int64_t o1)
{
    ClipRef c;
    const int64_t nn = o1 - o0;
    c.ok = nn > 0 && nn <= p.ncap;
    c.n = c.ok ? (int)nn : 0;
    c.base = o0 & ~(int64_t)7;
    c.lead = (int)(o0 - c.base);
    c.nvec = c.ok ? (c.lead + c.n + 7) >> 3 : 0;  // 0: loads of the clip read zeros
    c.nword = (c.lead + c.n + 31) >> 5;
    return c;
}
__device__ __forceinline__ ClipRef clip_ref(const ExtractParams &p, int i)
{
    return clip_ref_at(p, p.offsets[i], p.offsets[i + 1]);
}
__device__ __forceinline__ ClipRef clip_none()
{
    ClipRef c;
    c.base = 0;
    c.lead = c.n = c.nvec = c.nword = 0;
    c.ok = false;
    return c;
}

struct Ctx {
    Shared *sh;
    const float *wtab;  // EXTRACT_WROW(L) floats per shifted copy r = 0..3 (extract_layout.h)
    uint32_t *posw;      // bit u of the buffer: sample u is real and positive after preprocess
    unsigned long long *wS2;
    int *wS1;
    double *vE;
    int32_t *vZ;
    float *fE, *fM;
    int32_t *fZ;
    uint16_t *zw;  // FAST: sign changes before word w within its 64-word segment (zseg_word)
    int *ztot;     // FAST: sign changes of each 64-word segment, its last boundary left out
    int *rank;  // rank scratch: nvcap or 3 * fcap ints
    int *pS1;   // partial-word moments at the two ends of each VAD frame (2 * nvcap)
    unsigned long long *pS2;
    int32_t *orow;   // staged output rows of the clips of one chunk, slot = clip mod EXTRACT_OSTAGE:
                     // [slot][19] = feat[15] (f32 bits), start, end, n_frames, status
    int64_t total;
    int stamp_clip;  // clip index for the diagnostic stamps
};

// 16-B vectors of the clip buffer, read through a buffer descriptor spanning the clip's vectors:
// a vector index past the clip reads zeros (hardware range check), so no address
// clamping, and the four vectors of a word share one offset register (immediate offsets).  The
// clip's last vector may reach up to 15 bytes past offsets[B]; pcm is 16-B aligned, so such a
// vector never crosses a page.  Bytes outside a clip are masked by every consumer ([lead, lead + n)
// ranges, zero window weights), so no element-wise patching is needed.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t clip_rsrc(const ExtractParams &p, const ClipRef &c)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t *>(p.pcm + c.base), 0, c.nvec * 16, 0x00020000);
}
__device__ __forceinline__ short8 load_vec(const ExtractParams &p, const ClipRef &c, int v)
{
    return __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(clip_rsrc(p, c), 16 * v, 0, 0));
}
// the clip's own 8-sample vector v (clip samples 8v .. 8v + 7): 2-byte aligned when lead is odd
__device__ __forceinline__ short8 load_cvec(const ExtractParams &p, const ClipRef &c, int v)
{
    return __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(clip_rsrc(p, c), 2 * c.lead + 16 * v, 0, 0));
}
__device__ __forceinline__ void issue_word(short8 *q, const ExtractParams &p, const ClipRef &c, int w)
{
    const __amdgpu_buffer_rsrc_t rs = clip_rsrc(p, c);
#pragma unroll
    for (int k = 0; k < 4; k++)
        q[k] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, 64 * w + 16 * k, 0, 0));
}

// the clip's first RREG words into registers (word r * NT + tid -> regs[4r .. 4r+3]): one VGPR
// offset (the thread's word) for all of them, the row in the scalar offset and the vector in the
// immediate, so no vector instruction runs between the loads (a VGPR rewritten between them made
// the compiler's vmcnt bookkeeping wait for the first loads to land)
__device__ __forceinline__ void issue_clip(short8 (&regs)[NRV], const ExtractParams &p, const ClipRef &c,
                                           int tid = (int)threadIdx.x, int r0 = 0, int r1 = RREG)
{
    const __amdgpu_buffer_rsrc_t rs = clip_rsrc(p, c);
    const int voff = 64 * tid;
#pragma unroll
    for (int r = r0; r < r1; r++)
#pragma unroll
        for (int k = 0; k < 4; k++)
            regs[4 * r + k] = __builtin_bit_cast(
                short8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16 * k, 64 * NT * r, 0));
}
// the thread index, opaque to the optimiser where it is taken: index arithmetic that depends
// only on it is then recomputed there instead of being hoisted out of the persistent loop and kept
// live (spilled) across it.  The FAST clip body takes it only in a cold path: taken once per clip
// for the whole body it cost 9% in round 4's kernel (3.74 against 3.43 ms at 100 000 clips; DESIGN.md
// section 9, the raw record was not kept).
__device__ __forceinline__ int opaque_tid()
{
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// VAD noise estimates (src/audio_processing.py:188-195, :239-245) by one wave into sh->noise_e /
// sh->noise_z, computed while wave 0 selects the p90 order statistics
__device__ __forceinline__ void vad_noise(const Ctx &c, int nv, int lane)
{
    const double *vE = c.vE;
    const int32_t *vZ = c.vZ;
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
    if (lane == 0) {
        c.sh->noise_e = noise_e;
        c.sh->noise_z = noise_z;
    }
}

// Double-threshold endpoint scan (src/audio_processing.py:186-273) by wave 0 on vE/vZ with the
// p90 order statistics in sh->pa / sh->pb.  Writes sh->n3 (-1: no high-energy frame), n1, n6;
// returns the near-tie flag.
template <bool CERTIFY, bool FAST>
__device__ __forceinline__ int vad_scan(const ExtractParams &p, const Ctx &c, int nv, int lane)
{
    const double *vE = c.vE;
    const int32_t *vZ = c.vZ;
    Shared *sh = c.sh;
    const double noise_e = sh->noise_e, noise_z = sh->noise_z;  // vad_noise, another wave
    // np.percentile(E, 90) (:198): lerp of the two order statistics found by the workgroup
    const double vi = (double)(nv - 1) * 0.9;
    const double g = (vi >= (double)(nv - 1)) ? vi + 1.0 : vi - floor(vi);
    const double p90 = np_lerp(sh->pa, sh->pb, g);
    double t1, t2, tz;
    const ExtractParams &q = p;
    {
#pragma clang fp contract(off)
        t1 = p90 * q.hi;                        // :202
        t2 = noise_e + (p90 - noise_e) * q.lo;  // :217
        tz = noise_z * q.zr;                    // :247
    }
    STAMP(c.stamp_clip, 10);
    auto near = [&](double e, double t) {
        const double d = fabs(e - t);
        return d <= 1e-11 * fmax(fabs(e), fabs(t)) && !(e == 0.0 && t == 0.0);
    };
    int flag = 0, n3 = -1, n1 = 0, n6 = nv - 1;
    auto short_scan = [&](auto kc_t) {
        constexpr int KC = decltype(kc_t)::value;
        BitsK<KC> hiE, loE, loZ, nr1, nr2;
#pragma unroll
        for (int k = 0; k < KC; k++) {
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
    };
    if (FAST || nv <= 128) {
        short_scan(IntT<2>());
    } else if (nv <= 256) {
        short_scan(IntT<4>());
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
    STAMP(c.stamp_clip, 11);
    return flag;
}

// Ranks (ties broken by index) of nseq sequences of n elements, element (q, i) = get(q, i).  Wave w
// compares every element with its chunk of the other elements; the partial counts are combined
// with integer LDS atomics (exact, order-free).  rk[nseq * n] must be zeroed before the barrier
// that precedes this call; the ranks are complete after the next barrier.
template <typename Get>
__device__ __forceinline__ void rank_partial(Get get, int nseq, int n, int *rk, int wid, int lane)
{
    const int per = (n + NWAVE - 1) / NWAVE;
    const int jlo = wid * per, jhi = min(n, jlo + per);
    if (jlo >= jhi) return;
    for (int q = 0; q < nseq; q++)
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            const auto e = get(q, i < n ? i : 0);
            int r = 0;
#pragma unroll 4
            for (int j = jlo; j < jhi; j++) {
                const auto o = get(q, j);
                r += (o < e) || (o == e && j < i);
            }
            if (i < n && r) atomicAdd(&rk[q * n + i], r);
        }
}


// Order statistics r0 / r1 (ranks with ties broken by index) of v[0..n), n <= 256: every wave
// holds the whole sequence in registers (lane + 64k), wave w ranks elements w, w + NWAVE, ...
// with one ballot per chunk.  Lane 0 of the wave that finds them stores them.
template <typename T, typename Get>
__device__ __forceinline__ void ballot_select(Get get, int n, int r0, int r1, double *o0, double *o1,
                                              int wid, int lane)
{
    T x[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int j = lane + 64 * k;
        x[k] = j < n ? get(j) : (T)0;
    }
    const int kc = (n + 63) >> 6;
    for (int i = wid; i < n; i += NWAVE) {
        const int ki = i >> 6;
        const T e = lane_read(ki == 0 ? x[0] : ki == 1 ? x[1] : ki == 2 ? x[2] : x[3], i & 63);
        int r = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (k < kc) {
                const int j = lane + 64 * k;
                r += __popcll(__ballot(j < n && (x[k] < e || (x[k] == e && j < i))));
            }
        }
        if (lane == 0) {
            if (r == r0) *o0 = (double)e;
            if (r == r1) *o1 = (double)e;
        }
    }
}

// Endpoint frame ends (pass A): boundary t = 2f (start) / 2f + 1 (end) of VAD frame f lies inside
// a buffer word that the frame only partly covers; returns that word (or -1: the boundary is
// word aligned, or t >= 2 nv) and the covered element range [e0, e1) of it.
__device__ __forceinline__ int vad_partial_word(const ClipRef &cur, int L, int S, int nv, int t, int &e0, int &e1)
{
    e0 = e1 = 0;
    if (t >= 2 * nv) return -1;
    const int f = t >> 1;
    const bool end = t & 1;
    const int u0 = cur.lead + f * S, u1 = u0 + L;
    const int wa = u0 >> 5, wb = (u1 - 1) >> 5;
    if (!end && (u0 & 31)) {
        e0 = u0 & 31;
        e1 = min(32, u1 - 32 * wa);
        return wa;
    }
    if (end && (u1 & 31) && (wb != wa || !(u0 & 31))) {
        e0 = max(0, u0 - 32 * wb);
        e1 = u1 & 31;
        return wb;
    }
    return -1;
}
// exact moments (sum k, sum k^2) of elements [e0, e1) of one 32-sample word, branch-free: the
// range as a bit mask M; pair p's two bits become a 16-bit-lane mask (v_bfe_i32 of each bit,
// merged by v_bfi), and the pair's masked samples go through one v_dot2 each for sum k and sum k^2
// (a rolled loop with a branch per element cost ~1.9k instructions per clip, a third of them scalar)
__device__ __forceinline__ void partial_moments(const short8 (&q)[4], int e0, int e1, int &t1, unsigned long long &t2)
{
    const uint32_t hi = e1 >= 32 ? ~0u : (1u << e1) - 1u;
    const uint32_t M = hi & ~((1u << e0) - 1u);  // e0 < 32
    const short2v ones = {1, 1};
    int s1 = 0;
    unsigned long long s2 = 0;
    const short8 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];  // value selects (see r1_word)
#pragma unroll 1
    for (int k = 0; k < 4; k++) {
        const short8 v = k == 0 ? q0 : k == 1 ? q1 : k == 2 ? q2 : q3;
        const uint32_t Mk = M >> (8 * k);
#pragma unroll
        for (int h = 0; h < 4; h++) {  // pair 4k + h: elements 8k + 2h, 8k + 2h + 1
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_sbfe((int)Mk, 2 * h, 1);
            const uint32_t b1 = (uint32_t)__builtin_amdgcn_sbfe((int)Mk, 2 * h + 1, 1);
            const uint32_t m = (b0 & 0x0000FFFFu) | (b1 & 0xFFFF0000u);
            const short2v dm = __builtin_bit_cast(short2v, __builtin_bit_cast(uint32_t, half_pair(v, h)) & m);
            s1 = __builtin_amdgcn_sdot2(dm, ones, s1, false);
            s2 += (unsigned)sq2(dm);
        }
    }
    t1 += s1;
    t2 += s2;
}

// FAST pass A: partial_moments unrolled over the word's four vectors (no value selects) and with the
// squares of two pairs chained in one 32-bit v_dot2 (as R1's interior words: 4 x 32768^2 = 2^32
// wraps only when all four samples are -32768, so a clip holding a -32768 sample (kneg, clip-
// uniform) adds every pair's squares to the 64-bit sum on its own)
__device__ __forceinline__ void partial_moments_fast(const short8 (&q)[4], int e0, int e1, bool kneg, int &t1,
                                                     unsigned long long &t2)
{
    const uint32_t hi = e1 >= 32 ? ~0u : (1u << e1) - 1u;
    const uint32_t M = hi & ~((1u << e0) - 1u);  // e0 < 32
    const short2v ones = {1, 1};
    int s1 = 0;
    unsigned long long s2 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t Mk = M >> (8 * k);
        short2v dm[4];
#pragma unroll
        for (int h = 0; h < 4; h++) {  // pair 4k + h: elements 8k + 2h, 8k + 2h + 1
            const uint32_t b0 = (uint32_t)__builtin_amdgcn_sbfe((int)Mk, 2 * h, 1);
            const uint32_t b1 = (uint32_t)__builtin_amdgcn_sbfe((int)Mk, 2 * h + 1, 1);
            const uint32_t m = (b0 & 0x0000FFFFu) | (b1 & 0xFFFF0000u);
            dm[h] = __builtin_bit_cast(short2v, __builtin_bit_cast(uint32_t, half_pair(q[k], h)) & m);
            s1 = __builtin_amdgcn_sdot2(dm[h], ones, s1, false);
        }
        if (kneg) {
#pragma unroll
            for (int h = 0; h < 4; h++) s2 += (unsigned)sq2(dm[h]);
        } else {
            s2 += (unsigned)sq2acc(dm[1], sq2(dm[0]));
            s2 += (unsigned)sq2acc(dm[3], sq2(dm[2]));
        }
    }
    t1 += s1;
    t2 += s2;
}

// values every lane holds alike (read from LDS, say): pinned to scalar registers
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

__device__ __forceinline__ uint64_t uni_u64(uint64_t v)
{
    const unsigned lo = __builtin_amdgcn_readfirstlane((int)v), hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// R1 of one 32-sample buffer word w of a clip (lead, n, nword): exact moments (sum k, sum k^2) to
// wS1[w] / wS2[w]; the thread's running sum K, min and max (packed int16 min / max for the
// interior words, whose 32 samples are all the clip's)
struct R1Acc {
    int K, kmin, kmax;
    short2v pmin, pmax;
};
__device__ __forceinline__ R1Acc r1_acc_init()
{
    R1Acc a;
    a.K = 0;
    a.kmin = 0x7fffffff;
    a.kmax = -0x7fffffff - 1;
    a.pmin = (short2v){32767, 32767};
    a.pmax = (short2v){-32768, -32768};
    return a;
}
__device__ __forceinline__ void r1_word(const short8 *q, int w, int nword, int lead, int n, R1Acc &a, int *wS1,
                                        unsigned long long *wS2)
{
    int s1 = 0;
    unsigned long long s2 = 0;
    if (w > 0 && w < nword - 1) {  // all 32 samples are the clip's
        const short2v ones = {1, 1};
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const short2v d = half_pair(q[k], h);
                a.pmin = __builtin_elementwise_min(a.pmin, d);
                a.pmax = __builtin_elementwise_max(a.pmax, d);
                s1 = __builtin_amdgcn_sdot2(d, ones, s1, false);
                s2 += (unsigned)sq2(d);  // <= 2^31: unsigned
            }
    } else {  // first / last word of the clip: real samples only
        // select among values (v_cndmask), never among pointers into the caller's register array:
        // a pointer select in a rolled loop moves the whole array to scratch
        const short8 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
#pragma unroll 1
        for (int k = 0; k < 4; k++) {
            const short8 v = k == 0 ? q0 : k == 1 ? q1 : k == 2 ? q2 : q3;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int u = 32 * w + 8 * k + e;
                const int x = v[e];
                if (u >= lead && u < lead + n) {
                    s1 += x;
                    s2 += (unsigned)(x * x);
                    a.kmin = min(a.kmin, x);
                    a.kmax = max(a.kmax, x);
                }
            }
        }
    }
    wS1[w] = s1;
    wS2[w] = s2;
    a.K += s1;
}
// R1 of the FAST layout: the interior words from the registers, every lane alike (r1_interior),
// and the clip's two edge words -- whose samples outside the clip must not count -- by one wave,
// a sample per lane re-read from L2 (r1_edges): on the owning lanes the per-sample branches of
// r1_word's edge loop cost their waves ~300 instructions before the R1 barrier.
// Sum k^2 of two sample pairs in one 32-bit v_dot2 chain (sq2acc(d1, sq2(d0))), added to the
// 64-bit word sum once per two pairs: the four squares sum to at most 2^32, and reach it only when
// all four samples are -32768 -- the chain then wraps to 0.  A clip holding a -32768 sample
// (ClipStats::kneg, known after the R1 reduction) has its interior word sums redone pair by pair
// (r1_redo_s2) before anything reads them.
__device__ __forceinline__ void r1_interior(const short8 *q, int w, R1Acc &a, int *wS1, unsigned long long *wS2)
{
    int s1 = 0;
    unsigned long long s2 = 0;
    const short2v ones = {1, 1};
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int h = 0; h < 4; h += 2) {
            const short2v d0 = half_pair(q[k], h), d1 = half_pair(q[k], h + 1);
            a.pmin = __builtin_elementwise_min(a.pmin, d0);
            a.pmax = __builtin_elementwise_max(a.pmax, d0);
            a.pmin = __builtin_elementwise_min(a.pmin, d1);
            a.pmax = __builtin_elementwise_max(a.pmax, d1);
            s1 = __builtin_amdgcn_sdot2(d0, ones, s1, false);
            s1 = __builtin_amdgcn_sdot2(d1, ones, s1, false);
            s2 += (unsigned)sq2acc(d1, sq2(d0));  // < 2^32 unless all four are -32768
        }
    wS1[w] = s1;
    wS2[w] = s2;
    a.K += s1;
}
__device__ __forceinline__ void r1_redo_s2(const short8 *q, int w, unsigned long long *wS2)
{
    unsigned long long s2 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int h = 0; h < 4; h++) s2 += (unsigned)sq2(half_pair(q[k], h));  // <= 2^31: unsigned
    wS2[w] = s2;
}
// lane l: sample l & 31 of the first word (l < 32) or of the last (l >= 32, clips of two words or
// more); issued at R1's start, consumed (r1_edges) after the interior words
__device__ __forceinline__ int r1_edge_issue(const ExtractParams &p, const ClipRef &cur, int lane)
{
    const int w = lane < 32 ? 0 : cur.nword - 1, u = 32 * w + (lane & 31);
    const bool valid = (lane < 32 || cur.nword > 1) && u >= cur.lead && u < cur.lead + cur.n;
    const int x = (short)__builtin_amdgcn_raw_buffer_load_b16(clip_rsrc(p, cur), valid ? 2 * u : 0x40000000, 0, 0);
    return valid ? x : 0x7fffffff;  // the marker is outside int16
}
__device__ __forceinline__ void r1_edges(int xv, int nword, int lane, R1Acc &a, int *wS1, unsigned long long *wS2)
{
    const bool valid = xv != 0x7fffffff;
    const int x = valid ? xv : 0;
    if (valid) {
        a.kmin = min(a.kmin, x);
        a.kmax = max(a.kmax, x);
    }
    a.K += x;
    // the two words' moments by LDS integer atomics (exact in any order); one wave's LDS
    // operations execute in program order, so the zeroing lands first
    const int w = lane < 32 ? 0 : nword - 1;
    if ((lane & 31) == 0 && (lane == 0 || nword > 1)) {
        // (zeros made here: a 64-bit zero kept live from the prologue was spilled to scratch)
        int z1 = 0;
        unsigned long long z2 = 0;
        asm volatile("" : "+v"(z1), "+v"(z2));
        wS1[w] = z1;
        wS2[w] = z2;
    }
    if (valid) {
        __hip_atomic_fetch_add(wS1 + w, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(wS2 + w, (unsigned long long)(unsigned)(x * x), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
// the wave's R1 partials -> sh->red_*[wid] (every lane of the wave active)
__device__ __forceinline__ void r1_reduce(const R1Acc &a, Shared *sh, int wid, int lane)
{
    const int kmn = min(a.kmin, min((int)a.pmin.x, (int)a.pmin.y));
    const int kmx = max(a.kmax, max((int)a.pmax.x, (int)a.pmax.y));
    const long long ks = (long long)wave_sum(a.K);  // <= 64 threads' sums < 2^31
    const int wmn = wave_min(kmn), wmx = wave_max(kmx);
    if (lane == 0) {
        sh->red_k[wid] = ks;
        sh->red_a[wid] = wmn;
        sh->red_b[wid] = wmx;
    }
}
// FAST: the R1 partials of each 16-lane row (DPP within the row only) -> 32 slots of LDS per
// quantity (in the VAD energy array, unused until pass B); wave 0 combines them in clip_stats_rows
// (round 6: every wave reduced its 64 lanes with 4 readlanes per quantity)
__device__ __forceinline__ void r1_reduce_rows(const R1Acc &a, const Ctx &c, int wid, int lane)
{
    const int kmn = min(a.kmin, min((int)a.pmin.x, (int)a.pmin.y));
    const int kmx = max(a.kmax, max((int)a.pmax.x, (int)a.pmax.y));
    const int ks = dpp_row_reduce(a.K, OpAdd()), rmn = dpp_row_reduce(kmn, OpMin()), rmx = dpp_row_reduce(kmx, OpMax());
    if ((lane & 15) == 0) {
        int *rk = reinterpret_cast<int *>(c.vE);
        const int slot = 4 * wid + (lane >> 4);
        rk[slot] = ks;
        rk[32 + slot] = rmn;
        rk[64 + slot] = rmx;
    }
}
// R2 of one buffer word: bit b set <=> buffer sample 32w + b is the clip's and k >= tpos (positive
// after preprocess).  Per 16-B vector (8 samples): each pair's (k - tpos) saturated (v_pk_sub_i16),
// the four samples of two pairs gathered by ONE v_perm as 0xFF / 0x00 bytes (selectors 8-11
// replicate the sign bit of bytes 1, 3, 5, 7), and the two gathered dwords weighted (1, 2, 4, 8)
// and (16, 32, 64, 128) by v_dot4_u32_u8: 255 x the vector's byte of negative samples (+ acc).
// The word's four values X_k combine as Z = sum 2^(8k) X_k = 255 x NEG (mod 2^32), and with 255
// added to X_0, Z x 0x01010101 = -(NEG + 1) = ~NEG, the positive bits (255 x 0x01010101 = 2^32 - 1).
// 35 VALU + one multiply per word against 52 for round 5's per-pair v_pk_lshrrev + v_dot2_u32_u16
// gather (and round 4's v_perm + quarter-rate multiply per byte).
__device__ __forceinline__ uint32_t neg_byte255(const short8 &val, short2v tt, uint32_t acc)
{
    unsigned a[4];
#pragma unroll
    for (int h = 0; h < 4; h++) a[h] = __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(half_pair(val, h), tt));
    const unsigned s03 = __builtin_amdgcn_perm(a[1], a[0], 0x0B0A0908u);  // samples 0-3: 0xFF where k < tpos
    const unsigned s47 = __builtin_amdgcn_perm(a[3], a[2], 0x0B0A0908u);  // samples 4-7
    return __builtin_amdgcn_udot4(s47, 0x80402010u, __builtin_amdgcn_udot4(s03, 0x08040201u, acc, false), false);
}
__device__ __forceinline__ uint32_t pos_word(const short8 *q, int w, int nword, int lead, int n, int tpos)
{
    const bool tbig = tpos > 32767;
    const short2v tt = {(short)(tbig ? 32767 : tpos), (short)(tbig ? 32767 : tpos)};
    const uint32_t x0 = neg_byte255(q[0], tt, 255u), x1 = neg_byte255(q[1], tt, 0u), x2 = neg_byte255(q[2], tt, 0u),
                   x3 = neg_byte255(q[3], tt, 0u);
    uint32_t P = tbig ? 0u : ((((x3 << 8) + x2) << 8) + x1 << 8) + x0;
    P = tbig ? 0u : P * 0x01010101u;
    if (w == 0 || w == nword - 1) {  // real samples only
        const int lo_ = min(max(lead - 32 * w, 0), 32), hi_ = min(max(lead + n - 32 * w, 0), 32);
        const uint32_t mhi = hi_ >= 32 ? ~0u : ((1u << hi_) - 1u);
        const uint32_t mlo = lo_ >= 32 ? 0u : ~((1u << lo_) - 1u);
        P &= mhi & mlo;
    }
    return P;
}

// inclusive prefix sum over the wave's 64 lanes: row_shr 1 / 2 / 4 / 8 within each 16-lane row,
// then row_bcast 15 / 31 carry the row totals upwards (every lane active)
__device__ __forceinline__ int wave_incl_scan(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
// FAST R2: the sign changes of buffer word w (pair 32 w + b <-> samples 32 w + b, + 1; bit 31 against
// the next word's first sample, held by the next lane: one wave holds a 64-word segment of a
// register row) counted and prefix-summed over the segment -> zw[w] (changes before w in the
// segment) and ztot[seg] (the segment's changes without its last word's bit 31, which zseg_count
// reads from posw).  Every lane active; P = 0 past the clip, as posw.
__device__ __forceinline__ void zseg_word(const uint16_t *zw_, const int *zt_, uint32_t P, int w, int lane, int seg)
{
    uint16_t *zw = const_cast<uint16_t *>(zw_);
    int *ztot = const_cast<int *>(zt_);
    const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)P, 0x130, 0xF, 0xF, true);  // wave_shl:1
    uint32_t ch = P ^ ((P >> 1) | (nb << 31));
    if (lane == 63) ch &= 0x7fffffffu;
    const int cz = __popc(ch), inc = wave_incl_scan(cz);
    zw[w] = (uint16_t)(inc - cz);
    if (lane == 63) ztot[seg] = inc;
}
// sign changes (set bits of chg_word) at buffer pairs [x0, x1) from the segment prefixes (FAST, after
// the R2 barrier), for ranges of at most two segments (x1 - x0 <= 64 * 32)
__device__ __forceinline__ int zseg_count(const uint32_t *posw, const uint16_t *zw, const int *ztot, int x0, int x1)
{
    if (x1 <= x0) return 0;
    const int w0 = x0 >> 5, w1 = x1 >> 5, s0 = w0 >> 6;
    int cnt = (int)zw[w1] - (int)zw[w0] - __popc(chg_word(posw, w0) & ((1u << (x0 & 31)) - 1u));
    if (x1 & 31) cnt += __popc(chg_word(posw, w1) & ((1u << (x1 & 31)) - 1u));
    if ((w1 >> 6) != s0) cnt += ztot[s0] + (int)(chg_word(posw, 64 * s0 + 63) >> 31);
    return cnt;
}

// remove_dc / normalize_audio (:49-75) in sample units, computed redundantly by every thread from
// the per-wave partial sums in sh->red_*: the reference's float64 mean of k/32768 is exact, so
// m = fl(K/n) and the peak is max(fl(kmax - m), fl(m - kmin)); a sample is positive after
// preprocess <=> k >= tpos.
struct ClipStats {
    double mq, Mp, invM2;
    float invMf;
    int tpos, t0, nv;
    int kneg;  // the clip holds a -32768 sample (r1_interior's paired squares may have wrapped)
};
__device__ __forceinline__ ClipStats clip_stats(const Shared *sh, int n, int L, int S, int do_vad)
{
    long long Kt = 0;
    int kmin = 0x7fffffff, kmax = -0x7fffffff - 1;
#pragma unroll
    for (int w = 0; w < NWAVE; w++) {
        Kt += sh->red_k[w];
        kmin = min(kmin, sh->red_a[w]);
        kmax = max(kmax, sh->red_b[w]);
    }
    ClipStats s;
    s.mq = uni((double)Kt / (double)n);
    s.Mp = uni(fmax((double)kmax - s.mq, s.mq - (double)kmin));
    s.tpos = uni((int)floor(s.mq) + 1);
    s.t0 = uni((int)floor(s.mq + 0.5));
    s.invMf = uni(s.Mp > 0.0 ? (float)(1.0 / s.Mp) : 0.0f);  // as dsp_extract_general (same bits)
    s.invM2 = uni(s.Mp > 0.0 ? 1.0 / (s.Mp * s.Mp) : 0.0);   // endpoint energies (one rounding)
    s.nv = (do_vad && n >= L) ? (n - L) / S + 1 : 0;
    s.kneg = kmin == -32768;
    return s;
}
// clip_stats of the FAST layout, by wave 0 from r1_reduce_rows's 32 row partials (one per lane)
__device__ __forceinline__ ClipStats clip_stats_rows(const Ctx &c, int lane, int n, int L, int S, int do_vad)
{
    const int *rk = reinterpret_cast<const int *>(c.vE);
    const int K = wave_sum(lane < 32 ? rk[lane] : 0);  // |K| < 2^31 (n <= 49 152 samples)
    const int kmin = wave_min(lane < 32 ? rk[32 + lane] : 0x7fffffff);
    const int kmax = wave_max(lane < 32 ? rk[64 + lane] : -0x7fffffff - 1);
    ClipStats s;
    s.mq = uni((double)K / (double)n);
    s.Mp = uni(fmax((double)kmax - s.mq, s.mq - (double)kmin));
    s.tpos = uni((int)floor(s.mq) + 1);
    s.t0 = uni((int)floor(s.mq + 0.5));
    s.invMf = uni(s.Mp > 0.0 ? (float)(1.0 / s.Mp) : 0.0f);  // as dsp_extract_general (same bits)
    s.invM2 = uni(s.Mp > 0.0 ? 1.0 / (s.Mp * s.Mp) : 0.0);   // endpoint energies (one rounding)
    s.nv = (do_vad && n >= L) ? (n - L) / S + 1 : 0;
    s.kneg = kmin == -32768;
    return s;
}

// p90 order statistics of the VAD energies (:198) by ONE wave, nv <= 128: the high halves of the
// order-preserving keys at the two ranks by repeated wave maxima; the rank's element is the one
// holding that high half, or, when several do, the one of the right rank among them by the full
// key -> c.sh->pa / pb
// (a ballot radix select instead of the bitonic sorts, for p90 and the medians: 70% of the VALU of
// those phases, but three times the SALU on the CU's shared scalar unit -- 100k clips 2.64 -> 2.71
// ms, profiles/r05rs_ab_select.txt; removed)
__device__ __forceinline__ void p90_select_wave(const Ctx &c, int nv, int lane)
{
    const double vi = (double)(nv - 1) * 0.9;
    int r0, r1;
    if (vi >= (double)(nv - 1)) {
        r0 = r1 = nv - 1;
    } else {
        r0 = (int)floor(vi);
        r1 = r0 + 1;
    }
    const bool in0 = lane < nv, in1 = lane + 64 < nv;
    const unsigned long long f0 = in0 ? dkey(c.vE[lane]) : 0ull;  // pads: below every real key
    const unsigned long long f1 = in1 ? dkey(c.vE[lane + 64]) : 0ull;
    const unsigned o0 = (unsigned)(f0 >> 32), o1 = (unsigned)(f1 >> 32);
    // the high key words at ascending ranks r1 and r0 are the (nv - 1 - r1)-th and (nv - 1 - r0)-th
    // largest (0-based): that many wave maxima, one occurrence removed after each (11 rounds at
    // nv = 98; round 6 sorted all 128 slots: 28 bitonic stages over two registers, 0.31k VALU per
    // clip for the whole selection, profiles/r06t_ab_p90.txt)
    const int d1 = nv - 1 - r1, d0 = nv - 1 - r0;
    unsigned h0 = o0, h1 = o1, ka = 0, kb = 0;
    for (int t = 0;; t++) {
        const unsigned m = wave_reduce(h0 > h1 ? h0 : h1, OpMax());
        if (t == d1) kb = m;
        if (t == d0) {
            ka = m;
            break;
        }
        const unsigned long long b0 = __ballot(h0 == m);
        if (b0) {
            if (lane == __ffsll((long long)b0) - 1) h0 = 0u;
        } else {
            if (lane == __ffsll((long long)__ballot(h1 == m)) - 1) h1 = 0u;
        }
    }
    // the rank's element is the one holding that high word, or, when several do, the one of the
    // right rank among them by the full key
    auto full_at = [&](int r) -> double {
        const unsigned kh = r == r0 ? ka : kb;
        const unsigned long long c0 = __ballot(in0 && o0 == kh), c1 = __ballot(in1 && o1 == kh);
        if (__popcll(c0) + __popcll(c1) == 1)
            return dkey_value(c0 ? lane_read(f0, __ffsll((long long)c0) - 1)
                                 : lane_read(f1, __ffsll((long long)c1) - 1));
        const int rr = r - (__popcll(__ballot(in0 && o0 < kh)) + __popcll(__ballot(in1 && o1 < kh)));
        unsigned long long res = 0;
        for (int hh = 0; hh < 2; hh++) {
            unsigned long long cm = hh ? c1 : c0;
            while (cm) {
                const int l = __ffsll((long long)cm) - 1;
                cm &= cm - 1;
                const unsigned long long e = lane_read(hh ? f1 : f0, l);
                const int lt = __popcll(__ballot(in0 && o0 == kh && f0 < e)) + __popcll(__ballot(in1 && o1 == kh && f1 < e));
                const int eq = __popcll(__ballot(in0 && f0 == e)) + __popcll(__ballot(in1 && f1 == e));
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

// the partial word endpoint pass A needs for frame end t = tid (FAST layout: one frame end per
// thread), issued early so that it is in flight across a barrier; past the range it reads zeros
__device__ __forceinline__ int vad_partial_issue(const ExtractParams &p, const ClipRef &cur, int L, int S, int nv,
                                                 int t, short8 (&qa)[4], int &e0, int &e1)
{
    const int pw = vad_partial_word(cur, L, S, nv, t, e0, e1);
    const __amdgpu_buffer_rsrc_t rs = clip_rsrc(p, cur);
    const int off = pw >= 0 ? 64 * pw : 0x40000000;
#pragma unroll
    for (int k = 0; k < 4; k++)
        qa[k] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * k, 0, 0));
    return pw;
}

// VAD frames, FAST layout (nv <= 128 <= NT / 2): one lane pair per frame -- lane h of pair f owns
// frame end t = 2f + h = tid (its partial word qa issued by vad_partial_issue), adds that word's
// exact moments, and half of the interior word sums and of the sign changes; no pass-A barrier.
// Frame f = buffer samples [u0, u0 + L): exact moments (wS1/wS2 words + the partial words at its
// ends), sign changes from the positive bits -> c.vE / c.vZ.
__device__ __forceinline__ void vad_frames_fast(const Ctx &c, const ClipRef &cur, int L, int S, const ClipStats &cs,
                                                const short8 (&qa)[4], int pa_w, int pa_e0, int pa_e1, int tid)
{
    const int nv = cs.nv, lead = cur.lead;
    const int f = tid >> 1, lh = tid & 1;
    const bool act = f < nv;
    int s1 = 0;
    unsigned long long s2 = 0;
    int zc = 0;
    if (act) {
        const int u0 = lead + f * S, u1 = u0 + L;
        const int wa = u0 >> 5, wb = (u1 - 1) >> 5;
        const int wi0 = (u0 & 31) ? wa + 1 : wa, wi1 = (u1 & 31) ? wb - 1 : wb;
        const int per = (wi1 - wi0 + 2) >> 1;
        const int ws = wi0 + lh * per, we = min(ws + per - 1, wi1);
#pragma unroll 4
        for (int w = ws; w <= we; w++) {
            s1 += c.wS1[w];
            s2 += c.wS2[w];
        }
        // sign changes at pairs [u0, u1 - 1) from R2's segment prefixes (lane 0 of the pair)
        zc = lh ? 0 : zseg_count(c.posw, c.zw, c.ztot, u0, u1 - 1);
        // the partial word last: its load (issued before the R2 barrier) lands while the LDS
        // sums above run
        if (pa_w >= 0 && !(DSP_ABL & 8)) partial_moments_fast(qa, pa_e0, pa_e1, cs.kneg, s1, s2);
    }
    s1 += dpp_i(s1, DPP_QXOR1);
    {
        const unsigned lo = dpp_i((int)(unsigned)s2, DPP_QXOR1), hi = dpp_i((int)(unsigned)(s2 >> 32), DPP_QXOR1);
        s2 += ((unsigned long long)hi << 32) | lo;
    }
    zc += dpp_i(zc, DPP_QXOR1);
    if (act && lh == 0) {
        c.vE[f] = energy_from_moments(s2, s1, L, cs.t0, cs.mq - (double)cs.t0, cs.invM2);
        c.vZ[f] = zc;
    }
}

// R4: windowed frames over the crop [st, en) (:378, :299-333; fe.py:12-43) -> c.fE / fM / fZ.
// One 16-lane row per frame (4 frames per wave), in the canonical order of dsp_device.h: the
// frame's clip-relative 8-sample vectors are re-read from L2 (16-B loads at the clip's own 2-byte
// alignment) and lane rl takes vectors va + rl + 16k, so the sums do not depend on where the clip
// sits in the buffer and equal dsp_extract_general's.  Per sample y = w_j x (the reference's
// windowed frame, :329-331), E += y^2, M += |y|; the weights of a vector's 8 samples are two
// aligned 16-B reads from the window copy shifted by fs mod 4.  Returns F.
// vectors per lane in one batch from L2: 7 (896 samples per row) leaves the FAST kernel without
// VGPR spills; 9 (a whole 1102-sample frame) 2.71 ms, 7 2.65 ms, 6 / 8 2.61-2.64 / 2.66-2.68 ms at
// 100k clips (profiles/r05s_ab_prefetch_kv.txt, r05kv_ab_r4_batch.txt)
static constexpr int R4_KV = 7;
template <bool ZSEG>  // ZCR from R2's segment prefixes (clip_fast) or by the row's lanes (clip_body)
__device__ __forceinline__ int r4_frames(const ExtractParams &p, const Ctx &c, const ClipRef &cur, int L, int S,
                                         int st, int en, const ClipStats &cs, int j0, int j1, int wrank, int lane)
{
    const int n = cur.n, lead = cur.lead;
    const int m = en - st;  // > 0 always (start < end)
    const int F = (m <= L) ? 1 : (m - L + S - 1) / S + 1;
    const float sE = cs.invMf * cs.invMf, sM = cs.invMf;
    const int wrow = EXTRACT_WROW(L);
    const CanonX cx = canon_x(cs.mq, cs.t0);
    // a 16-B load ending past the clip's last buffer vector drops a dword that straddles the
    // descriptor's end (range checks are per dword): with an odd lead and a clip ending on a
    // vector boundary that dword holds the last sample, patched in from the aligned vector
    const int vfix = ((lead & 1) && ((lead + n) & 7) == 0) ? (n - 1) >> 3 : -1;
    const short klast = vfix >= 0 ? load_vec(p, cur, cur.nvec - 1)[7] : (short)0;
    auto frame_vec = [&](auto padded_t, auto near_t, const short8 &x8, const float *wr, int jb, int lim,
                         float2v &ea, float &m0, float &m1) {
        constexpr bool PADDED = decltype(padded_t)::value, NEAR0 = decltype(near_t)::value;
        const float4 wa = *reinterpret_cast<const float4 *>(wr + jb);
        const float4 wb = *reinterpret_cast<const float4 *>(wr + jb + 4);
        const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
        for (int h = 0; h < 4; h++) {
            float2v w = {wv[2 * h], wv[2 * h + 1]};
            if (PADDED) {  // samples past the crop are zero padding
                const int j = jb + 2 * h;  // window index of the pair's first sample
                w.x = j < lim ? w.x : 0.f;
                w.y = j + 1 < lim ? w.y : 0.f;
            }
            canon_pair(w, canon_x2<NEAR0>(x8[2 * h], x8[2 * h + 1], cx), ea, m0, m1);
        }
    };
    constexpr int KV = R4_KV;
    const int rl = lane & 15, row = lane >> 4;
    for (int gi = wrank; !(DSP_ABL & 1) && 4 * gi < F; gi += NWAVE) {
        const int g = 4 * gi + row;
        const bool act = g < F;
        const int gc = act ? g : F - 1;
        const int fs = st + gc * S;
        const int lim = min(L, en - fs);  // samples beyond the crop are zero padding
        const bool padded = lim < L;
        const int va = fs >> 3, vb = (fs + lim - 1) >> 3;
        const int r = fs & 3;  // copy whose rows start at window index = -fs (mod 4)
        const float *wr = c.wtab + r * wrow + EXTRACT_WPAD + r;  // wr[j] = w[j], j = -7 .. L + 7
        float2v ea = {0.f, 0.f};
        float m0 = 0.f, m1 = 0.f;
        for (int v0 = va; v0 <= vb; v0 += 16 * KV) {
            // the lane's vectors v0 + rl + 16k: one per-lane base (vl) and immediate offsets, a
            // per-lane bound (vlim) against uniform 16k -- nine hoisted per-k indices spilled at
            // 80 VGPRs and every reload waited for all of the batch's loads
            const int vl = v0 + rl, vlim = vb - vl;
            short8 xv[KV];
#pragma unroll
            for (int k = 0; k < KV; k++) xv[k] = load_cvec(p, cur, vl + 16 * k);
            if (vfix >= 0)  // clip-uniform, rare
#pragma unroll
                for (int k = 0; k < KV; k++)
                    if (vl + 16 * k == vfix) xv[k][(n - 1) & 7] = klast;
            const int jl = 8 * vl - fs;  // window index of the lane's first vector
            auto run = [&](auto pt, auto nt, auto ft) {
#pragma unroll
                for (int k = 0; k < KV; k++)
                    if (decltype(ft)::value || 16 * k <= vlim) frame_vec(pt, nt, xv[k], wr, jl + 128 * k, lim, ea, m0, m1);
            };
            // a batch every lane fills (the first of an unpadded frame) runs without the per-vector
            // lane bounds
            const bool full = !padded && __all(vlim >= 16 * (KV - 1));
            if (padded)
                cx.near0 ? run(BoolT<true>(), BoolT<true>(), BoolT<false>()) : run(BoolT<true>(), BoolT<false>(), BoolT<false>());
            else if (cx.near0)
                full ? run(BoolT<false>(), BoolT<true>(), BoolT<true>()) : run(BoolT<false>(), BoolT<true>(), BoolT<false>());
            else
                full ? run(BoolT<false>(), BoolT<false>(), BoolT<true>()) : run(BoolT<false>(), BoolT<false>(), BoolT<false>());
        }
        const float E1 = dpp_row_reduce(ea.x + ea.y, OpAdd()) * sE;
        const float M1 = dpp_row_reduce(m0 + m1, OpAdd()) * sM;
        // ZCR of the windowed, padded frame: a sample's sign survives where w_j > 0 (j in
        // [j0, j1]) and j < lim; transitions into the window's zero ends / padding count too
        const int ia = fs + j0, ib = min(fs + j1, en - 1);  // sample coords
        int z = 0;
        if constexpr (ZSEG) {  // one lane per frame
            if (rl == 0 && ia <= ib) {
                z = zseg_count(c.posw, c.zw, c.ztot, ia + lead, ib + lead);
                if (j0 > 0) z += pos_bit(c.posw, ia + lead);
                if (ib < fs + L - 1) z += pos_bit(c.posw, ib + lead);
            }
        } else {
            z = dpp_row_reduce(ia < ib ? chg_count(c.posw, ia + lead, ib + lead, rl, 16) : 0, OpAdd());
            if (ia <= ib) {
                if (j0 > 0) z += pos_bit(c.posw, ia + lead);
                if (ib < fs + L - 1) z += pos_bit(c.posw, ib + lead);
            }
        }
        if (act && rl == 0) {
            c.fE[g] = E1;
            c.fM[g] = M1;
            c.fZ[g] = z;
        }
    }
    return F;
}

// R5 for F <= 128 (compute_statistics x 3, fe.py:46-62): six jobs on waves 0..5 -- wave q (q < 3)
// the median of sequence q (E, M, ZCR) by an in-wave bitonic sort, wave 3 + q its mean /
// population std (fp64 sums) / max / min -- no barrier.  np.median: the middle order statistic
// (odd F) or the mean of the two middle ones.
__device__ __forceinline__ void r5_fast(const Ctx &c, int F, float *featb, int wid, int lane)
{
    const int r0 = (F - 1) / 2, r1 = F / 2;
    for (int job = wid; !(DSP_ABL & 2) && job < 6; job += NWAVE) {
        const int q = job % 3;
        auto get = [&](int j) -> float { return q == 0 ? c.fE[j] : q == 1 ? c.fM[j] : (float)c.fZ[j]; };
        const bool in0 = lane < F, in1 = lane + 64 < F;
        const float x0 = in0 ? get(lane) : 0.f, x1 = in1 ? get(lane + 64) : 0.f;
        if (job < 3) {  // median by an in-wave bitonic sort
            unsigned a[2] = {in0 ? fkey(x0) : ~0u, in1 ? fkey(x1) : ~0u};
            float v0, v1;
            if (F <= 32) {  // (the typical crop: 15 compare-exchange stages instead of 21)
                unsigned b[1] = {a[0]};
                wave_bitonic<1, unsigned, 32>(b, lane);
                v0 = fkey_value(sorted_at<1>(b, r0));
                v1 = fkey_value(sorted_at<1>(b, r1));
            } else if (F <= 64) {
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
        }
        if (job >= 3) {  // mean, population std (fp64 sums), max, min
            const double s = wave_sum((in0 ? (double)x0 : 0.0) + (in1 ? (double)x1 : 0.0));
            const float mx = wave_reduce(fmaxf(in0 ? x0 : -INFINITY, in1 ? x1 : -INFINITY), OpMax());
            const float mn = wave_reduce(fminf(in0 ? x0 : INFINITY, in1 ? x1 : INFINITY), OpMin());
            const double mean = s / (double)F;
            const double d0 = in0 ? (double)x0 - mean : 0.0, d1 = in1 ? (double)x1 - mean : 0.0;
            const double qq = wave_sum(fma(d0, d0, d1 * d1));
            if (lane < 4) {
                const double o = lane == 0 ? mean : lane == 1 ? sqrt(qq / (double)F) : lane == 2 ? (double)mx
                                 : (double)mn;
                featb[5 * q + lane] = (float)o;
            }
        }
    }
}

// Clip queue (ABI 5).  p.queue: the caller's zeroed 4 KiB scratch, words 0-7 the claim counters
// of eight ranges of clip chunks (p.qchunk consecutive clips each), word 8 the count of workgroups
// done.  Workgroup b's first chunk is chunk b, taken without a claim; the chunks after the first G
// ([G, nch)) form the eight ranges (range x = [G + x D / 8, G + (x + 1) D / 8), D = nch - G).  A
// workgroup claims chunks from the range of the XCD it runs on (HW_REG_XCC_ID: placement is a
// performance matter only, any id is correct), then from the others in turn once its own is
// exhausted: one atomic per chunk instead of per clip, consecutive clips on one XCD -- their 76-B
// output rows share cache lines in that XCD's L2 instead of leaving it as partial-line writes --
// and fast workgroups take more chunks (a static i, i + G, ... split ends on the slowest
// workgroup: 3.19-3.98 ms spread at 100 000 clips).  The chunk is 4 clips, 2 for batches of fewer
// than 64 clips per workgroup (12 500 clips: 0.506 -> 0.484 ms, a shorter tail; 100 000: 3.387
// against 3.409 ms with 2; profiles/r04x_queue_chunk_ab.txt).  p.qchunk == 0 (at most two clips
// per workgroup) or p.queue == NULL: the static split, no claims.  Thread 0 only.
static constexpr int XCD_RANGES = 8;  // one per XCD (queue_ws holds 8 range counters)
// queue_ws word w of the layout lives at word w * QSTRIDE: every counter on its own 256-B
// line.  Agent-scope atomics on one line serialise (across the eight XCDs they go past the L2s),
// and with all eight counters in one 64-B line the claims of 768 workgroups queued behind each
// other: at 12 500 clips the clips that claimed late in the launch took up to 85 us (p99 73 us).
// One line per counter: 12.5k clips 0.454-0.459 -> 0.436-0.440 ms (span p99 73 -> 35 us, workgroups
// p50 402 -> 363 us), 100k 2.634-2.656 -> 2.616-2.621 ms (profiles/r05qs_ab_queue_lines.txt,
// r05qs_stamps.txt).  Probing the other ranges with loads before claiming: 2.75 ms at 100k.
static constexpr int QSTRIDE = 64;
static_assert(11 * QSTRIDE * 4 <= DSP_QUEUE_WS_BYTES, "queue_ws too small for the counter layout");
__device__ __forceinline__ unsigned *qword(unsigned *q, int w) { return q + w * QSTRIDE; }
struct ClipQueue {  // wave-uniform; the mutable state lives in Shared (thread 0 only)
    unsigned *q;
    int B, nch, xcd, ch;
    int s0;  // chunks [0, s0) are the workgroups' first, one each (chunk blockIdx.x), without a claim
};
__device__ __forceinline__ ClipQueue queue_open(const ExtractParams &p, Shared *sh)
{
    ClipQueue Q;
    Q.q = p.qchunk > 0 ? p.queue : nullptr;  // qchunk 0: the static split (short batches)
    Q.B = p.B;
    Q.ch = max(p.qchunk, 1);  // a power of two <= EXTRACT_OSTAGE (host), so chunks never straddle a stage group
    Q.nch = (p.B + Q.ch - 1) / Q.ch;
    Q.s0 = min(Q.nch, (int)gridDim.x);
    Q.xcd = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7;  // HW_REG_XCC_ID[3:0]
    if (threadIdx.x == 0) {
        // the first chunk is chunk blockIdx.x: no launch-time claim (768 workgroups on 8 counters
        // serialised ~4.8 us of every workgroup's prologue)
        const int b = (int)blockIdx.x;
        sh->qnext = b < Q.nch ? b * Q.ch : 0;
        sh->qend = b < Q.nch ? min(Q.B, b * Q.ch + Q.ch) : 0;
        sh->qrange = 0;
        sh->qcursor = (int)blockIdx.x - (int)gridDim.x;
    }
    return Q;
}
// Claiming is split so that the counter's atomic never stalls the clip: queue_begin (at the clip's
// start, right after its loads) issues the atomic when the current chunk is used up, and
// queue_end (before R5) consumes its result.  The vmcnt counter is in order, so a wait for an
// atomic issued after the clip's loads would also wait for those loads.  Thread 0 only.
// The pending claim's state sits in LDS (sh->cdir: the next clip, -1, or -2 = pending on the
// atomic; sh->cy: its range); only the atomic's return value stays in a register.
__device__ __forceinline__ unsigned queue_begin(const ClipQueue &Q, Shared *sh)
{
    if (!Q.q) {
        const int t = sh->qcursor + (int)gridDim.x;
        sh->qcursor = t;
        sh->cdir = t < Q.B ? t : -1;
        return 0;
    }
    const int nx = sh->qnext;
    if (nx < sh->qend) {
        sh->qnext = nx + 1;
        sh->cdir = nx;
        return 0;
    }
    if (sh->qrange >= XCD_RANGES || Q.s0 == Q.nch) {  // every range exhausted, or none
        sh->cdir = -1;
        return 0;
    }
    const int y = (Q.xcd + sh->qrange) % XCD_RANGES;
    sh->cy = y;
    sh->cdir = -2;
    return __hip_atomic_fetch_add(qword(Q.q, y), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int queue_end(const ClipQueue &Q, Shared *sh, unsigned ret)
{
    constexpr int NR = XCD_RANGES;
    if (sh->cdir != -2) return sh->cdir;
    int y = sh->cy;
    for (;;) {
        const int D = Q.nch - Q.s0;  // the claimed chunks [s0, nch), in NR ranges
        const int c0 = Q.s0 + y * D / NR, c1 = Q.s0 + (y + 1) * D / NR;
        // the range's clips [r0, r1): chunks of ch, then its last ~2 clips per workgroup of an XCD
        // one at a time, so that the workgroups run out of work together (guided tail)
        const int r0 = c0 * Q.ch, r1 = min(Q.B, c1 * Q.ch);
        const int nbig = max(0, r1 - r0 - 2 * ((int)gridDim.x / NR)) / Q.ch;
        const int first = (int)ret < nbig ? r0 + (int)ret * Q.ch : r0 + nbig * Q.ch + ((int)ret - nbig);
        if ((int)ret < nbig || first < r1) {
            sh->qnext = first + 1;
            sh->qend = (int)ret < nbig ? first + Q.ch : first + 1;
            return first;
        }
        // this range is used up: the next one (a blocking claim, rare: the end of the launch)
        int r = ++sh->qrange;
        if (r >= NR) return -1;
        y = (Q.xcd + r) % NR;
        ret = __hip_atomic_fetch_add(qword(Q.q, y), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__device__ __forceinline__ int queue_next(const ClipQueue &Q, Shared *sh) { return queue_end(Q, sh, queue_begin(Q, sh)); }
// the last workgroup out resets the queue for the next launch on the stream: every claim of every
// workgroup precedes its increment of the done count.  Thread 0 only.
__device__ __forceinline__ void queue_done(const ExtractParams &p)
{
    if (!p.queue) return;
    const unsigned d = __hip_atomic_fetch_add(qword(p.queue, 8), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == gridDim.x - 1) {
#pragma unroll
        for (int y = 0; y < 8; y++) __hip_atomic_store(qword(p.queue, y), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(qword(p.queue, 8), 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One clip, start to finish; its first RREG words are already in flight into regs (word
// r * NT + tid in regs[4r .. 4r+3]).  EXACT = false: endpoint energies from exact moments,
// decisions certified; returns false on a near tie (the clip is then redone with EXACT = true
// after the persistent loop).
// FAST: the compile-time LDS layout (extract_carve_fast); the clip is in registers and there are
// at most 128 VAD and feature frames, so the long-clip paths drop out
struct NoClaim {
    __device__ int operator()() const { return -1; }
};
template <bool EXACT, bool FAST, typename Resolve = NoClaim>
__device__ __forceinline__ bool clip_body(const ExtractParams &p, const Ctx &c, int i, const ClipRef &cur,
                                          short8 (&regs)[NRV], Resolve resolve = NoClaim())
{
    Shared *sh = c.sh;
    // (the generic layout's and the exact redo's index arithmetic spills when hoisted: opaque
    // thread index there)
    const int tid = (FAST && !EXACT) ? (int)threadIdx.x : opaque_tid(), lane = tid & 63,
              wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
    // frame sizes opaque per clip as well: constants derived from them ((double)L, ...) are
    // recomputed in the clip instead of being kept live across the loop
    int L = p.L, S = p.S;
    asm volatile("" : "+s"(L), "+s"(S));
    const int n = cur.n, lead = cur.lead, nword = cur.nword;
    // outputs: the main kernel stages them in LDS (slot i mod EXTRACT_OSTAGE) and the workgroup
    // writes a chunk's clips together (flush_outputs); the exact redo writes them directly
    const int oslot = i & (EXTRACT_OSTAGE - 1);
    float *featb = EXACT ? out_feat(p, i) : reinterpret_cast<float *>(c.orow + DSP_OUT_ROW_WORDS * oslot);
    const int16_t *clip_g = p.pcm + cur.base + lead;  // the clip in global memory, sample coords
    STAMP(i, 0);
#ifdef DSP_STAMPS
    if (p.stamps) {  // diagnostic build: the clip's loads landed (stamp 13; per wave: 24 + wave)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP(i, 13);
        if (lane == 0) p.stamps[(size_t)i * 32 + 24 + wid] = __builtin_amdgcn_s_memtime();
    }
#endif

    // ---- R1: integer sum / min / max; exact moments per 32-sample word -----------------------
    R1Acc acc = r1_acc_init();  // K <= RREG * 32 * 32768 per thread (longer clips: one word per trip)
    // clips of up to RREG * NT words stream from the registers loaded before this call; longer
    // ones are read word by word here and again in R2 (the second read hits L2)
    const bool inreg = FAST || nword <= RREG * NT;
    if (inreg) {
#pragma unroll
        for (int r = 0; r < RREG; r++) {
            const int w = r * NT + tid;
            if (w < nword) r1_word(&regs[4 * r], w, nword, lead, n, acc, c.wS1, c.wS2);
        }
    } else {
#pragma unroll 1
        for (int w = tid; w < nword; w += NT) {
            short8 q[4];
            issue_word(q, p, cur, w);
            r1_word(q, w, nword, lead, n, acc, c.wS1, c.wS2);
        }
    }
    r1_reduce(acc, sh, wid, lane);
    __syncthreads();
    if (!EXACT && tid == 0 && sh->sclear) {  // the last flush's slots (every thread has read them)
        sh->smask = 0;
        sh->schunk = -1;
        sh->sclear = 0;
    }
    // wave 0 computes the clip statistics once and shares them (a second barrier), instead of
    // every wave repeating the fp64 work (3.415 -> 3.386 ms at 100k clips, round 4)
    if (wid == 0) {
        const ClipStats c0 = clip_stats(sh, n, L, S, p.do_vad);
        if (lane == 0) sh->cs = {c0.mq, c0.Mp, c0.invM2, c0.invMf, c0.tpos, c0.t0, c0.nv, c0.kneg};
    }
    __syncthreads();
    ClipStats cs;
    cs.mq = uni(sh->cs.mq);
    cs.Mp = uni(sh->cs.Mp);
    cs.invM2 = uni(sh->cs.invM2);
    cs.invMf = uni(sh->cs.invMf);
    cs.tpos = uni(sh->cs.tpos);
    cs.t0 = uni(sh->cs.t0);
    cs.nv = uni(sh->cs.nv);
    const double mq = cs.mq, Mp = cs.Mp;
    const int tpos = cs.tpos, t0 = cs.t0, nv = cs.nv;
    STAMP(i, 1);

    // ---- R2: positive-sample bits, one 32-bit word per 32 buffer samples ---------------------
    if (inreg) {
#pragma unroll
        for (int r = 0; r < RREG; r++) {
            const int w = r * NT + tid;
            if (w < nword) c.posw[w] = (DSP_ABL & 4) ? 0u : pos_word(&regs[4 * r], w, nword, lead, n, tpos);
        }
    } else {
#pragma unroll 1
        for (int w = tid; w < nword; w += NT) {
            short8 q[4];
            issue_word(q, p, cur, w);
            c.posw[w] = pos_word(q, w, nword, lead, n, tpos);
        }
    }
    if (tid < 2) c.posw[nword + tid] = 0;
    // the partial words that endpoint pass A needs (FAST: one frame end per thread), issued
    // before the barrier so that they are in flight while the workgroup synchronises
    short8 qa[4];
    int pa_w = -1, pa_e0 = 0, pa_e1 = 0;
    if constexpr (!EXACT) {
        if constexpr (FAST) pa_w = vad_partial_issue(p, cur, L, S, nv, tid, qa, pa_e0, pa_e1);
    }
    __syncthreads();
    STAMP(i, 2);

    // ---- R3: endpoint detection (:161-273) ------------------------------------------------
    int st = 0, en = n;
    if (nv > 0) {
        // frame f = buffer samples [u0, u0 + L): exact moments from the word sums plus the two
        // partial words at its ends, sign changes from the bits.
        // Pass A, one thread per frame end: the partial word's moments (FAST: loaded before the
        // next clip's prefetch; otherwise re-read from L2 here).
        if constexpr (FAST && !EXACT) {
            vad_frames_fast(c, cur, L, S, cs, qa, pa_w, pa_e0, pa_e1, tid);
            STAMP(i, 7);
        } else {
            {
                if constexpr (!EXACT) {
                    {  // generic layout: the partial words re-read from L2 here
                        for (int t = tid; t < 2 * nv; t += NT) {
                            int e0, e1, t1 = 0;
                            unsigned long long t2 = 0;
                            const int pw = vad_partial_word(cur, L, S, nv, t, e0, e1);
                            if (pw >= 0) {
                                short8 q[4];
    #pragma unroll
                                for (int k = 0; k < 4; k++) q[k] = load_vec(p, cur, 4 * pw + k);
                                partial_moments(q, e0, e1, t1, t2);
                            }
                            c.pS1[t] = t1;
                            c.pS2[t] = t2;
                        }
                    }
                    __syncthreads();
                    STAMP(i, 7);
                }
                // Pass B, one quad per frame: interior word sums and sign changes, each lane a
                // contiguous quarter
                const int q4 = tid >> 2, lq = tid & 3;
                for (int f0 = 0; f0 < nv; f0 += NT / 4) {
                    const int f = f0 + q4;
                    const bool act = f < nv;
                    int s1 = 0;  // |frame sum| <= L * 32768 < 2^31 for L < 65536
                    unsigned long long s2 = 0;
                    int zc = 0;
                    if (act) {
                        const int u0 = lead + f * S, u1 = u0 + L;
                        if (!EXACT) {
                            const int wa = u0 >> 5, wb = (u1 - 1) >> 5;
                            const int wi0 = (u0 & 31) ? wa + 1 : wa, wi1 = (u1 & 31) ? wb - 1 : wb;
                            const int per = (wi1 - wi0 + 4) >> 2;
                            const int ws = wi0 + lq * per, we = min(ws + per - 1, wi1);
    #pragma unroll 3
                            for (int w = ws; w <= we; w++) {
                                s1 += c.wS1[w];
                                s2 += c.wS2[w];
                            }
                            if (lq == 0) {
                                s1 += c.pS1[2 * f] + c.pS1[2 * f + 1];
                                s2 += c.pS2[2 * f] + c.pS2[2 * f + 1];
                            }
                        }
                        const int np_ = L - 1, pq = (np_ + 3) >> 2;  // pairs [u0, u1 - 1) in quarters
                        const int x0 = u0 + min(lq * pq, np_), x1 = u0 + min((lq + 1) * pq, np_);
                        zc = chg_run(c.posw, x0, x1);
                    }
                    s1 = dpp_quad_reduce(s1, OpAdd());
                    s2 = dpp_quad_sum64(s2);
                    zc = dpp_quad_reduce(zc, OpAdd());
                    if (act && lq == 0) {
                        if (!FAST) c.rank[f] = 0;
                        c.vE[f] = EXACT ? np_energy_exact(clip_g, f * S, L, mq, Mp)
                                        : energy_from_moments(s2, s1, L, t0, mq - (double)t0, cs.invM2);
                        c.vZ[f] = zc;
                    }
                }
            }
        }
        __syncthreads();
        STAMP(i, 8);
        {
            // p90 order statistics (:198)
            {
                const double vi = (double)(nv - 1) * 0.9;
                int r0, r1;
                if (vi >= (double)(nv - 1)) {
                    r0 = r1 = nv - 1;
                } else {
                    r0 = (int)floor(vi);
                    r1 = r0 + 1;
                }
                if (FAST || nv <= 128) {
                    // wave 0: bitonic sort of the high halves of the order-preserving keys; the rank's
                    // element is the one holding that high half, or, when several do, the one of the
                    // right rank among them by the full key
                    if (wid == 0) {
                        // the workgroup's critical path (p90, then the scan) runs on this one wave:
                        // it takes issue priority over the co-resident workgroup's waves until the
                        // decisions are made (2% at 100k clips)
                        __builtin_amdgcn_s_setprio(2);
                        p90_select_wave(c, nv, lane);
                    }
                } else if (nv <= 256) {
                    ballot_select<double>([&](int j) { return c.vE[j]; }, nv, r0, r1, &sh->pa, &sh->pb, wid, lane);
                } else {  // long clips: partial ranks over all waves
                    rank_partial([&](int, int j) { return c.vE[j]; }, 1, nv, c.rank, wid, lane);
                    __syncthreads();
                    for (int f = tid; f < nv; f += NT) {
                        const int r = c.rank[f];
                        if (r == r0) sh->pa = c.vE[f];
                        if (r == r1) sh->pb = c.vE[f];
                    }
                }
            }
            if (wid == 1 % NWAVE) vad_noise(c, nv, lane);  // beside wave 0's p90 selection
            __syncthreads();
        }
        STAMP(i, 3);
        if (wid == 0) {
            const int flag = vad_scan<!EXACT, FAST>(p, c, nv, lane);
            if (lane == 0) sh->exact = (!EXACT && Mp > 0.0) ? flag : 0;
            __builtin_amdgcn_s_setprio(0);
        }
        __syncthreads();
        if (!EXACT && sh->exact) {  // near tie: redo in numpy's exact order after the loop
            return false;
        }
        if (sh->n3 >= 0) {
            st = sh->n1 * S;              // :272
            en = min(sh->n6 * S + L, n);  // :273
        }
        if (p.vad_energy)
            for (int f = opaque_tid(); f < nv && f < p.ld_vad; f += NT) {
                p.vad_energy[(size_t)i * p.ld_vad + f] = c.vE[f];
                p.vad_zcr[(size_t)i * p.ld_vad + f] = c.vZ[f];
            }
    }
    STAMP(i, 4);

    // ---- R4: windowed frames over the crop [st, en) (r4_frames) --------------------------------
    const int F = r4_frames<false>(p, c, cur, L, S, st, en, cs, sh->j0, sh->j1, wid, lane);
    STAMP(i, 12);
    if (!FAST && F > 128)
        for (int t = tid; t < 3 * F; t += NT) c.rank[t] = 0;
    if constexpr (!EXACT)
        if (tid == 0) sh->next = resolve();  // claimed at the clip's start (-1: none)
    __syncthreads();
    if constexpr (!EXACT) {
        // regs are dead since R2: the next clip's words load while R5 runs (unconditional, a
        // clip_none() reads zeros, so the compiler's vmcnt bookkeeping stays exact)
        const int nx = sh->next;
        issue_clip(regs, p, nx >= 0 ? clip_ref(p, nx) : clip_none(), tid);
    }
    STAMP(i, 5);

    // ---- R5: 15-d statistics (compute_statistics x 3, fe.py:46-62) ------------------------
    // np.median: the middle order statistic (odd F) or the mean of the two middle ones
    const int r0 = (F - 1) / 2, r1 = F / 2;
    {
        if (FAST || F <= 128) {
            r5_fast(c, F, featb, wid, lane);
        } else {  // long sequences: partial ranks over all waves, then one wave per sequence
            rank_partial([&](int q, int j) { return q == 2 ? (float)c.fZ[j] : (q == 0 ? c.fE[j] : c.fM[j]); },
                         3, F, c.rank, wid, lane);
            __syncthreads();
            for (int t = tid; t < 3 * F; t += NT) {
                const int q = t / F, e = t - q * F;
                const int r = c.rank[t];
                const double val = q == 2 ? (double)c.fZ[e] : (double)(q == 0 ? c.fE[e] : c.fM[e]);
                if (r == r0) sh->oslo[q] = val;
                if (r == r1) sh->oshi[q] = val;
            }
            __syncthreads();
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
        }
    }
    STAMP(i, 9);
    if (p.seq)
        for (int g = tid; g < F && g < p.ld_seq; g += NT) {
            float *o = p.seq + ((size_t)i * p.ld_seq + g) * 3;
            o[0] = c.fE[g];
            o[1] = c.fM[g];
            o[2] = (float)c.fZ[g];
        }
    if (tid == 0) {
        if constexpr (EXACT) {
            out_se(p, i)[0] = st;
            out_se(p, i)[1] = en;
            *out_nf(p, i) = F;
            *out_st(p, i) = DSP_CLIP_OK | DSP_CLIP_FLAG_VAD_EXACT;
        } else {
            int32_t *orow = c.orow + DSP_OUT_ROW_WORDS * oslot;
            orow[15] = st;
            orow[16] = en;
            orow[17] = F;
            orow[18] = DSP_CLIP_OK;
            const int ch = i / EXTRACT_OSTAGE;  // the staged slots belong to chunk sh->schunk
            const unsigned m0 = sh->schunk == ch ? sh->smask : 0u;
            sh->schunk = ch;
            sh->smask = m0 | (1u << oslot);
        }
    }
    STAMP(i, 6);
    return true;
}

// ==== FAST launches: clip_fast =================================================================
// Three 512-thread workgroups per CU (80 VGPRs), one clip at a time each; the clip's words are
// loaded at its start and the two other workgroups on the CU cover the wait.  Round 5's A/B at
// 100 000 clips (profiles/r05e_ab_variants.txt): 3.04 ms against 3.36 for two workgroups per CU with
// the next clip's words prefetched during R5 -- more clips in flight per CU, not earlier loads, is
// what the kernel needed (2.64 ms after the R4, edge-word and compiler changes).
// Measured and not kept (profiles/r05c_ab_crop.txt, r05d_ab_crop.txt): the crop copied into an LDS buffer after the
// decisions so that R4 reads LDS and the registers take the next clip earlier -- from the
// registers (16-way LDS bank conflicts on the copy) 3.78 ms, by LDS-DMA from L2 3.55 ms: R4 from LDS
// took as long as from L2 (2.34 against 2.39 us per clip in the stamps; it is bound by its own
// arithmetic), and the DMA's round trip sat on the critical path.  Rows of the next clip's words
// loaded during R5 (the rest at its start): 1 row 3.52 ms, 2 rows 3.70 ms against 2.85 ms without at
// 100k clips (spills; profiles/r05j_ab_prefetch_rows.txt), and with 0 spills 2.65-2.68 against
// 2.65 ms (r05s_ab_prefetch_kv.txt): not kept.

// One clip, FAST layout, not the exact redo; its RREG words are already in flight into regs (word
// r * NT + tid in regs[4r .. 4r+3]).  Endpoint energies from exact moments, decisions certified;
// returns false on a near tie (the clip is then redone by extract_exact_kernel).  Thread 0 resolves
// the next clip (sh->next) before R4, also for a deferred clip.
template <typename Resolve>
__device__ __forceinline__ bool clip_fast(const ExtractParams &p, const Ctx &c, int i, const ClipRef &cur,
                                          short8 (&regs)[NRV], Resolve resolve)
{
    Shared *sh = c.sh;
    // the thread index opaque: index arithmetic that depends only on it is recomputed where it is
    // used, instead of being hoisted out of the persistent loop and held (spilled) across it
    const int tid = opaque_tid(), lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    int L = p.L, S = p.S;
    asm volatile("" : "+s"(L), "+s"(S));  // per clip: constants derived from them are recomputed
    const int n = cur.n, lead = cur.lead, nword = cur.nword;
    const int oslot = i & (EXTRACT_OSTAGE - 1);
    float *featb = reinterpret_cast<float *>(c.orow + DSP_OUT_ROW_WORDS * oslot);
    STAMP(i, 0);
#ifdef DSP_STAMPS
    if (p.stamps) {  // diagnostic build: the clip's loads landed (stamp 13; per wave: 24 + wave)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP(i, 13);
        if (lane == 0) p.stamps[(size_t)i * 32 + 24 + wid] = __builtin_amdgcn_s_memtime();
    }
#endif

    // ---- R1: integer sum / min / max; exact moments per 32-sample word --------------------------
    MARK(R1);
    R1Acc acc = r1_acc_init();
#pragma unroll
    for (int r = 0; r < RREG; r++) {
        const int w = r * NT + tid;
        if (w < nword && w > 0 && w < nword - 1) r1_interior(&regs[4 * r], w, acc, c.wS1, c.wS2);
    }
    if (wid == NWAVE - 1) r1_edges(r1_edge_issue(p, cur, lane), nword, lane, acc, c.wS1, c.wS2);
    MARK(R1red);
    r1_reduce_rows(acc, c, wid, lane);
    __syncthreads();
    if (tid == 0 && sh->sclear) {  // the last flush's slots (every thread has read them by now)
        sh->smask = 0;
        sh->schunk = -1;
        sh->sclear = 0;
    }
    MARK(stats);
    if (wid == 0) {  // the clip statistics once, shared through LDS
        const ClipStats c0 = clip_stats_rows(c, lane, n, L, S, p.do_vad);
        if (lane == 0) sh->cs = {c0.mq, c0.Mp, c0.invM2, c0.invMf, c0.tpos, c0.t0, c0.nv, c0.kneg};
    }
    __syncthreads();
    ClipStats cs;
    cs.mq = uni(sh->cs.mq);
    cs.Mp = uni(sh->cs.Mp);
    cs.invM2 = uni(sh->cs.invM2);
    cs.invMf = uni(sh->cs.invMf);
    cs.tpos = uni(sh->cs.tpos);
    cs.t0 = uni(sh->cs.t0);
    cs.nv = uni(sh->cs.nv);
    cs.kneg = uni(sh->cs.kneg);
    const int nv = cs.nv;
    STAMP(i, 1);

    // ---- R2: positive-sample bits, one 32-bit word per 32 buffer samples ---------------------
    MARK(R2);
    if (cs.kneg) {  // rare: a -32768 sample may have wrapped r1_interior's paired squares
#pragma unroll
        for (int r = 0; r < RREG; r++) {
            const int w = r * NT + tid;
            if (w < nword && w > 0 && w < nword - 1) r1_redo_s2(&regs[4 * r], w, c.wS2);
        }
    }
    // then the partial word of the frame end this thread sums in pass A (one frame end per thread),
    // re-read from L2 and issued before the barrier so that it is in flight while the workgroup
    // synchronises.  Issued earlier, with the clip's words still live, it costs spills whose
    // reloads wait for it: at the end of R1 3.38 ms, before R2 3.18, after R2 2.82
    // (profiles/r05h_ab.txt, r05i_ab.txt)
    uint32_t P[RREG];
#pragma unroll
    for (int r = 0; r < RREG; r++) {
        const int w = r * NT + tid;
        P[r] = (w < nword && !(DSP_ABL & 4)) ? pos_word(&regs[4 * r], w, nword, lead, n, cs.tpos) : 0u;
        if (w < nword) c.posw[w] = P[r];
    }
#pragma unroll
    for (int r = 0; r < RREG; r++) zseg_word(c.zw, c.ztot, P[r], r * NT + tid, lane, r * NWAVE + wid);
    if (tid < 2) c.posw[nword + tid] = 0;
    if (tid == 0) c.zw[RREG * NT] = 0;  // (a range ending at the last register word's end)
    MARK(paissue);
    short8 qa[4];
    int pa_e0 = 0, pa_e1 = 0, pa_w = -1;
    if (64 * wid < 2 * nv)  // waves holding frame ends (2 nv <= 256: waves 0-3)
        pa_w = vad_partial_issue(p, cur, L, S, nv, tid, qa, pa_e0, pa_e1);
    __syncthreads();
    STAMP(i, 2);

    // ---- R3: endpoint detection (:161-273) ------------------------------------------------
    MARK(passAB);
    if (nv > 0) {
        vad_frames_fast(c, cur, L, S, cs, qa, pa_w, pa_e0, pa_e1, tid);
        STAMP(i, 7);
        __syncthreads();
        STAMP(i, 8);
        MARK(p90);
        if (wid == 0) {
            // the workgroup's critical path (p90, then the scan) runs on this one wave: it takes
            // issue priority over the co-resident workgroups' waves until the decisions are made
            __builtin_amdgcn_s_setprio(2);
            if (DSP_ABL & 64) {  // ablation only: no selection (thresholds from 0.8 x the largest energy)
                const double mx = wave_maxd(fmax(lane < nv ? c.vE[lane] : 0.0, lane + 64 < nv ? c.vE[lane + 64] : 0.0));
                if (lane == 0) sh->pa = sh->pb = 0.8 * mx;
            } else {
                p90_select_wave(c, nv, lane);
            }
        }
        if (wid == 1) vad_noise(c, nv, lane);  // beside wave 0's p90 selection
        __syncthreads();
        STAMP(i, 3);
        MARK(scan);
        if (wid == 0) {
            const int flag = vad_scan<true, true>(p, c, nv, lane);
            if (lane == 0) sh->exact = cs.Mp > 0.0 ? flag : 0;
        }
    }
    MARK(resolve);
    if (tid == 0) sh->next = resolve();  // claimed at the clip's start (-1: none)
    if (wid == 0) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    int st = 0, en = n;
    if (nv > 0) {
        if (sh->exact) return false;  // near tie: redone in numpy's exact order by the exact kernel
        if (sh->n3 >= 0) {
            st = sh->n1 * S;              // :272
            en = min(sh->n6 * S + L, n);  // :273
        }
        const ExtractParams &q = p;
        if (q.vad_energy)
            for (int f = opaque_tid(); f < nv && f < q.ld_vad; f += NT) {
                q.vad_energy[(size_t)i * q.ld_vad + f] = c.vE[f];
                q.vad_zcr[(size_t)i * q.ld_vad + f] = c.vZ[f];
            }
    }
    STAMP(i, 4);

    // ---- R4: windowed frames over the crop [st, en) (r4_frames) --------------------------------
    MARK(R4);
    const int F = r4_frames<true>(p, c, cur, L, S, st, en, cs, sh->j0, sh->j1, wid, lane);
    STAMP(i, 12);
    __syncthreads();
    STAMP(i, 5);

    // ---- R5: 15-d statistics (compute_statistics x 3, fe.py:46-62) ------------------------
    MARK(R5);
    r5_fast(c, F, featb, wid, lane);
    if (wid == NWAVE - 1) {
        // idle in R5: the next clip's offsets to LDS, so that the loop top does not wait for a global
        // load (nor, through the in-order vmcnt, for the flushed output stores before it)
        const int nx = sh->next;
        if (nx >= 0 && lane < 2) sh->noff[lane] = p.offsets[nx + lane];
        if (lane == 0) sh->noff_for = nx;
    }
    STAMP(i, 9);
    MARK(tail);
    const ExtractParams &qs = p;
    if (qs.seq)
        for (int g = tid; g < F && g < qs.ld_seq; g += NT) {
            float *o = qs.seq + ((size_t)i * qs.ld_seq + g) * 3;
            o[0] = c.fE[g];
            o[1] = c.fM[g];
            o[2] = (float)c.fZ[g];
        }
    if (tid == 0) {
        int32_t *orow = c.orow + DSP_OUT_ROW_WORDS * oslot;
        orow[15] = st;
        orow[16] = en;
        orow[17] = F;
        orow[18] = DSP_CLIP_OK;
        const int ch = i / EXTRACT_OSTAGE;  // the staged slots belong to chunk sh->schunk
        const unsigned m0 = sh->schunk == ch ? sh->smask : 0u;
        sh->schunk = ch;
        sh->smask = m0 | (1u << oslot);
    }
    STAMP(i, 6);
    return true;
}

__device__ __forceinline__ void write_bad_clip(const ExtractParams &p, int i, int tid)
{
    if (tid < 15) out_feat(p, i)[tid] = __builtin_nanf("");
    if (tid == 0) {
        const int64_t nn = p.offsets[i + 1] - p.offsets[i];
        *out_st(p, i) = nn <= 0 ? DSP_CLIP_EMPTY : DSP_CLIP_TOO_LONG;
        int z = 0;
        asm volatile("" : "+v"(z));
        out_se(p, i)[0] = z;
        out_se(p, i)[1] = z;
        *out_nf(p, i) = 0;
    }
}


__device__ __forceinline__ Ctx ctx_from(const ExtractCarve &cv, unsigned char *lds)
{
    Ctx c;
    c.sh = reinterpret_cast<Shared *>(lds + cv.sh);
    c.wtab = reinterpret_cast<const float *>(lds + cv.wtab);
    c.posw = reinterpret_cast<uint32_t *>(lds + cv.posw);
    c.wS2 = reinterpret_cast<unsigned long long *>(lds + cv.wS2);
    c.wS1 = reinterpret_cast<int *>(lds + cv.wS1);
    c.vE = reinterpret_cast<double *>(lds + cv.vE);
    c.vZ = reinterpret_cast<int32_t *>(lds + cv.vZ);
    c.fE = reinterpret_cast<float *>(lds + cv.fE);
    c.fM = reinterpret_cast<float *>(lds + cv.fM);
    c.fZ = reinterpret_cast<int32_t *>(lds + cv.fZ);
    c.rank = reinterpret_cast<int *>(lds + cv.rank);
    c.zw = reinterpret_cast<uint16_t *>(lds + cv.zw);
    c.ztot = reinterpret_cast<int *>(lds + cv.ztot);
    c.pS1 = reinterpret_cast<int *>(lds + cv.pS1);
    c.pS2 = reinterpret_cast<unsigned long long *>(lds + cv.pS2);
    c.orow = reinterpret_cast<int32_t *>(lds + cv.ost);
    c.total = 0;
    c.stamp_clip = 0;
    return c;
}
template <bool FAST>
__device__ __forceinline__ Ctx make_ctx(const ExtractParams &p, unsigned char *lds)
{
    if constexpr (FAST) {
        constexpr ExtractCarve cv = extract_carve_fast();
        return ctx_from(cv, lds);
    } else {
        return ctx_from(p.cv, lds);
    }
}

// window (create_window, :278-296) -> LDS once as four shifted zero-padded fp32 copies, and its
// support [j0, j1] (sh->j0 / j1) by ballots: every weight read is issued before the first use, so
// the prologue costs one L2 round trip (windows longer than WPRE * NT loop over the rest).  Ends
// with a barrier.
__device__ __forceinline__ void build_window(const ExtractParams &p, const Ctx &c, int tid, int lane, int wid)
{
    float *wt = const_cast<float *>(c.wtab);  // 4 copies of wrow floats
    Shared *sh = c.sh;
    const int L = p.L;
    constexpr int WPRE = 3;
    double wv[WPRE];
#pragma unroll
    for (int k = 0; k < WPRE; k++) {
        const int j = tid + NT * k;
        wv[k] = j < L ? p.window[j] : 0.0;
    }
    if (tid == 0) {
        sh->j0 = L;
        sh->j1 = -1;
    }
    const int wrow = EXTRACT_WROW(L);
    for (int t = tid; t < 4 * (wrow - L); t += NT) {  // zero pads: m < WPAD + r, m >= L + WPAD + r
        const int r = t / (wrow - L), q = t - r * (wrow - L);
        wt[r * wrow + (q < EXTRACT_WPAD + r ? q : q + L)] = 0.f;
    }
    __syncthreads();
    auto put_weight = [&](int q0, double w) {  // weight j = q0 + lane (q0 wave-uniform)
        const int j = q0 + lane;
        const bool in = j < L;
        if (in) {
#pragma unroll
            for (int r = 0; r < 4; r++) wt[r * wrow + j + EXTRACT_WPAD + r] = (float)w;
        }
        const unsigned long long m = __ballot(in && w > 0.0);
        if (lane == 0 && m) {
            atomicMin(&sh->j0, q0 + __ffsll((long long)m) - 1);
            atomicMax(&sh->j1, q0 + 63 - __clzll((long long)m));
        }
    };
#pragma unroll
    for (int k = 0; k < WPRE; k++) put_weight(NT * k + wid * 64, wv[k]);
    for (int q0 = NT * WPRE + wid * 64; q0 < L; q0 += NT) put_weight(q0, q0 + lane < L ? p.window[q0 + lane] : 0.0);
    __syncthreads();
}


// the staged outputs of the chunk holding clip `done` (slots in sh->smask) to global memory: slot j
// is one 19-word row in LDS (feat[15], start, end, n_frames, status), written as whole rows -- one
// clip's 76 B written on its own reach HBM as ~190 B of partial sectors once L2 has evicted the
// lines between neighbouring clips' writes; with the packed row layout (ostride 19, ABI 6) a
// chunk's rows are one contiguous 304-B range
__device__ __forceinline__ void flush_outputs(const ExtractParams &p, const Ctx &c, int done, int tid)
{
    constexpr int CH = EXTRACT_OSTAGE, RW = DSP_OUT_ROW_WORDS;
    const int cb = done & ~(CH - 1);
    // nothing staged for this chunk (its clips were deferred or bad: written directly) -> 0
    const unsigned m = c.sh->schunk == cb / CH ? c.sh->smask : 0u;
    if (tid < RW * CH) {
        const int j = tid / RW, col = tid - RW * j;
        if ((m >> j) & 1) {
            const int32_t v = c.orow[tid];
            int32_t *dst = col < 15   ? (int32_t *)out_feat(p, cb + j) + col
                           : col < 17 ? out_se(p, cb + j) + (col - 15)
                           : col == 17 ? out_nf(p, cb + j)
                                       : out_st(p, cb + j);
            *dst = v;
        }
    }
}

// FAST launches run extract_kernel<true>, one clip at a time per workgroup (clip_fast).  A two-clip
// pipeline (the single-wave phases of one clip beside the multi-wave phases of the other, round 4)
// measured 3.41 against 3.35 ms: it added 10% VALU and 49% SALU instructions, and was removed
// (the A/B's raw record was not kept).

// registers: a 512-thread workgroup puts 2 waves on each SIMD, so W workgroups per CU allow
// 512 / (2 W) VGPRs -- FAST 80 (three per CU), generic 128 (two per CU)

// ---- one clip at a time per workgroup (both layouts) --------------------------------------------
// A near tie (an endpoint decision within the certification margin) leaves the clip with status
// DSP_CLIP_UNCERTIFIED; extract_exact_kernel, launched next on the stream, redoes it.
template <bool FAST>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2 * (FAST ? EXTRACT_WG_PER_CU : EXTRACT_WG_PER_CU_GENERIC))))
void extract_kernel(ExtractParams p)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    Ctx c = make_ctx<FAST>(p, lds);
    Shared *sh = c.sh;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    WG_STAMP(16);
    short8 regs[NRV];
    // FAST: the first clip (chunk blockIdx.x's first, or clip blockIdx.x in the static split: what
    // queue_next returns below) is loaded before the window is built, so that its loads and the
    // window's round trip overlap (1 000 clips: 0.0558 -> 0.0533 ms per step; 12.5k and 100k
    // unchanged; profiles/r05pre_ab_first_clip.txt)
    // FAST: a clip's loads are issued at the bottom of the previous trip (the first clip's here), on
    // every path -- a clip_none() range when there is no clip or a bad one, whose loads read zeros --
    // so the register array is never live across the loop's back edge (a path that skipped the issue
    // left it live around the whole loop: 84 VGPR spills)
    if constexpr (FAST) {
        const int b = (int)blockIdx.x, ch = max(p.qchunk, 1);
        const int first = (p.qchunk > 0 && p.queue) ? (b < (p.B + ch - 1) / ch ? b * ch : -1) : (b < p.B ? b : -1);
        const ClipRef c0 = first >= 0 ? clip_ref(p, first) : clip_none();
        issue_clip(regs, p, c0.ok ? c0 : clip_none(), opaque_tid());
    }
    build_window(p, c, tid, lane, wid);
    WG_CK(18);
    // (starting the second and third workgroup of each CU 2 or 5 us after the first, against the
    // lockstep start of round 5's stamps: 12.5k clips 0.405-0.415 against 0.400-0.403 ms per step,
    // 100k unchanged -- profiles/r06d_ab_stagger.txt; not kept)
    const ClipQueue Q = queue_open(p, sh);
    if (tid == 0) {
        sh->next = queue_next(Q, sh);
        sh->smask = 0;
        sh->schunk = -1;
        sh->sclear = 0;
        sh->noff_for = -1;
    }
    __syncthreads();
    WG_CK(19);
    bool inflight = false;  // generic kernel: regs already hold clip i's loads (issued during the previous clip's R5)
    for (int i = sh->next; i >= 0;) {
        STAMP(i, 20);
#ifdef DSP_STAMPS
        if (threadIdx.x == 0 && p.stamps) p.stamps[(size_t)i * 32 + 21] = blockIdx.x;  // the clip's workgroup
#endif
        const ClipRef cur = (FAST && sh->noff_for == i) ? clip_ref_at(p, sh->noff[0], sh->noff[1]) : clip_ref(p, i);
        if (!cur.ok) {
            __syncthreads();  // everyone has read sh->next (the ok path has barriers in its body)
            if (tid == 0) sh->next = queue_next(Q, sh);
            write_bad_clip(p, i, opaque_tid());
            inflight = false;
        } else {
            if (!FAST && !inflight) issue_clip(regs, p, cur, opaque_tid());
            unsigned cl = 0;
            if (tid == 0) cl = queue_begin(Q, sh);
            c.stamp_clip = i;
            bool done;
            if constexpr (FAST) {
                // resolves sh->next itself (before the crop), also for a deferred clip
                done = clip_fast(p, c, i, cur, regs, [&]() { return queue_end(Q, sh, cl); });
            } else {
                done = clip_body<false, false>(p, c, i, cur, regs, [&]() { return queue_end(Q, sh, cl); });
                if (!done && tid == 0) sh->next = queue_end(Q, sh, cl);  // a deferred clip returns before R4
            }
            if (!done && tid == 0) {
                *out_st(p, i) = DSP_CLIP_UNCERTIFIED;
                if (p.queue) __hip_atomic_fetch_add(qword(p.queue, 9), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            inflight = !FAST && done;
        }
        __syncthreads();  // LDS summaries are rewritten by the next clip; sh->next published
        STAMP(i, 14);
        const int prev = i;
        i = sh->next;
        if (i < 0 || (i ^ prev) >= EXTRACT_OSTAGE) {  // next clip in another chunk
            flush_outputs(p, c, prev, opaque_tid());  // (addresses computed here, not hoisted and spilled)
            if (tid == 0) sh->sclear = 1;
        }
        if constexpr (FAST) {  // the next clip's loads (see the prologue), from a wave-uniform range
            ClipRef nx = i < 0 ? clip_none() : sh->noff_for == i ? clip_ref_at(p, sh->noff[0], sh->noff[1]) : clip_ref(p, i);
            if (!nx.ok) nx = clip_none();
            nx.base = (int64_t)uni_u64((uint64_t)nx.base);  // (a per-lane value here made the compiler
            nx.nvec = uni(nx.nvec);                          // waterfall every load over the lanes)
            issue_clip(regs, p, nx, opaque_tid());
        }
        STAMP(prev, 15);
    }
    if (tid == 0) queue_done(p);
    WG_STAMP(22);
}

// Launched after extract_kernel on the same stream: every clip they left
// DSP_CLIP_UNCERTIFIED (rare) is redone from the start by one workgroup, on the bit-exact
// (numpy-order) energy path, and gets its final outputs and DSP_CLIP_FLAG_VAD_EXACT.  With the
// clip queue, extract_kernel counts its near ties in queue word 9: a launch with none returns at
// once (one load per workgroup); otherwise the last workgroup out zeroes words 9 and 10 again.
template <bool FAST>
__global__ __launch_bounds__(NT) void extract_exact_kernel(ExtractParams p)
{
    if (p.queue && __hip_atomic_load(qword(p.queue, 9), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    Ctx c = make_ctx<FAST>(p, lds);
    Shared *sh = c.sh;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // NT ints past the layout (the host launches this kernel with 4 NT more bytes of LDS)
    int *list = reinterpret_cast<int *>(lds + (FAST ? extract_carve_fast().total : p.cv.total));
    bool built = false;
    // the workgroup's clips blockIdx.x + G (t + NT k), NT statuses read at once, the near ties listed
    for (int64_t b0 = 0; b0 < p.B; b0 += (int64_t)gridDim.x * NT) {
        const int64_t i = b0 + blockIdx.x + (int64_t)gridDim.x * tid;
        const bool tie = i < p.B && *out_st(p, (int)i) == DSP_CLIP_UNCERTIFIED;
        if (tid == 0) sh->next = 0;
        __syncthreads();
        if (tie) list[atomicAdd(&sh->next, 1)] = (int)i;
        __syncthreads();
        const int nt = sh->next;
        for (int t = 0; t < nt; t++) {
            const int ci = list[t];
            if (!built) {
                build_window(p, c, tid, lane, wid);
                built = true;
            }
            c.stamp_clip = ci;
            const ClipRef cr = clip_ref(p, ci);
            short8 regs[NRV];
            issue_clip(regs, p, cr);
            clip_body<true, FAST>(p, c, ci, cr, regs);
            __syncthreads();
        }
    }
    if (p.queue && tid == 0) {  // every workgroup has read word 9 before its increment of word 10
        const unsigned d = __hip_atomic_fetch_add(qword(p.queue, 10), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (d == gridDim.x - 1) {
            __hip_atomic_store(qword(p.queue, 9), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(qword(p.queue, 10), 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace dsp

static void *g_stamp_buffer = nullptr;
#ifdef DSP_STAMPS
extern "C" int dsp_debug_set_stamp_buffer(void *buf)
{
    g_stamp_buffer = buf;
    return 0;
}
#endif

extern "C" size_t dsp_extract_lds_bytes(int64_t max_len, int frame_length, int frame_shift)
{
    if (max_len < 1 || frame_length < 1 || frame_shift < 1) return 0;
    if (max_len > (1 << 24) || frame_length > (1 << 20)) return 0;
    const ExtractCarve c = extract_carve((int)max_len, frame_length, frame_shift);
    // + the exact kernel's list of near ties (4 bytes per thread past the layout)
    return c.total + 4 * EXTRACT_THREADS <= EXTRACT_LDS_LIMIT ? (size_t)c.total : 0;
}

// CU count per device (the persistent grid), cached on first use of each device
static int g_num_cus[64];

extern "C" int dsp_extract_features(const int16_t *pcm, const int64_t *offsets, int B,
                                    int64_t max_len, int frame_length, int frame_shift,
                                    const double *window, int do_vad, double hi, double lo,
                                    double zr, float *feat, int32_t *start_end, int32_t *n_frames,
                                    int32_t *status, int out_stride, double *vad_energy, int32_t *vad_zcr,
                                    int ld_vad, float *seq, int ld_seq, void *queue_ws, void *stream)
{
    if (B < 0 || !offsets || !window || !feat || !start_end || !n_frames || !status)
        return DSP_ERR_ARGS;
    if (out_stride != 0 && out_stride < DSP_OUT_ROW_WORDS) return DSP_ERR_ARGS;
    if (frame_length < 1 || frame_shift < 1 || max_len < 1) return DSP_ERR_ARGS;
    if (((uintptr_t)pcm & 15) != 0 || ((uintptr_t)queue_ws & 3) != 0) return DSP_ERR_ARGS;
    if ((vad_energy == nullptr) != (vad_zcr == nullptr)) return DSP_ERR_ARGS;
    if (vad_energy && ld_vad < 1) return DSP_ERR_ARGS;
    if (seq && ld_seq < 1) return DSP_ERR_ARGS;
    if (B == 0) return DSP_OK;
    const size_t lds = dsp_extract_lds_bytes(max_len, frame_length, frame_shift);
    if (lds == 0) return DSP_ERR_TOO_LONG;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return DSP_ERR_HIP;
    if (g_num_cus[dev] == 0) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return DSP_ERR_HIP;
        g_num_cus[dev] = prop.multiProcessorCount;
        (void)hipFuncSetAttribute((const void *)dsp::extract_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, EXTRACT_LDS_LIMIT);
        (void)hipFuncSetAttribute((const void *)dsp::extract_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, EXTRACT_LDS_LIMIT);
        (void)hipFuncSetAttribute((const void *)dsp::extract_exact_kernel<true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, EXTRACT_LDS_LIMIT);
        (void)hipFuncSetAttribute((const void *)dsp::extract_exact_kernel<false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, EXTRACT_LDS_LIMIT);
    }
    const int num_cus = g_num_cus[dev];
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
    p.ostride = out_stride;
    p.vad_energy = vad_energy;
    p.vad_zcr = vad_zcr;
    p.ld_vad = ld_vad;
    p.seq = seq;
    p.ld_seq = ld_seq;
    p.stamps = (unsigned long long *)g_stamp_buffer;
    p.queue = (unsigned *)queue_ws;
    p.qchunk = 4;  // set below from the batch size
    p.cv = extract_carve((int)max_len, frame_length, frame_shift);
    // persistent grid: two workgroups per CU when their LDS fits (one otherwise), each walking
    // clip blockIdx first, then clips from the launch's queue; the compile-time layout whenever the
    // launch fits it
    const bool fast = extract_fast_fits((int)max_len, frame_length, frame_shift);
    const size_t lds_launch = fast ? (size_t)extract_carve_fast().total : lds;
    const int per_cu = std::max(1, std::min<int>(fast ? EXTRACT_WG_PER_CU : EXTRACT_WG_PER_CU_GENERIC,
                                                 (int)(EXTRACT_LDS_LIMIT / lds_launch)));
    const int slots = per_cu * num_cus;
    const int grid = B < slots ? B : slots;
    // short batches: a finer tail
    // up to 1.5 clips per workgroup the static split (the second clips start on no claim; 1 000
    // clips: 0.056 against 0.060 ms per step with 1-clip chunks), up to 2 claimed 1-clip chunks (the
    // workgroups done first take them; 1 500 clips: 0.075 against 0.081 ms static;
    // profiles/r05d1_ab_short.txt)
    p.qchunk = 2 * B <= 3 * (int64_t)grid ? 0 : B <= 2 * (int64_t)grid ? 1 : B < 64 * (int64_t)grid ? 2 : 4;
    static_assert(EXTRACT_OSTAGE >= 4, "qchunk <= EXTRACT_OSTAGE");
    const hipStream_t s = (hipStream_t)stream;
    // the near-tie redo: one workgroup per CU (near ties are rare; a launch without any returns at
    // once, and dispatching a third of the main grid makes that empty launch shorter)
    const int xgrid = std::min(grid, num_cus);
    if (fast) {
        hipLaunchKernelGGL(dsp::extract_kernel<true>, dim3(grid), dim3(dsp::NT), lds_launch, s, p);
        hipLaunchKernelGGL(dsp::extract_exact_kernel<true>, dim3(xgrid), dim3(dsp::NT), lds_launch + 4 * dsp::NT, s, p);
    } else {
        hipLaunchKernelGGL(dsp::extract_kernel<false>, dim3(grid), dim3(dsp::NT), lds_launch, s, p);
        hipLaunchKernelGGL(dsp::extract_exact_kernel<false>, dim3(xgrid), dim3(dsp::NT), lds_launch + 4 * dsp::NT, s, p);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DSP_OK : DSP_ERR_HIP + (int)e;
}
