// LDS carve-up of the extraction kernel (host and device agree on it).
//
// The clip itself is NOT in LDS: it is held in registers (EXTRACT_RREG 32-sample words per
// thread) for the two passes that need every sample, and re-read from L2 by the phases that need
// a few (crop frames, partial words at VAD frame edges).  LDS holds per-word summaries (positive-
// sample bits, exact moments, sign-change prefixes), the window table and the small per-frame arrays (~52 KB in the
// compile-time layout), so three workgroups share a CU.
#ifndef DSP_EXTRACT_LAYOUT_H
#define DSP_EXTRACT_LAYOUT_H

#ifndef EXTRACT_THREADS
#define EXTRACT_THREADS 512
#endif
#ifndef EXTRACT_RREG
#define EXTRACT_RREG 3                   // 32-sample words per thread held in registers
#endif
#ifndef EXTRACT_WG_PER_CU
#define EXTRACT_WG_PER_CU 3              // resident FAST workgroups per CU (80 VGPRs, <= 53 KB LDS each)
#endif
#ifndef EXTRACT_WG_PER_CU_GENERIC
#define EXTRACT_WG_PER_CU_GENERIC 2      // the generic layout's kernel (128 VGPRs)
#endif
#define EXTRACT_LDS_LIMIT (160 * 1024)   // one CU
#define EXTRACT_SHARED_BYTES 512         // sizeof(dsp::Shared) rounded up (static_assert'ed)
#ifndef EXTRACT_OSTAGE
#define EXTRACT_OSTAGE 4                 // clips per queue chunk, whose outputs are written together
#endif
#define EXTRACT_WPAD 8                   // zero window entries on each side of the window table
// floats per shifted window copy: copy r holds w[m - WPAD - r] at m (zero outside [0, L)), so
// that 4 consecutive weights starting at any window index are one aligned 16-B LDS read
#define EXTRACT_WROW(L) ((((L) + 2 * EXTRACT_WPAD + 4) + 3) & ~3)

struct ExtractCarve {
    int sh, wtab, posw, wS2, wS1, vE, vZ, fE, fM, fZ, rank, pS2, pS1, ost, total;
    int zw, ztot;  // FAST: sign-change counts, prefix within 64-word segments (u16) and segment totals
    int nvcap, fcap, nwmax;
};

// Region offsets from the capacities: nwmax 32-sample words (incl. the alignment lead), nvcap VAD
// frames, fcap feature frames, wrow floats per shifted window copy.
__host__ __device__ constexpr ExtractCarve extract_carve_caps(int nwmax, int nvcap, int fcap, int wrow,
                                                              bool rank = true)
{
    ExtractCarve c{};
    int o = 0;
#define DSP_TAKE(field, bytes)             \
    do {                                   \
        c.field = o;                       \
        o = (o + (int)(bytes) + 15) & ~15; \
    } while (0)
    c.nvcap = nvcap;
    c.fcap = fcap;
    c.nwmax = nwmax;
    DSP_TAKE(sh, EXTRACT_SHARED_BYTES);
    DSP_TAKE(wtab, 16 * wrow);                   // 4 zero-padded window copies, shifted by 0..3
    DSP_TAKE(posw, 4 * (c.nwmax + 2));           // positive-sample bits (+2 zero sentinels)
    DSP_TAKE(wS2, 8 * c.nwmax);                  // per word: sum k^2 (exact, u64)
    DSP_TAKE(wS1, 4 * c.nwmax);                  // per word: sum k
    DSP_TAKE(vE, 8 * c.nvcap);
    DSP_TAKE(vZ, 4 * c.nvcap);
    DSP_TAKE(fE, 4 * c.fcap);
    DSP_TAKE(fM, 4 * c.fcap);
    DSP_TAKE(fZ, 4 * c.fcap);
    DSP_TAKE(rank, rank ? 4 * (c.nvcap > 3 * c.fcap ? c.nvcap : 3 * c.fcap) : 0);  // long clips only
    DSP_TAKE(pS2, 16 * c.nvcap);  // partial-word moments at the two ends of each VAD frame
    DSP_TAKE(pS1, 8 * c.nvcap);
    DSP_TAKE(ost, 4 * 19 * EXTRACT_OSTAGE);  // staged outputs of one clip chunk (feat, start/end, frames, status)
    c.zw = c.ztot = o;  // FAST layout only
#undef DSP_TAKE
    c.total = o;
    return c;
}

// ncap = longest clip of the launch (samples)
__host__ __device__ inline ExtractCarve extract_carve(int ncap, int L, int S)
{
    const int nvcap = ncap >= L ? (ncap - L) / S + 1 : 0;
    const int fcap = ncap <= L ? 1 : (ncap - L + S - 1) / S + 1;
    const int nwmax = (ncap + 7 + 31) / 32 + 1;
    return extract_carve_caps(nwmax, nvcap, fcap, EXTRACT_WROW(L));
}

// The fast kernel's layout is fixed at compile time (every LDS address an immediate) and serves
// every launch whose clips fit it: the whole clip in registers, <= 128 VAD and feature frames,
// window rows of <= EXTRACT_FAST_WROW floats (frame_length <= 1256).
#define EXTRACT_FAST_NV 128
#define EXTRACT_FAST_NF 128
#ifndef EXTRACT_FAST_WROW
#define EXTRACT_FAST_WROW 1280
#endif
#define EXTRACT_FAST_NWORD (EXTRACT_THREADS * EXTRACT_RREG)
__host__ __device__ constexpr ExtractCarve extract_carve_fast()
{
    ExtractCarve c{};
    int o = 0;
#define DSP_TAKE(field, bytes)             \
    do {                                   \
        c.field = o;                       \
        o = (o + (int)(bytes) + 15) & ~15; \
    } while (0)
    c.nvcap = EXTRACT_FAST_NV;
    c.fcap = EXTRACT_FAST_NF;
    c.nwmax = EXTRACT_FAST_NWORD + 1;
    DSP_TAKE(sh, EXTRACT_SHARED_BYTES);
    DSP_TAKE(wtab, 16 * EXTRACT_FAST_WROW);
    DSP_TAKE(posw, 4 * (c.nwmax + 2));
    DSP_TAKE(wS2, 8 * c.nwmax);
    DSP_TAKE(wS1, 4 * c.nwmax);
    DSP_TAKE(vE, 8 * c.nvcap);
    DSP_TAKE(vZ, 4 * c.nvcap);
    DSP_TAKE(fE, 4 * c.fcap);
    DSP_TAKE(fM, 4 * c.fcap);
    DSP_TAKE(fZ, 4 * c.fcap);
    DSP_TAKE(ost, 4 * 19 * EXTRACT_OSTAGE);
    DSP_TAKE(zw, 2 * (c.nwmax + 2));           // per word: sign changes before it in its 64-word segment
    DSP_TAKE(ztot, 4 * (EXTRACT_FAST_NWORD / 64 + 1));  // per segment: its sign changes (last boundary excluded)
    c.rank = c.pS1 = c.pS2 = o;  // unused by the FAST layout (<= 128 frames; pass A sums in registers)
#undef DSP_TAKE
    c.total = o;
    return c;
}
static_assert(EXTRACT_WG_PER_CU * extract_carve_fast().total <= EXTRACT_LDS_LIMIT,
              "the FAST layout must fit EXTRACT_WG_PER_CU workgroups per CU");
__host__ __device__ inline bool extract_fast_fits(int ncap, int L, int S)
{
    const ExtractCarve c = extract_carve(ncap, L, S);
    return (ncap + 7 + 31) / 32 <= EXTRACT_FAST_NWORD && c.nvcap <= EXTRACT_FAST_NV &&
           c.fcap <= EXTRACT_FAST_NF && EXTRACT_WROW(L) <= EXTRACT_FAST_WROW;
}

#endif
