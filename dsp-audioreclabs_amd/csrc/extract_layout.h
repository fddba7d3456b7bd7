// extract_layout.h -- LDS carve-up of the fused extraction kernel, shared by host and device.
#ifndef DSP_EXTRACT_LAYOUT_H
#define DSP_EXTRACT_LAYOUT_H

#include <hip/hip_runtime.h>

#define EXTRACT_THREADS 512
#define EXTRACT_LDS_LIMIT (160 * 1024)
#define EXTRACT_MAX_ROUNDS 20   // 16-B loads per thread: clips up to 8*20*512-16 samples
#define EXTRACT_PREFETCH 12     // of which prefetched into registers (clips <= 49136 samples)
#define EXTRACT_DEFER_CAP 512   // near-tie clips one workgroup can redo exactly
#define EXTRACT_SHARED_BYTES 512  // sizeof(dsp::Shared) rounded up (static_assert'ed)

struct ExtractCarve {
    int sh, clip, wtab, chg, seg, vE, vZ, fE, fM, fZ, defer, total;
    int nvcap, fcap, nvecmax, nseg;
};

// ncap: longest clip (samples); L, S: frame length / shift (samples);
// per_wg: clips one persistent workgroup walks (sizes the deferred-clip list)
__host__ __device__ inline ExtractCarve extract_carve(int ncap, int L, int S, int per_wg)
{
    ExtractCarve c;
    int o = 0;
#define DSP_TAKE(field, bytes)             \
    do {                                   \
        c.field = o;                       \
        o = (o + (int)(bytes) + 15) & ~15; \
    } while (0)
    c.nvcap = ncap >= L ? (ncap - L) / S + 1 : 0;
    c.fcap = ncap <= L ? 1 : (ncap - L + S - 1) / S + 1;
    c.nvecmax = (ncap + 7 + 7) / 8 + 1;     // 16-B vectors incl. alignment lead
    c.nseg = 2 * (c.nvcap + L / S + 1);     // hop segments [qS, qS+r), [qS+r, (q+1)S)
    DSP_TAKE(sh, EXTRACT_SHARED_BYTES);
    DSP_TAKE(clip, 16 * c.nvecmax + 32);    // int16, buffer coordinates (lead <= 7)
    DSP_TAKE(wtab, 8 * L);                  // (window, window^2) pairs
    DSP_TAKE(chg, c.nvecmax + 16);          // positive bits, then sign-change bits (in place)
    DSP_TAKE(seg, 16 * c.nseg);             // per segment: sum k^2 (u64), sum k, sign changes
    DSP_TAKE(vE, 8 * c.nvcap);
    DSP_TAKE(vZ, 4 * c.nvcap);
    DSP_TAKE(fE, 4 * c.fcap);
    DSP_TAKE(fM, 4 * c.fcap);
    DSP_TAKE(fZ, 4 * c.fcap);
    DSP_TAKE(defer, 4 * per_wg);
#undef DSP_TAKE
    c.total = o;
    return c;
}

#endif
