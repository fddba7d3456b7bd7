// extract_layout.h -- LDS carve-up of the fused extraction kernel, shared by host and device.
#ifndef DSP_EXTRACT_LAYOUT_H
#define DSP_EXTRACT_LAYOUT_H

#include <hip/hip_runtime.h>

#define EXTRACT_THREADS 1024
#define EXTRACT_LDS_LIMIT (160 * 1024)
#define EXTRACT_SHARED_BYTES 640  // sizeof(dsp::Shared) rounded up (static_assert'ed in the kernel)

struct ExtractCarve {
    int sh, clip, win, chg, pref, seg1, seg2, vE, vZ, vS, fE, fM, fZ, total;
    int nvcap, fcap, nseg, nwords;
};

// ncap: longest clip (samples); L, S: frame length / shift (samples)
__host__ __device__ inline ExtractCarve extract_carve(int ncap, int L, int S)
{
    ExtractCarve c;
    int o = 0;
#define DSP_TAKE(field, bytes)                          \
    do {                                                \
        c.field = o;                                    \
        o = (o + (int)(bytes) + 15) & ~15;              \
    } while (0)
    c.nvcap = ncap >= L ? (ncap - L) / S + 1 : 0;
    c.fcap = ncap <= L ? 1 : (ncap - L + S - 1) / S + 1;
    c.nseg = 2 * (c.nvcap + L / S + 1);
    c.nwords = (ncap + 31) / 32 + 2;
    DSP_TAKE(sh, EXTRACT_SHARED_BYTES);
    DSP_TAKE(clip, 2 * (ncap + 32));   // <= 7 samples of alignment lead + vector overrun
    DSP_TAKE(win, 4 * L);
    DSP_TAKE(chg, 4 * c.nwords);
    DSP_TAKE(pref, 4 * (c.nwords + 1));
    DSP_TAKE(seg1, 8 * c.nseg);
    DSP_TAKE(seg2, 8 * c.nseg);
    DSP_TAKE(vE, 8 * c.nvcap);
    DSP_TAKE(vZ, 4 * c.nvcap);
    DSP_TAKE(vS, 8 * c.nvcap);
    DSP_TAKE(fE, 4 * c.fcap);
    DSP_TAKE(fM, 4 * c.fcap);
    DSP_TAKE(fZ, 4 * c.fcap);
#undef DSP_TAKE
    c.total = o;
    return c;
}

#endif
