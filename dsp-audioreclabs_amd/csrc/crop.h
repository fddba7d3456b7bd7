// crop.h -- the canonical order of the crop frames' windowed sums E and M, shared by the fused
// extraction kernels (csrc/extract.hip, on the matrix cores) and the general kernel
// (csrc/general.hip, its scalar restatement): a clip's features have the same bits whichever kernel
// ran it and wherever it sits in the packed buffer.
#ifndef DSP_CROP_H
#define DSP_CROP_H
#include "dsp_device.h"

namespace dsp {
// ---- crop frames as a blocked product (round 7 canonical order of E and M; both kernels) --------
// The crop [st, en) is cut into blocks of S samples: block b = crop samples [bS, bS + S).  Frame g
// (crop samples [gS, gS + L), zero past en) is the sum over d < D = ceil(L / S) of block g + d
// against window entries [dS, dS + S) (zero at j >= L): a [blocks x S] x [S x D] product, which one
// v_mfma_f32_4x4x1f32 computes 16 units at a time (a unit = 4 weight rows x 4 data columns):
//   * sample value at crop position a < en - st: x = canon_xval(k) (above), else 0 (the padding);
//     E operands w2_j = fl(w_j * w_j) (from the double window) and fl(x * x); M operands |w_j| and |x|
//   * blocks in quads (columns c of quad q: block 4q + c); the S positions of a block in P parts of
//     T steps (part p: positions pT + s, s < T, none past S); unit u = q P + p; NG = ceil(D / 4)
//     groups of 4 weight rows (row d = 4 g + v)
//   * the unit partial of row d, column c: two chains over its steps (even s, odd s), each a
//     sequential fp32 fma from +0 (one MFMA step is fmaf: tools/ubench/mfma4x4.hip), then
//     chain0 + chain1
//   * frame g: for d = 0..D-1, for p = 0..P-1: acc += partial(q = (g+d)/4, p; row d, column
//     (g+d)%4), fp32 from +0; times invMf^2 (E) or invMf (M)
// P depends only on the quad and row-group counts (CROP_SLOTS units of work): every kernel, every
// clip position and every launch shape sums a frame's terms in this one order.
constexpr int CROP_SLOTS = 128;
struct CropPlan {
    int D, NG, nb, nq, P, T;
};
__host__ __device__ inline CropPlan crop_plan(int F, int L, int S)
{
    CropPlan c;
    c.D = (L + S - 1) / S;
    c.NG = (c.D + 3) >> 2;
    c.nb = F + c.D - 1;
    c.nq = (c.nb + 3) >> 2;
    const int per = c.nq * c.NG, pm = per >= CROP_SLOTS ? 1 : CROP_SLOTS / per;
    c.T = (S + pm - 1) / pm;
    c.P = (S + c.T - 1) / c.T;
    return c;
}
// index of a unit partial in a parts array (quantity Q: 0 E, 1 M; units * NG * 16 floats each)
__host__ __device__ inline int crop_part_index(const CropPlan &c, int Q, int u, int g, int col, int v)
{
    return Q * (c.nq * c.P * c.NG * 16) + ((u * c.NG + g) * 4 + col) * 4 + v;
}
#pragma clang fp contract(off)
// frame g's sum of quantity Q from the unit partials (the canonical order above)
__device__ __forceinline__ float crop_frame_sum(const float *parts, const CropPlan &c, int g, int Q)
{
    float acc = 0.f;
    for (int d = 0; d < c.D; d++) {
        const int b = g + d;
        const float *pp = parts + crop_part_index(c, Q, (b >> 2) * c.P, d >> 2, b & 3, d & 3);
        for (int p = 0; p < c.P; p++) acc += pp[p * c.NG * 16];
    }
    return acc;
}
#pragma clang fp contract(on)

}  // namespace dsp
#endif
