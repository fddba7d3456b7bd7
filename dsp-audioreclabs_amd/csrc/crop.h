// crop.h -- the canonical order of the crop frames' windowed sums E and M, shared by the fused
// extraction kernels (csrc/extract.hip, on the matrix cores) and the general kernel
// (csrc/general.hip, its scalar restatement): a clip's features have the same bits whichever kernel
// ran it and wherever it sits in the packed buffer.
//
// The crop [st, en) is cut into blocks of S samples: block b = crop samples [bS, bS + S).  Frame g
// (crop samples [gS, gS + L), zero past en) is the sum over d < D = ceil(L / S) of block g + d
// against window entries [dS, dS + S) (zero at j >= L): a [blocks x S] x [S x D] product, which one
// v_mfma_f32_4x4x1f32 computes 16 units at a time (a unit: 4 weight rows x 4 data columns):
//   * sample value at crop position a < en - st: x = canon_xval(k) (dsp_device.h), else 0 (the
//     padding); E operands w2_j = fl(w_j * w_j) (from the double window) and fl(x * x); M operands
//     |w_j| and |x|
//   * blocks in quads (columns c of quad q: block 4q + c); the S positions of a block in P parts of
//     T steps (part p: positions pT + s, s < T, none past S); unit u = q P + p; NG = ceil(D / 4)
//     groups of 4 weight rows (row d = 4 g + v)
//   * the unit partial of row d, column c: two chains over its steps (even s, odd s), each a
//     sequential fp32 fma from +0 (one MFMA step is fmaf: tools/ubench/mfma4x4.hip), then
//     chain0 + chain1
//   * B(b, d) = the pairwise tree over the P parts of block b's partials of row d
//     (((t0 + t1) + (t2 + t3)) + ...; P is a power of two <= 16: an xor butterfly across lanes)
//   * frame g: acc = +0; for d = 0..D-1: acc += B(g + d, d); times invMf^2 (E) or invMf (M)
// P depends only on the quad and row-group counts: every kernel, clip position and launch shape
// sums a frame's terms in this one order.
#ifndef DSP_CROP_H
#define DSP_CROP_H
#include "dsp_device.h"

namespace dsp {

constexpr int CROP_SLOTS = 128;  // units per row group the fused kernel's 8 waves take at once
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
    const int per = c.nq * c.NG;
    int P = 1;
    while (P < 16 && 2 * P * per <= CROP_SLOTS) P *= 2;
    c.P = P;
    c.T = (S + P - 1) / P;
    return c;
}
// index of a unit partial (quantity Q: 0 E, 1 M; unit u, row group g, column col, row 4 g + v) in a
// parts array of 2 * units * NG * 16 floats; B(b, d) is stored over the partial of unit (b / 4) P
// (part 0) of column b % 4 and row d
__host__ __device__ inline int crop_part_index(const CropPlan &c, int Q, int u, int g, int col, int v)
{
    return Q * (c.nq * c.P * c.NG * 16) + ((u * c.NG + g) * 4 + col) * 4 + v;
}
__host__ __device__ inline int crop_bsum_index(const CropPlan &c, int Q, int b, int d)
{
    return crop_part_index(c, Q, (b >> 2) * c.P, d >> 2, b & 3, d & 3);
}
// frame g's sum of quantity Q from the block sums (the canonical order above)
__device__ __forceinline__ float crop_frame_sum(const float *parts, const CropPlan &c, int g, int Q)
{
    float acc = 0.f;
    for (int d = 0; d < c.D; d++) acc += parts[crop_bsum_index(c, Q, g + d, d)];
    return acc;
}
// the pairwise tree of crop.h over the P <= 16 parts get(0 .. P-1), in halves of 8 (parts past P are
// +0: adding them changes nothing)
template <typename Get>
__device__ __forceinline__ float crop_tree(Get get, int P)
{
    auto tree8 = [&](int o) {
        float a[8];
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = o + i < P ? get(o + i) : 0.f;
#pragma unroll
        for (int w = 1; w < 8; w *= 2)
            if (w < P)
#pragma unroll
                for (int i = 0; i < 8; i += 2 * w) a[i] += a[i + w];
        return a[0];
    };
    const float lo = tree8(0);
    return P > 8 ? lo + tree8(8) : lo;
}

}  // namespace dsp
#endif
