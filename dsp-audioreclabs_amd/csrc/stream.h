// stream.h -- host interface of the two-kernel extraction path (stream.hip), used by the C ABI
// entry point dsp_extract_features (extract.hip).
#ifndef DSP_STREAM_H
#define DSP_STREAM_H
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#define STREAM_WPAD 32    // zero weights on each side of a window copy (a word may start 32 before it)
#define STREAM_WROWF 1344 // floats per shifted window copy: frame_length <= 1276
#define STREAM_PQ 11      // 128-sample quads one frame may overlap: frame_length <= 1281
#define STREAM_FCAP 128   // endpoint / windowed frames per clip (one wave holds two per lane)

// per-clip frame summary written by frame_kernel, read by decide_kernel (byte offsets):
//   [0] mq f64, [8] M' f64, vE f64[nv], fE f32[F], fM f32[F], vZ u16[nv], fZ u16[F]
struct RecLayout {
    int vE, fE, fM, vZ, fZ, stride;
};

bool dsp_stream_fits(int64_t max_len, int frame_length, int frame_shift);
RecLayout dsp_stream_layout(int64_t max_len, int frame_length, int frame_shift);
size_t dsp_stream_lds_bytes();
int dsp_stream_launch(const int16_t *pcm, const int64_t *offsets, int B, int64_t max_len, int L, int S,
                      const double *window, int do_vad, double hi, double lo, double zr, float *feat,
                      int32_t *start_end, int32_t *n_frames, int32_t *status, double *vad_energy,
                      int32_t *vad_zcr, int ld_vad, float *seq, int ld_seq, void *workspace,
                      size_t workspace_bytes, int num_cus, hipStream_t stream);
#endif
