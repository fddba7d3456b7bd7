/* oracle/dsp_oracle.h -- CPU restatement of the reference hot path.
 * TEST INFRASTRUCTURE ONLY (see dsp_oracle.c header). */
#ifndef DSP_ORACLE_H
#define DSP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORA_OK = 0,
    ORA_ERR_EMPTY = 1,     /* zero-length clip: np.max of empty array raises */
    ORA_ERR_NO_AUDIO = 2,  /* "No audio remaining after ..." (src/audio_processing.py:388-389) */
    ORA_ERR_NO_FRAMES = 3, /* "No frames provided ..." (src/feature_extraction.py:27-28) */
    ORA_ERR_ARGS = 5
};

double ora_np_sum(const double *a, int64_t n);
void ora_compute_statistics(const double *seq, int64_t n, double out[5]);
int ora_preprocess(const double *x, int64_t n, double *out);
double ora_short_time_energy(const double *frame, int64_t L, double *scratch);
double ora_short_time_magnitude(const double *frame, int64_t L, double *scratch);
double ora_zero_crossing_rate(const double *frame, int64_t L);
int64_t ora_vad_frame_count(int64_t n, int64_t L, int64_t S);
int64_t ora_endpoint_detection(const double *x, int64_t n, int64_t L, int64_t S, double hi,
                               double lo, double zr, int64_t *start, int64_t *end, double *E,
                               double *Z);
int64_t ora_frame_count(int64_t n, int64_t L, int64_t S);
int64_t ora_frame_features(const double *x, int64_t n, int64_t L, int64_t S, const double *window,
                           double *E, double *M, double *Z);
int ora_process_pcm_i16(const int16_t *pcm, int64_t n, int64_t L, int64_t S, const double *window,
                        int do_vad, double hi, double lo, double zr, double *feat15,
                        int64_t *start_end, int64_t *n_frames, double *vad_e, double *vad_z,
                        int64_t *n_vad, double *seq, int64_t seq_cap);
int ora_process_f64(const double *audio, int64_t n, int64_t L, int64_t S, const double *window,
                    int do_vad, double hi, double lo, double zr, double *feat15,
                    int64_t *start_end, int64_t *n_frames, double *vad_e, double *vad_z,
                    int64_t *n_vad, double *seq, int64_t seq_cap);
int ora_process_batch_i16(const int16_t *pcm, const int64_t *offsets, int64_t B, int64_t L,
                          int64_t S, const double *window, int do_vad, double hi, double lo,
                          double zr, double *feat, int64_t *start_end, int64_t *n_frames,
                          int32_t *status, int nthreads);
void ora_zscore_fit(const double *X, int64_t n, int d, double *mean, double *std);
void ora_knn(const double *ref, const int32_t *ref_lbl, int64_t Nr, const double *q, int64_t Nq,
             int D, int k, int64_t self_offset, int n_classes, int32_t *idx, double *dist,
             int32_t *pred);

#ifdef __cplusplus
}
#endif
#endif
