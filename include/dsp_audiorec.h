/*
 * dsp_audiorec.h -- C ABI of the MI355X (gfx950) feature-extraction + KNN path.
 *
 * Drop-in boundary for the reference's hot path (Hypersonic-cpu/DSP-AudioRecLabs):
 * every entry point names the reference function(s) it replaces.  The reference is
 * pure Python, so its "FFI" is the Python module surface src/audio_processing.py,
 * src/feature_extraction.py and src/models.py; the host mirror of that surface
 * (dsp-audioreclabs_amd/src/) binds this header with ctypes.
 *
 * Conventions
 *  - All pointers are DEVICE pointers unless stated; buffers are caller-allocated.
 *  - Every launch is stream-ordered on `stream` (a hipStream_t passed as void*;
 *    NULL = the legacy default stream).  No entry point allocates, frees, copies
 *    to the host or synchronises, so all of them may be captured in a hipGraph.
 *  - Scratch buffers (workspace, queue_ws) belong to one launch at a time, like any
 *    scratch: launches that may run concurrently (other streams, other instances of a
 *    captured graph) need their own.  No entry point keeps state between launches.
 *  - Return value: 0 on success, a DSP_ERR_* code (argument checks, done on the
 *    host before launching), or DSP_ERR_HIP + hipError_t when a launch fails.
 *  - Per-item failures (the reference raises ValueError and its callers skip the
 *    file, experiments/run_experiments.py:109-111) are reported in `status[b]`.
 */
#ifndef DSP_AUDIOREC_H
#define DSP_AUDIOREC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSP_ABI_VERSION 6  /* 2: dsp_extract_features takes the clip-queue scratch (queue_ws);
                              3: queue_ws is 64 bytes (per-XCD chunk counters);
                              4: the batch WAV reader (dsp_wav_scan / dsp_wav_read);
                              5: queue_ws is 4 KiB (each counter on its own 256-B line);
                              6: the extraction entry points take out_stride (packed result rows);
                                 dsp_knn_classify takes flags (DSP_KNN_REF_READY) */

/* return codes */
#define DSP_OK 0
#define DSP_ERR_ARGS 1        /* bad sizes / null pointers / misaligned buffers */
#define DSP_ERR_TOO_LONG 2    /* a clip does not fit the on-chip (LDS) pipeline */
#define DSP_ERR_WORKSPACE 3   /* workspace too small */
#define DSP_ERR_HIP 1000      /* + hipError_t of the failed launch */

#define DSP_QUEUE_WS_BYTES 4096  /* dsp_extract_features' queue_ws */
#define DSP_OUT_ROW_WORDS 19     /* one clip's results as a packed row of 4-byte words: feat[15] (f32),
                                    start, end, n_frames, status (int32) -- 76 B */

/* per-clip status[b] (low byte) -- same codes as the oracle */
#define DSP_CLIP_OK 0
#define DSP_CLIP_EMPTY 1      /* zero-length clip: np.max of an empty array raises (audio_processing.py:72) */
#define DSP_CLIP_NO_AUDIO 2   /* "No audio remaining ..." (audio_processing.py:388-389) */
#define DSP_CLIP_NO_FRAMES 3  /* "No frames provided ..." (feature_extraction.py:27-28) */
#define DSP_CLIP_TOO_LONG 4   /* longer than the max_len given at launch (dsp_extract_general
                                 processes such clips) */
#define DSP_CLIP_UNCERTIFIED 5 /* internal, never left in status on return of the stream:
                                  the fused kernel marks a clip whose endpoint decision is a
                                  near tie (within the 1e-11 certification margin) with it, and
                                  the exact kernel that dsp_extract_features launches next on
                                  the same stream redoes every such clip on the bit-exact path */
/* status[b] flag bits (informational) */
#define DSP_CLIP_FLAG_VAD_EXACT 0x100 /* endpoint decision was a near tie: re-decided on the
                                         bit-exact (numpy-order) fp64 path */

/* Bytes of dynamic LDS dsp_extract_features needs for clips of up to max_len samples
 * (0 if it exceeds the 160 KiB of one CU). Host-only helper. */
size_t dsp_extract_lds_bytes(int64_t max_len, int frame_length, int frame_shift);

/*
 * dsp_extract_features -- fused per-clip pipeline: persistent workgroups (three per CU on the
 * compile-time layout), each taking one clip at a time -- its first clip by its own index, the
 * rest from a clip queue -- with the clip held in registers until its endpoints are decided and
 * the crop's frames re-read from L2.  A second launch on the same stream redoes near-tie endpoint
 * decisions on the bit-exact path (it returns at once when the first counted none in queue_ws).
 * Replaces, per clip, the chain
 *   preprocess            src/audio_processing.py:78-90   (remove_dc :49-59, normalize_audio :62-75)
 *   endpoint_detection    src/audio_processing.py:135-275 (when do_vad != 0)
 *   crop                  src/audio_processing.py:378
 *   frame_signal          src/audio_processing.py:299-333 (with create_window :278-296 supplied as `window`)
 *   extract_frame_features src/feature_extraction.py:12-43
 *   extract_statistical_features src/feature_extraction.py:65-88  (15-d vector)
 * as called per file by experiments/run_experiments.py:90-104.
 *
 * pcm       int16 samples of all clips back to back; clip b = pcm[offsets[b] .. offsets[b+1]).
 *           16-bit PCM as read by load_wav (:35-38); 8-bit PCM is passed as ((u8 - 128) mod 256),
 *           which is what load_wav's uint8 arithmetic computes (:31-34) -- any power-of-two
 *           scale cancels in preprocess.  `pcm` must be 16-byte aligned.
 * offsets   int64 [B+1], non-decreasing.
 * window    float64 [frame_length] = create_window(window_type, frame_length) (np.hamming etc.),
 *           zero only at its ends (true for the three reference windows).
 * hi/lo/zr  energy_high_ratio, energy_low_ratio, zcr_threshold_ratio (config.py:43-45).
 * max_len   longest clip in the batch (sizes the LDS carve-up; see dsp_extract_lds_bytes).
 * feat      float32 [B,15]: energy, magnitude, zcr x (mean, std, max, min, median).
 * start_end int32 [B,2]: start_point / end_point (0, len when do_vad == 0).
 * n_frames  int32 [B]: metadata['n_frames'] (frames after the crop).
 * status    int32 [B]: DSP_CLIP_* | flags.
 * out_stride 0: the four arrays above, each row-major as given.  >= DSP_OUT_ROW_WORDS: row b of
 *           each output starts b * out_stride 4-byte words after its pointer -- one packed row
 *           buffer rows[B][19] is feat = rows, start_end = rows + 15, n_frames = rows + 17, status
 *           = rows + 18, out_stride = 19: each clip's 76-B record is contiguous, so the per-clip
 *           results of a shard travel in one collective without packing.
 * vad_energy/vad_zcr (optional, may be NULL): float64 / int32 [B, ld_vad]: metadata energy_list,
 *           zcr_list (first (len-L)//S+1 entries; rows of clips with len < L are untouched).
 * seq       (optional, may be NULL): float32 [B, ld_seq, 3] per-frame (E, M, ZCR) -- the
 *           'sequence' method of extract_features_from_frames (:114-129); frames beyond
 *           ld_seq are dropped.
 * queue_ws  (optional, may be NULL): DSP_QUEUE_WS_BYTES (4096) bytes of device scratch, zero
 *           before the launch: the counters of the dynamic clip queue (persistent workgroups
 *           claim chunks of consecutive clips, from their own XCD's share first, so fast
 *           workgroups take more clips); the launch leaves it zero again, so it can be reused by
 *           the next launch on the same stream.  NULL: a static round-robin split of the clips
 *           over the workgroups (same results, slower).
 *           One launch at a time per queue_ws (see Conventions).
 */
int dsp_extract_features(const int16_t *pcm, const int64_t *offsets, int B, int64_t max_len,
                         int frame_length, int frame_shift, const double *window, int do_vad,
                         double hi, double lo, double zr, float *feat, int32_t *start_end,
                         int32_t *n_frames, int32_t *status, int out_stride, double *vad_energy,
                         int32_t *vad_zcr, int ld_vad, float *seq, int ld_seq, void *queue_ws,
                         void *stream);

/*
 * dsp_extract_general -- the same pipeline for clips outside the fused kernel's on-chip plan:
 * any length (process_audio_file has no limit, src/audio_processing.py:336-396) and samples
 * wider than int16: 16-bit stereo, whose exact sample is the sum of the two channels (load_wav
 * averages them, :35-44; the power-of-two scale cancels in preprocess).  One workgroup per clip
 * from global memory; results identical to dsp_extract_features' where both apply.
 *
 * pcm          int16 (sample_bytes 2) or int32 (sample_bytes 4) samples, clips at offsets[b].
 * clip_index   int32 [nclip] clip numbers b to process (device; NULL: b = 0 .. nclip-1).  Only
 *              clips with min_len < len <= max_len are processed (min_len = 0: every clip,
 *              empty ones reported DSP_CLIP_EMPTY and ones longer than max_len
 *              DSP_CLIP_TOO_LONG); with min_len > 0 the outputs of the others are untouched, so
 *              a batch can be split between the two entry points without a host round trip.
 * outputs      as dsp_extract_features, indexed by clip number b.
 * workspace    device scratch of dsp_extract_general_workspace_bytes(nclip, max_len, L, S).
 */
size_t dsp_extract_general_workspace_bytes(int64_t nclip, int64_t max_len, int frame_length,
                                           int frame_shift);
int dsp_extract_general(const void *pcm, int sample_bytes, const int64_t *offsets,
                        const int32_t *clip_index, int nclip, int64_t min_len, int64_t max_len,
                        int frame_length, int frame_shift, const double *window, int do_vad,
                        double hi, double lo, double zr, float *feat, int32_t *start_end,
                        int32_t *n_frames, int32_t *status, int out_stride, double *vad_energy,
                        int32_t *vad_zcr, int ld_vad, float *seq, int ld_seq, void *workspace,
                        size_t workspace_bytes, void *stream);

/*
 * KNN -- KNeighborsClassifier(n_neighbors=k) as configured in src/models.py:33-35 and used by
 * TraditionalClassifier.fit/predict (:52-58): exact Euclidean k nearest neighbours of each query
 * row among the reference rows, ascending distance, then a uniform majority vote in which the
 * smallest label wins ties (scipy.stats.mode).  Screening runs in fp32: for D < 16 / D < 32
 * (the 15-d features) in the expanded form |q|^2 + q'.r' on the matrix cores
 * (v_mfma_f32_16x16x4_f32, f32 in / f32 accumulate -- a deliberate departure from north_star's
 * "no MFMA", measured 6.9 -> 5.7 ms at 100k x 100k), for D = 16 / 32 in the
 * direct form (q - r)^2 on the VALU, for D > 32 in the direct form in chunks of 16.  The screen
 * only nominates candidates: its error bound (knn.hip knn_err_coeffs) holds for any summation
 * order inside an MFMA with at most one rounding per product and per addition, so the
 * certification below does not rest on the matrix core matching an fmaf chain bit for bit.
 * Survivors are re-ranked with the reference's own fp64 distance (sequential sum of squared
 * differences, no FMA, sqrt), and any query whose fp32 screen cannot certify the fp64 top-k is
 * re-solved exhaustively in fp64 on the device.  Exact-distance ties are ordered by smaller
 * reference index.
 *
 * ref        float64 [Nr, D] row-major,  ref_labels int32 [Nr] in [0, n_classes)
 * query      float64 [Nq, D] row-major
 * self_offset  >= 0: query q is reference row self_offset + q and is excluded from its own
 *              neighbour list (kneighbors(X=None) semantics); -1: no exclusion.
 * idx        int32 [Nq, k] (-1 where fewer than k candidates), dist float64 [Nq, k],
 * pred       int32 [Nq] (may be NULL, or ref_labels NULL, to skip the vote)
 * workspace  device scratch of dsp_knn_workspace_bytes(Nr, Nq, D, k) bytes.  Its first part holds
 *            the reference set converted for the screen, at offsets that depend on (Nr, D) only.
 * flags      DSP_KNN_REF_READY: the workspace already holds that conversion, left by an earlier call
 *            with the same ref, Nr, D and k on the same stream (any Nq): the conversion -- the
 *            fit() side of KNeighborsClassifier, src/models.py:52-55 -- is skipped.  0: convert.
 * Requires 1 <= D <= 4096, 1 <= k <= 32.  D <= 32: queries in registers, reference tiles in LDS;
 * D > 32 (the sequence method's flattened features): dimensions walked in chunks of 16.
 */
#define DSP_KNN_REF_READY 1
size_t dsp_knn_workspace_bytes(int64_t Nr, int64_t Nq, int D, int k);
/* Diagnostic: byte offset in that workspace of an int32 that dsp_knn_classify leaves holding the
 * number of queries the screen could not certify (answered by the exhaustive fp64 fallback). */
size_t dsp_knn_workspace_fallbacks_offset(int64_t Nr, int64_t Nq, int D, int k);
int dsp_knn_classify(const double *ref, const int32_t *ref_labels, int64_t Nr, const double *query,
                     int64_t Nq, int D, int k, int64_t self_offset, int n_classes, int32_t *idx,
                     double *dist, int32_t *pred, void *workspace, size_t workspace_bytes, int flags,
                     void *stream);

/*
 * normalize_features (src/feature_extraction.py:157-181): column mean and population std
 * (ddof = 0, numpy axis-0 order: sequential over rows), std == 0 -> 1, then (X - mean) / std.
 * dsp_zscore_fit writes mean/std [D] (std already with the 0 -> 1 substitution);
 * dsp_zscore_apply writes out [N, D] (may alias X).  float64 throughout.
 */
int dsp_zscore_fit(const double *X, int64_t N, int D, double *mean, double *std, void *stream);
int dsp_zscore_apply(const double *X, int64_t N, int D, const double *mean, const double *std,
                     double *out, void *stream);

/*
 * Batch WAV reader -- host only (no GPU, no stream): the file side of load_wav
 * (src/audio_processing.py:9-46) for a whole file list, on n_threads native threads.
 * dsp_wav_scan walks each file's RIFF chunks ('fmt ' with WAVE_FORMAT_PCM before 'data', chunks
 * padded to even sizes, nframes = data bytes // frame bytes, the data fully present) and reports
 * kind[i] = DSP_WAV_S16_MONO or DSP_WAV_U8_MONO with nsamp[i] samples at byte data_off[i], or
 * DSP_WAV_OTHER (any other layout, stereo included, or an unreadable / malformed file: the
 * caller's own reader decodes it or reports the reference's error).  dsp_wav_read writes the
 * samples of every S16/U8 mono file with nsamp > 0 to dst + dst_off[i] (HOST memory, e.g. a pinned
 * staging buffer): int16 as stored, 8-bit as ((u8 - 128) mod 256) like load_wav's uint8
 * arithmetic (:31-34); a file that fails to read is turned into DSP_WAV_OTHER in kind[].
 * paths: NUL-terminated file names.  Returns DSP_OK or DSP_ERR_ARGS.
 */
#define DSP_WAV_OTHER 0
#define DSP_WAV_S16_MONO 1
#define DSP_WAV_U8_MONO 2
int dsp_wav_scan(const char *const *paths, int64_t n, int n_threads, int32_t *kind, int64_t *nsamp,
                 int64_t *data_off);
int dsp_wav_read(const char *const *paths, int64_t n, int n_threads, int32_t *kind, const int64_t *nsamp,
                 const int64_t *data_off, const int64_t *dst_off, int16_t *dst);

/* ABI version of the loaded library (DSP_ABI_VERSION). */
int dsp_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DSP_AUDIOREC_H */
