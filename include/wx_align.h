/*
 * wx_align.h — C ABI of the MI355X (gfx950) forced-alignment + VAD-segmentation library
 * (libwxalign.so, built from whisperx_amd/csrc/wx_align.hip).
 *
 * The reference (NADOOIT/whisperX @ 2025-01-12) is pure Python; these entry points replace
 * the CPU functions on its alignment / VAD hot path, batched over many segments:
 *
 *   wx_trellis        <- whisperx/alignment.py:359  get_trellis(emission, tokens, blank_id)
 *   wx_backtrack      <- whisperx/alignment.py:387  backtrack(trellis, emission, tokens, blank_id)
 *   wx_merge_repeats  <- whisperx/alignment.py:438  merge_repeats(path, transcript)
 *   wx_align_dp       <- whisperx/alignment.py:242-250 (get_trellis -> backtrack ->
 *                        merge_repeats as align() chains them), fused: the trellis is never
 *                        materialised; a 1-bit decision map replaces it for the backtrack.
 *   wx_binarize       <- whisperx/vad.py:118  Binarize.__call__ (hysteresis + min-cut),
 *                        the kernel under vad.py:264 merge_chunks
 *   wx_channel_norm   <- whisperx/alignment.py:226-233 (wav2vec2 forward: feature encoder's
 *                        GroupNorm + GELU, time-major)
 *   wx_conv0_channel_norm <- the same layer with its 1-channel convolution fused (one pass
 *                        over the output)
 *   wx_attention_f32  <- whisperx/alignment.py:226-233 (wav2vec2 forward: the encoder's
 *                        self-attention, fp32)
 *   wx_vad_aggregate  <- whisperx/vad.py:198-240 VoiceActivitySegmentation.apply's
 *                        segmentation overlap-add (pyannote Inference.aggregate)
 *   wx_sincnet_stage  <- whisperx/vad.py:198-240 (the segmentation model's SincNet stages:
 *                        |.| / max-pool / instance norm / leaky ReLU, fused)
 *
 * Conventions
 *   - All data pointers are DEVICE pointers (allocated by the caller; the library never
 *     allocates).  Sizes passed by value are host integers.  `stream` is a hipStream_t
 *     (NULL = default stream); every call only enqueues work on it.
 *   - Segments are CSR-packed.  Segment s has T_s = em_off[s+1]-em_off[s] emission rows
 *     starting at row em_off[s] of `em` ([sum_T, V] fp32 row-major log-probabilities) and
 *     N_s = tok_off[s+1]-tok_off[s] token ids starting at tok[tok_off[s]].
 *   - Return 0 on success or a WX_E_* / hipError_t code; wx_strerror() names it.
 *     A per-segment alignment failure (the reference's backtrack() returning None) is data
 *     (status / path_len = -1), never an error code.
 *   - Reentrant; no global mutable state; one device per call (the current device).
 *   - Semantics follow the reference's torch-CPU arithmetic bit-for-bit (fp32 adds,
 *     NaN-propagating max, strict `>` backtrack test, fp64-accumulated column-0 cumsum),
 *     except path probabilities, which use the correctly rounded fp32 exp (the reference's
 *     MKL exp differs from it by at most 1 ULP).
 */
#ifndef WX_ALIGN_H
#define WX_ALIGN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    WX_OK = 0,
    WX_E_INVALID = 1001,   /* bad argument (null pointer, negative size, blank out of range) */
    WX_E_VOCAB = 1002,     /* V outside [1, WX_MAX_VOCAB] */
    WX_E_TOO_LONG = 1003,  /* a segment has more tokens than WX_MAX_TOKENS */
    WX_E_WORKSPACE = 1004, /* workspace too small (see the *_workspace_bytes queries) */
    WX_E_LAUNCH = 1005     /* kernel launch failed */
};

#define WX_MAX_VOCAB 16384   /* emission columns (V > 64: each segment's used columns are
                                gathered into a compact row of at most 256) */
#define WX_MAX_SEGMENT_COLUMNS 256 /* V > 64: distinct columns one segment may use (column 0,
                                      the blank and its token ids) */
#define WX_MAX_TOKENS 16000  /* tokens per segment (8 waves x 64 lanes x 32 cells, less halos) */

/* wx_align_dp status word: low bits = outcome, high bits = how the segment was computed */
#define WX_STATUS_MASK 15        /* 0 aligned, 1 None, 2 / 3 not computed (see wx_align_dp) */
#define WX_STATUS_RECOVERED 16   /* recomputed by the generic forward after a lost hand-off */
#define WX_STATUS_GENERIC 32     /* computed by the generic forward (> 256 distinct columns) */

const char* wx_version(void);
const char* wx_strerror(int code);

/* get_trellis (alignment.py:359-379), batched.  trellis is CSR: segment s occupies
 * (T_s+1)*(N_s+1) floats starting at element tr_off[s] (row-major [T_s+1][N_s+1]).
 * max_N = max_s N_s (host).  A segment over WX_MAX_SEGMENT_COLUMNS (V > 64) is all NaN. */
int wx_trellis(const float* em, const int64_t* em_off, int32_t V,
               const int32_t* tok, const int64_t* tok_off, const int32_t* blank_id,
               int32_t S, int64_t max_N, float* trellis, const int64_t* tr_off, void* stream);

/* Column 0 of get_trellis (alignment.py:367, `torch.cumsum(emission[:, 0], 0)`): the running
 * sums S(t) = em[0,0] + ... + em[t-1,0] for t = 0..T, accumulated in double in row order as
 * torch's CPU cumsum does, written to S[0..T] (fp64; the trellis holds them rounded to fp32).
 * em is a [T, V] fp32 row-major matrix on the device.  The fused DP's column-0 routine, one
 * wave (it exists to pin that routine bit for bit against the sequential sum). */
int wx_column0_cumsum(const float* em, int64_t T, int32_t V, double* S, void* stream);

/* backtrack (alignment.py:387-421) from a materialised trellis, batched.  The path of
 * segment s is written in forward (time-increasing) order at element em_off[s] of
 * path_tok/path_time/path_prob (capacity T_s); path_len[s] = its length or -1 (None);
 * t_start[s] = argmax of the trellis' last column (first max, NaN counted as max). */
size_t wx_backtrack_workspace_bytes(int32_t S, int64_t sum_T, int64_t max_N);
int wx_backtrack(const float* trellis, const int64_t* tr_off,
                 const float* em, const int64_t* em_off, int32_t V,
                 const int32_t* tok, const int64_t* tok_off, const int32_t* blank_id,
                 int32_t S, int64_t max_N, int64_t sum_T,
                 int32_t* path_tok, int32_t* path_time, float* path_prob,
                 int32_t* path_len, int32_t* t_start,
                 void* workspace, size_t workspace_bytes, void* stream);

/* merge_repeats (alignment.py:438-454), batched over paths stored at path_off[s] with
 * length path_len[s] (<0 = no path -> seg_count 0).  Segments are written at the same
 * offsets (capacity = path length): token index, start frame, end frame (exclusive), mean
 * probability (left-to-right fp64 sum / count, as Python's sum()). */
int wx_merge_repeats(const int32_t* path_tok, const int32_t* path_time, const float* path_prob,
                     const int64_t* path_off, const int32_t* path_len, int32_t S,
                     int32_t* seg_tok, int32_t* seg_start, int32_t* seg_end, double* seg_score,
                     int32_t* seg_count, void* stream);

/* The fused align() DP.  For every segment: trellis recurrence with a 1-bit decision map
 * (never materialised), argmax, backtrack and merge_repeats.  Outputs are CSR by tok_off:
 * seg_start/seg_end (frames, end exclusive) and seg_score of token k (the k-th
 * merge_repeats segment; a successful path always yields exactly N_s of them).
 * t_start[s] as above; status[s] & WX_STATUS_MASK = 0 aligned, 1 backtrack failed
 * (reference: None).
 * Segments the fast kernels cannot finish are recomputed in-kernel by a generic (slow,
 * barrier-per-step, ~1-3 ms per 30 s segment) forward with the same arithmetic, and say so
 * in status's flag bits: WX_STATUS_RECOVERED for a split segment whose cross-CU hand-off
 * timed out (transient starvation: another launch held the CUs), WX_STATUS_GENERIC for a
 * V > 64 segment using more than WX_MAX_SEGMENT_COLUMNS distinct emission columns.  That
 * forward keeps two rows and one decision word per cell in the kernel's LDS (3 (N + 1)
 * floats), so it holds N <= 5460 tokens in the one-wave (throughput) buckets of V > 64,
 * N <= 7167 in the latency / split buckets of V <= 64 and N <= 10921 in those of V > 64.
 * Beyond that the segment is left uncomputed and reported 2 (too many columns: split the
 * segment) or 3 (hand-off lost: re-running the call normally succeeds).
 * min_N/max_N/sum_T describe the batch (host values).
 * Split launches hand halo cells between CUs through a hand-off region of granules tagged
 * with the launch's 32-bit epoch, plus per-segment arrival counters.  wx_align_dp /
 * wx_align_dp_mode carve it out of the workspace and zero it on the stream before the launch
 * (hipMemsetAsync: the workspace may hold anything); wx_align_dp_ex takes a separate,
 * caller-owned region instead, which must be all zero before its first use and must hold
 * nothing but hand-off data afterwards: launches leave only their own granules (an older
 * launch's epoch never matches a later one) and reset the counters, so no per-launch memset
 * is needed.  One hand-off region must not be used by two launches that may run at the same
 * time (e.g. on two streams). */
size_t wx_align_dp_workspace_bytes(int32_t S, int64_t sum_T, int64_t max_N);
int wx_align_dp(const float* em, const int64_t* em_off, int32_t V,
                const int32_t* tok, const int64_t* tok_off, const int32_t* blank_id,
                int32_t S, int64_t min_N, int64_t max_N, int64_t sum_T,
                int32_t* seg_start, int32_t* seg_end, double* seg_score,
                int32_t* t_start, int32_t* status,
                void* workspace, size_t workspace_bytes, void* stream);

/* wx_align_dp with an explicit launch shape (results are identical in every mode):
 *   WX_MODE_AUTO        latency shape for batches of <= 256 segments (split over 4 CUs per
 *                       segment when the device has 4 CUs per segment), else throughput;
 *   WX_MODE_THROUGHPUT  one wave per segment up to 2048 tokens (most segments in flight);
 *   WX_MODE_LATENCY     each segment's columns spread over up to 8 waves (shortest time
 *                       per segment when the batch cannot fill the GPU), one CU each;
 *   WX_MODE_SPLIT2..4   the latency shape with each segment spread over 2..4 CUs (capped
 *                       at the device's CUs / S; 4x the emission reads).
 * wx_align_dp == wx_align_dp_mode(..., WX_MODE_AUTO) unless the environment variable
 * WX_ALIGN_MODE=0/1 forces a shape (benchmarking); WX_PARTS=2..4 opts latency launches
 * into the split. */
enum {
    WX_MODE_AUTO = -1,
    WX_MODE_THROUGHPUT = 0,
    WX_MODE_LATENCY = 1,     /* one CU per segment (WX_PARTS=2..4: split) */
    WX_MODE_LATENCY_1CU = 2, /* latency shape, one CU per segment, whatever WX_PARTS says */
    WX_MODE_SPLIT2 = 12,     /* latency shape, 2 / 3 / 4 CUs per segment */
    WX_MODE_SPLIT3 = 13,
    WX_MODE_SPLIT4 = 14
};
int wx_align_dp_mode(const float* em, const int64_t* em_off, int32_t V,
                     const int32_t* tok, const int64_t* tok_off, const int32_t* blank_id,
                     int32_t S, int64_t min_N, int64_t max_N, int64_t sum_T,
                     int32_t* seg_start, int32_t* seg_end, double* seg_score,
                     int32_t* t_start, int32_t* status,
                     void* workspace, size_t workspace_bytes, int32_t mode, void* stream);

/* Bytes of the hand-off region wx_align_dp_ex needs for a batch (0 < result; caller-owned,
 * zeroed once before first use). */
size_t wx_align_dp_handoff_bytes(int32_t S, int64_t sum_T);
/* wx_align_dp_mode with a caller-owned hand-off region (see wx_align_dp above).  handoff
 * may be NULL: then the region is carved out of the workspace and zeroed per launch. */
int wx_align_dp_ex(const float* em, const int64_t* em_off, int32_t V,
                   const int32_t* tok, const int64_t* tok_off, const int32_t* blank_id,
                   int32_t S, int64_t min_N, int64_t max_N, int64_t sum_T,
                   int32_t* seg_start, int32_t* seg_end, double* seg_score,
                   int32_t* t_start, int32_t* status,
                   void* workspace, size_t workspace_bytes,
                   void* handoff, size_t handoff_bytes, int32_t mode, void* stream);

/* Diagnostics (no device work): the kernels wx_align_dp_mode would launch for a batch of S
 * segments with token counts in [min_N, max_N] and vocabulary size V, written to buf as a
 * ';'-separated list of their rocprof names (truncated to n bytes).  Returns their number. */
int wx_align_dp_plan(int32_t S, int64_t min_N, int64_t max_N, int32_t V, int32_t mode, char* buf, size_t n);

/* Binarize.__call__ (vad.py:118-180) for n_files score columns (CSR by f_off) with
 * pyannote sliding-window geometry per file (frame i is centred at
 * 0.5*(s + (s + duration)), s = start + i*step).  onset/offset compared in fp32.
 * Regions [reg_start, reg_end] (seconds) of file f are written at reg_off[f] (capacity
 * reg_off[f+1]-reg_off[f]; F_f+1 always suffices); reg_count[f] = count, or -1 on
 * overflow.  Regions of length <= 1e-6 s are dropped (pyannote Annotation semantics). */
int wx_binarize(const float* scores, const int64_t* f_off, int32_t n_files,
                const double* sw_start, const double* sw_step, const double* sw_duration,
                float onset, float offset, double max_duration, double pad_onset, double pad_offset,
                double* reg_start, double* reg_end, const int64_t* reg_off, int64_t* reg_count,
                void* stream);

/* wx_binarize in two passes with a caller-owned workspace (same results): a chip-wide pass
 * writes per-64-frame onset/offset bit words and first-minimum records, then one wave per
 * file jumps from event to event over them (cost per event, not per frame).  total_frames =
 * f_off[n_files] (the host sizes the pre-pass grid from it). */
size_t wx_binarize_workspace_bytes(int32_t n_files, int64_t total_frames);
int wx_binarize_ex(const float* scores, const int64_t* f_off, int32_t n_files, int64_t total_frames,
                   const double* sw_start, const double* sw_step, const double* sw_duration,
                   float onset, float offset, double max_duration, double pad_onset, double pad_offset,
                   double* reg_start, double* reg_end, const int64_t* reg_off, int64_t* reg_count,
                   void* workspace, size_t workspace_bytes, void* stream);

/* Diagnostics (no device work): the kernels wx_binarize_ex launches for these thresholds
 * (compared in fp32, as wx_binarize_ex does), ';'-separated rocprof names written to buf
 * (truncated to n bytes).  offset <= onset takes the parallel scan, offset > onset (a frame
 * may both set and reset the state, vad.py:146-175) the event-jumping state machine.
 * Returns their number. */
int wx_binarize_plan(float onset, float offset, int64_t total_frames, char* buf, size_t n);

/* Emission producer (alignment.py:226-233, the wav2vec2 forward): GroupNorm with one group
 * per channel (the first feature-encoder layer) over time-major activations x [L, C] (C % 4
 * == 0, 16-byte aligned), with the affine gamma/beta (may be NULL) and, when gelu != 0, the
 * exact erf GELU fused: y = gelu((x - mean_c) / sqrt(var_c + eps) * gamma_c + beta_c).
 * Statistics in fp64 (biased variance).  y may alias x.  Workspace: see the query. */
size_t wx_channel_norm_workspace_bytes(int32_t C);
int wx_channel_norm(const float* x, int64_t L, int32_t C, const float* gamma, const float* beta, float eps,
                    int32_t gelu, float* y, void* workspace, size_t workspace_bytes, void* stream);

/* wav2vec2's first feature-encoder layer (alignment.py:226-233, the emission forward; HF
 * Wav2Vec2GroupNormConvLayer): y[t, c] = act(GroupNorm_c(conv(x)[t, c])) with conv a 1-input-
 * channel Conv1d (K <= 16 taps, stride; w [C, K], bias [C] or NULL) over the S samples of x,
 * GroupNorm with one group per channel (statistics over time in fp64, biased variance, affine
 * gamma / beta, eps) and act the exact erf GELU when gelu != 0 (identity otherwise).  y is
 * [Lout, C] time-major, Lout = (S - K) / stride + 1.  The convolution is recomputed in the
 * second pass instead of being stored.  Equal to torch's conv + GroupNorm + GELU to fp32
 * tolerance (its own summation order). */
size_t wx_conv0_channel_norm_workspace_bytes(int64_t L, int32_t C);
int wx_conv0_channel_norm(const float* x, int64_t S, int32_t K, int32_t stride, const float* w, const float* bias,
                          int32_t C, const float* gamma, const float* beta, float eps, int32_t gelu, float* y,
                          void* workspace, size_t workspace_bytes, void* stream);

/* wav2vec2 self-attention (alignment.py:226-233, the emission forward's encoder layers):
 * o[b, t, h, :] = softmax(scale * q[b, h, t, :] . k[b, h, :, :]^T) v[b, h, :, :], fp32, no mask,
 * head dim D = 64 only.  q/k/v are [B, H, T, 64] with element strides {batch, head, time}
 * (*_strides[0..2]; the head dim is contiguous; rows 16-byte aligned) — transformers' views
 * of the q/k/v projections need no copy; o is [B, T, H, 64] contiguous.  f32 MFMA, not
 * bit-identical to torch's attention (different summation order). */
int wx_attention_f32(const float* q, const float* k, const float* v, float* o, int32_t B, int32_t H, int32_t T,
                     int32_t D, const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                     float scale, void* stream);

/* The same attention over nseg segments packed back to back in one launch (the emission
 * producer's packed encoder: every segment's rows in one [rows, H, 64] batch, each segment
 * attending only to itself — the reference's one-unpadded-forward-per-segment semantics,
 * alignment.py:217-233).  seg_rows (device, nseg + 1): segment s owns rows [seg_rows[s],
 * seg_rows[s + 1]); seg_units (device, nseg + 1): prefix of H * ceil(T_s / 32), n_units its
 * last entry.  q/k/v element strides {head, row} (*_strides[0..1]); o [rows, H, 64] contiguous.
 * split: waves per 32-query tile (1, 2 or 4; 0 = chosen from n_units). */
int wx_attention_f32_packed(const float* q, const float* k, const float* v, float* o, int32_t nseg,
                            const int32_t* seg_rows, const int32_t* seg_units, int32_t n_units, int32_t H, int32_t D,
                            const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides, float scale,
                            int32_t split, void* stream);

/* wav2vec2 positional convolution over packed segments (alignment.py:226-233: the encoder's
 * Wav2Vec2PositionalConvEmbedding, run per segment): for each segment s (rows [seg_rows[s],
 * seg_rows[s + 1]) of h [rows, D], 16-byte aligned) out[t] = GELU_erf(bias + conv(h)[t]) (+ h[t]
 * when residual), conv = Conv1d(D, D, K = 128, padding 64, groups G) with zero padding at the
 * segment's ends and the last output dropped (transformers' SamePadLayer).  D / G in {48, 64}.
 * w_packed: [G][K][Cg / 4][Cg][4], w_packed[g][j][i / 4][o][i % 4] = weight[g Cg + o][i][j].
 * seg_tiles (device, nseg + 1): prefix of ceil(T_s / 128), n_tiles its last entry.  out must not
 * alias h.  f32 MFMA: equal to torch's conv to fp32 tolerance, not bit-identical. */
int wx_posconv_packed(const float* h, int32_t D, const float* w_packed, const float* bias, int32_t G, int32_t K,
                      int32_t nseg, const int32_t* seg_rows, const int32_t* seg_tiles, int32_t n_tiles,
                      int32_t residual, float* out, void* stream);

/* wav2vec2 encoder layer's residual add + LayerNorm (alignment.py:226-233, the emission
 * forward: `layer_norm(residual + x)` twice per layer): for each of `rows` rows of D floats
 * (D in {256, 512, 768, 1024}; row strides a_stride / b_stride elements, multiples of 4; all
 * pointers 16-byte aligned), s = a + b, y = (s - mean(s)) / sqrt(var(s) + eps) * gamma + beta
 * (biased variance, fp32, two passes over the row in registers).  y is [rows][D] contiguous;
 * sum_out (may be NULL) receives s in the same layout.  Equal to torch's add + LayerNorm to
 * fp32 tolerance (torch uses Welford), not bit-identical. */
int wx_add_layernorm(const float* a, const float* b, int64_t rows, int32_t D, int64_t a_stride, int64_t b_stride,
                     const float* gamma, const float* beta, float eps, float* y, float* sum_out, void* stream);

/* VAD producer (vad.py:198-240 -> pyannote SincNet): the epilogue of one SincNet stage on the
 * time-major conv output x [B windows][L][C] (window stride x_window_stride elements, row
 * stride C; C % 4 == 0, C <= 128, 16-byte aligned): y[b][t][c] = leaky_relu(InstanceNorm1d(
 * MaxPool1d(3, 3)((|)x(|)))) with |.| when do_abs (the sinc filterbank stage), the norm's
 * biased variance over the L / 3 pooled rows, eps and affine gamma/beta (may be NULL), and
 * negative slope `slope`.  y is [B][L / 3][C] contiguous.  Statistics in fp64. */
int wx_sincnet_stage(const float* x, int64_t B, int64_t L, int32_t C, int64_t x_window_stride,
                     int32_t do_abs, const float* gamma, const float* beta, float eps, float slope,
                     float* y, void* stream);
/* wx_sincnet_stage with an input affine applied before |.|: x[b][t][c] * in_scale[b] +
 * in_shift[b][c] (both NULL or both given; in_shift 16-byte aligned), and windows that may
 * overlap (any x_window_stride >= 0, a multiple of 4).  The producer runs the sinc filterbank
 * once over the waveform and reads every window's conv output from that shared buffer
 * (window stride = hop / conv stride rows): the waveform InstanceNorm of the window, a
 * per-window affine of the input, commutes with the bias-free convolution into
 * scale * conv(x) + shift_c (shift_c = the norm's offset times filter c's tap sum). */
int wx_sincnet_stage_ex(const float* x, int64_t B, int64_t L, int32_t C, int64_t x_window_stride,
                        int32_t do_abs, const float* in_scale, const float* in_shift, const float* gamma,
                        const float* beta, float eps, float slope, float* y, void* stream);

/* VAD producer's overlap-add (vad.py:198-240 -> pyannote Inference.aggregate with the
 * multi-label max-over-classes hook): scores [n_chunks, frames_per_chunk, n_classes] fp32
 * (the segmentation model's sigmoid outputs per chunk), start_frame[c] = the file-grid frame
 * where chunk c's first frame lands (non-decreasing).  out[f] = (sum over covering chunks, in
 * chunk order, of max_k scores[c, f - start_frame[c], k]) / (number of them), NaN outputs
 * masked out; `missing` where no chunk covers f.  Feeds wx_binarize on the device. */
/* VAD producer (vad.py:198-240 -> pyannote SincNet's stage 1 on the shared-sinc route): the
 * bias-free strided filterbank convolution (K taps) of one waveform span x [n] (fp32):
 * y[t][c] = sum_{j < K} x[stride t + j] w_padded[j][c] for t < (n - K) / stride + 1, y
 * time-major [rows][C].  w_padded [KP][C]: the K taps zero-padded to KP (a multiple of 4), so
 * the kernel sums KP taps, reading zeros past the end of x.  Instantiated for pyannote's
 * C = 80, KP = 260 (K = 251), stride <= 16.  fp32 (f32 MFMA: tolerance-equal to the unfold
 * GEMM it replaces). */
int wx_sinc_filterbank(const float* x, int64_t n, int32_t stride, const float* w_padded, int32_t C, int32_t K,
                       int32_t KP, float* y, void* stream);

/* VAD producer (vad.py:198-240 -> pyannote SincNet's stages 2 and 3): Conv1d(Cin, Cout, K)
 * with no padding and stride 1 over every window of a time-major batch x [B][L][Cin]
 * (contiguous, 16-byte aligned, Cin % 4 == 0, Cin <= 80, Cout <= 64, K == 5):
 * y[b][t][o] = bias[o] + sum_{j<K, i<Cin} x[b][t + j][i] w[o][i][j], y [B][L - K + 1][Cout].
 * w_packed [K][CINP / 4][64][4] (CINP = 64 for Cin <= 64, else 80), zero-padded:
 * w_packed[j][i / 4][o][i % 4] = w[o][i][j].  fp32 (f32 MFMA: tolerance-equal to the GEMM route). */
int wx_conv1d_taps_tm(const float* x, int64_t B, int64_t L, int32_t Cin, const float* w_packed, const float* bias,
                      int32_t Cout, int32_t K, float* y, void* stream);

/* VAD producer (vad.py:198-240 -> pyannote PyanNet's LSTM): one bidirectional LSTM layer,
 * hidden size H = 128, over B sequences of T steps, both directions in one persistent launch.
 * xp [B][T][2][4H]: each step's input projection x W_ih^T + b_ih + b_hh per direction (gate
 * order i, f, g, o as torch.nn.LSTM); whh [2][4H][H]: weight_hh of the forward and reverse
 * direction; y [B][T][2H] (16-byte aligned): h of the forward direction, then the reverse.
 * h0 = c0 = 0.  fp32; equal to torch.nn.LSTM to fp32 tolerance (f32 MFMA fma chains). */
int wx_lstm_bidir_layer(const float* xp, const float* whh, float* y, int64_t B, int64_t T, int32_t H, void* stream);

int wx_vad_aggregate(const float* scores, const int64_t* start_frame, int32_t n_chunks,
                     int32_t frames_per_chunk, int32_t n_classes, int64_t n_frames, float missing,
                     float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WX_ALIGN_H */
