/*
 * cbw.h — C ABI of libcbw.so, the MI355X (gfx950) CB-Whisper hot path.
 *
 * The reference (Priberam/Enhance-CB-Whisper) is pure Python/PyTorch and has
 * no FFI; each entry point below replaces the reference call it names
 * (paths relative to the reference src/).  The Python shim in
 * enhance-cb-whisper_amd/{efficient_kws,cbw} binds these with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - every buffer argument is a DEVICE pointer owned by the caller (PyTorch
 *     caching allocator); host pointers appear only in *_set_param;
 *   - `stream` is a hipStream_t (NULL = legacy default stream); calls are
 *     asynchronous, never synchronise, never allocate (capturable in hipGraphs);
 *     scratch comes from a caller-provided workspace sized by *_workspace_bytes;
 *   - return 0 on success, a negative CBW_ERR_* code otherwise; the message of
 *     the last failure on the calling thread is cbw_last_error();
 *   - bf16 tensors are passed as uint16_t*; layouts are given per argument;
 *   - handles are per device and not thread-safe.
 */
#ifndef CBW_H
#define CBW_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBW_OK 0
#define CBW_ERR_INVALID (-1)   /* bad argument / unsupported shape (cf. ValueError in the reference) */
#define CBW_ERR_HIP (-2)       /* HIP runtime error */
#define CBW_ERR_OOM (-3)       /* device allocation failed / workspace too small */
#define CBW_ERR_STATE (-4)     /* handle not finalized / parameter missing */
#define CBW_ERR_NOT_FOUND (-5) /* unknown parameter name */

typedef void* cbw_stream_t; /* hipStream_t */
typedef struct cbw_kws cbw_kws;
typedef struct cbw_encoder cbw_encoder;

int cbw_version(void);
const char* cbw_last_error(void);
/* first 16 hex digits of sha256 over the library's sources as built (csrc/Makefile SRC_ID): a stale libcbw.so shows */
const char* cbw_source_id(void);

/* ---------------------------------------------------------------- KWS classifier
 * Replaces efficient_kws.model.KWSModel (efficient_kws/model.py:18-221) and the
 * Resnet it owns (efficient_kws/resnet.py:7-58).                                */
typedef struct {
    int n_layers;       /* L: Whisper layers = ResNet input channels (<= 4; <= 16 for variant 0,
                           the 12-channel CB-Whisper CNN, model/model.py:55-58)  model.py:29,73 */
    int embedding_dim;  /* D                                                         model.py:32    */
    int variant;        /* 0 = L (no projection), 1 = LE (proj_mlp), 2 = LEF (+frames_conv)       */
    int proj_units;     /* proj_mlp_units (64)                                       model.py:37    */
    int resnet_depth;   /* 18 | 34 | 50 (resnet_version)                             resnet.py:23-30 */
} cbw_kws_config;

int cbw_kws_create(const cbw_kws_config* cfg, cbw_kws** out);
int cbw_kws_destroy(cbw_kws* h);
/* one reference state_dict entry (KWSModel.state_dict() naming, fp32 host data);
 * replaces load_state_dict / KWSModel.load_from_checkpoint (cb_whisper.py:60)  */
int cbw_kws_set_param(cbw_kws* h, const char* name, const float* host, int64_t numel);
/* fold BatchNorm (eval statistics) into conv weights, convert, upload */
int cbw_kws_finalize(cbw_kws* h);

/* projector (model.py:143-166): x f32 [B][L][T][D] (per-frame L2-normalised hs),
 * mask f32 [B][L][T] -> out bf16 [B][L][T'][E] rows L2-normalised with
 * clamp(norm, 1e-6) (the sim_matrix normalisation, model.py:210-218), E = proj_units
 * (LE/LEF) or D (L); T' = floor((T-1)/2)+1 for LEF else T.  mask_out f32 [B][L][T']
 * (LEF: max-pooled; else a copy).                                */
int64_t cbw_kws_project_workspace_bytes(cbw_kws* h, int B, int T);
int cbw_kws_project(cbw_kws* h, const float* x, const float* mask, int B, int T, uint16_t* out, float* mask_out,
                    void* ws, int64_t ws_bytes, cbw_stream_t stream);

/* forward tail (model.py:167-193 + resnet.py:51-58): masked cosine-similarity maps
 * of utt bf16 [L][Tu][E] vs kwd bf16 [K][L][Tk][E] -> ResNet -> logits f32 [K][2].
 * features (optional) f32 [K][L][Tk][Tu] = KWSOutput.features (model.py:202-208).
 * Keywords are processed in chunks of `chunk` pairs.                            */
int64_t cbw_kws_workspace_bytes(cbw_kws* h, int Tk, int Tu, int chunk);
int cbw_kws_score(cbw_kws* h, const uint16_t* utt, const float* utt_mask, const uint16_t* kwd, const float* kwd_mask,
                  int K, int Tk, int Tu, float* logits, float* features, int chunk, void* ws, int64_t ws_bytes,
                  cbw_stream_t stream);

/* fp8 first tier of the exact-decision cascade (BASELINE C5 "fp8 MFMA"; the ResNet of efficient_kws/resnet.py:51-58
 * called at efficient_kws/model.py:193): the stem and stage 1 on the bf16 network, stages 2-4 of ResNet-50 on
 * e4m3 operands (v_mfma_scale_f32_16x16x128_f8f6f4), one static scale per activation tensor, per-channel weight
 * scales.  cbw_kws_calibrate_fp8 (setup, synchronises): the fp32 network over the calibration pairs (sel, inputs as
 * cbw_kws_rescore) measures every stage-2..4 tensor's absolute maximum, scale = amax * margin / 448, and quantizes
 * the weights; cbw_kws_score_fp8: as cbw_kws_score (no features), logits of every pair from the fp8 network;
 * cbw_kws_set_score_offset_fp8: that pass's classifier bias = reference bias + offset; cbw_kws_fp8_scales: the
 * calibrated scales [stage-1 output, then per fp8 block x, t1, t2, shortcut] (returns their count). */
int cbw_kws_calibrate_fp8(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask,
                          int K, int Tk, int Tu, const int32_t* sel, int n_sel, float margin, void* ws, int64_t ws_bytes,
                          cbw_stream_t stream);
int cbw_kws_score_fp8(cbw_kws* h, const uint16_t* utt, const float* utt_mask, const uint16_t* kwd,
                      const float* kwd_mask, int K, int Tk, int Tu, float* logits, int chunk, void* ws, int64_t ws_bytes,
                      cbw_stream_t stream);
int cbw_kws_set_score_offset_fp8(cbw_kws* h, const float* offset);
int cbw_kws_fp8_scales(cbw_kws* h, float* scales, int max_n);

/* Resnet.forward on caller-built maps (efficient_kws/resnet.py:51-58):
 * maps f32 NCHW [K][L][Tk][Tu] -> logits f32 [K][2]; same workspace as cbw_kws_score. */
int cbw_kws_classify(cbw_kws* h, const float* maps, int K, int Tk, int Tu, float* logits, int chunk, void* ws,
                     int64_t ws_bytes, cbw_stream_t stream);

/* CB-Whisper's own spotter (model/cb_whisper.py:93-129, :189-210; model/model.py:78-93):
 * per-layer similarity of keyword frames vs utterance frames (plain inner products of
 * L2-normalised hs, no masks), each keyword's [Tk_k x Tu] matrices bilinearly resized to
 * (Ho, Wo) (torchvision resize, antialias=False), the n_layers-channel ResNet -> logits f32 [K][2].
 * Needs variant 0 (raw hs).  utt bf16 [L][Tu][D]; kwd bf16 [L][R][D] with keyword k on rows
 * off[k] .. off[k+1]-1; off_dev / off_host: the same int32 [K+1] offsets on device and host. */
int64_t cbw_kws_score_resized_workspace_bytes(cbw_kws* h, const int32_t* off_host, int K, int Tu, int D, int Ho,
                                              int Wo, int chunk);
int cbw_kws_score_resized(cbw_kws* h, const uint16_t* utt, int Tu, const uint16_t* kwd, int R, int D,
                          const int32_t* off_dev, const int32_t* off_host, int K, int Ho, int Wo, float* logits,
                          int chunk, void* ws, int64_t ws_bytes, cbw_stream_t stream);

/* fp32 re-scoring (exact decisions; the reference evaluates in fp32, eval-*-comp-*.yaml precision
 * 32-true).  Same forward as cbw_kws_project / cbw_kws_score, every tensor fp32 and every conv on the
 * fp32-input MFMA (exact products, fp32 accumulation), BN folded in fp32, no conv fusion:
 *   cbw_kws_project_f32: x f32 [B][L][T][D] -> out f32 [B][L][T'][E] (rows L2-normalised, clamp 1e-6);
 *   cbw_kws_rescore: logits[sel[i]] (f32 [K][2]) <- the fp32 ResNet logits of keyword sel[i] (device
 *     int32 [n_sel]) vs the utterance; utt f32 [L][Tu][E], kwd f32 [K][L][Tk][E], masks as cbw_kws_score.
 * Used on the pairs whose bf16 probability lies near the threshold (efficient_kws KWSModel exact_band).
 * n_layers <= 4 only.                                                                           */
int64_t cbw_kws_project_f32_workspace_bytes(cbw_kws* h, int B, int T);
int cbw_kws_project_f32(cbw_kws* h, const float* x, const float* mask, int B, int T, float* out, float* mask_out,
                        void* ws, int64_t ws_bytes, cbw_stream_t stream);
int64_t cbw_kws_rescore_workspace_bytes(cbw_kws* h, int Tk, int Tu);
int cbw_kws_rescore(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask, int K,
                    int Tk, int Tu, const int32_t* sel, int n_sel, float* logits, void* ws, int64_t ws_bytes,
                    cbw_stream_t stream);

/* compensated-bf16 re-scoring (the middle tier between the bf16 scores and cbw_kws_rescore): the same
 * arguments and result as cbw_kws_rescore, but the 52 ResNet convs run on the bf16 MFMA kernels over a
 * 3-term split (activations [x_hi | x_hi | x_lo], weights [w_hi | w_lo | w_hi], fp32 accumulation: the
 * products of fp32 values to ~2^-16 relative), similarity maps, stem, pooling and the classifier in fp32.
 * About 3x the bf16 cost per pair instead of 16x for fp32-input MFMA; the band it leaves within the
 * decision threshold goes to cbw_kws_rescore.  n_layers <= 4 only.                                    */
int64_t cbw_kws_rescore_x3_workspace_bytes(cbw_kws* h, int Tk, int Tu);
int cbw_kws_rescore_x3(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask,
                       int K, int Tk, int Tu, const int32_t* sel, int n_sel, float* logits, void* ws,
                       int64_t ws_bytes, cbw_stream_t stream);

/* bias correction of the bf16 scoring network (setup, no counterpart in the reference: it only narrows the
 * bf16 error the exact tiers must cover).  Runs the fp32 network (cbw_kws_rescore's arguments and
 * workspace) over the n_sel calibration pairs, takes each conv's mean input per channel E[x_c], and sets
 * the bf16 conv's bias to b + sum_{kh,kw,c} E[x_c] (w - bf16(w)) (the mean output shift of rounding the
 * weights; Nagel et al. 2019).  The fp32 and compensated tiers are unchanged.  Synchronises `stream`;
 * n_sel == 0 restores the folded biases.  n_layers <= 4 only.                                     */
int cbw_kws_calibrate_bias(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask,
                           int K, int Tk, int Tu, const int32_t* sel, int n_sel, void* ws, int64_t ws_bytes,
                           cbw_stream_t stream);
/* the bf16 scoring pass's logit offset: its classifier bias becomes classifier.1.bias + offset (host f32 [2]);
 * the compensated and fp32 tiers keep the reference bias.  KwsEngine.calibrate_bias sets it to the mean
 * fp32 - bf16 logit difference over the calibration pairs (the systematic error the weight correction
 * leaves); {0, 0} restores the reference bias.  Synchronous.                                            */
int cbw_kws_set_score_offset(cbw_kws* h, const float* offset);

/* measurement hooks (bench.py roofline): with max_launches > 0, every following
 * implicit-GEMM conv launch of this handle (up to max_launches) is bracketed by
 * hipEvents on its stream; _read (after the work completed) returns the summed
 * kernel time (ms), the summed algorithmic FLOPs 2*M*Cout*Cin*KH*KW and the
 * launch count, and rewinds.  max_launches = 0 disables.  Allocates events:
 * call outside graph capture.                                                   */
int cbw_kws_profile(cbw_kws* h, int max_launches);
int cbw_kws_profile_read(cbw_kws* h, double* ms, double* flop, int* n_launches);
/* the recorded launches themselves (call before _read, which rewinds): per launch its start / end (ms after
 * the first recorded launch started) and algorithmic FLOPs, up to max_records; returns the number recorded */
int cbw_kws_profile_records(cbw_kws* h, double* start_ms, double* end_ms, double* flop, int max_records);
/* The tier of each recorded launch (0 the bf16 scoring pass, 1 the compensated re-scoring tier, whose convs are
 * recorded too: their FLOPs are the split GEMMs' 2 M N K with K over the three segments).  Returns the count. */
int cbw_kws_profile_tiers(cbw_kws* h, int32_t* tier, int max_records);
/* The kernel each recorded launch ran (rocprofv3's short kernel name with its template arguments, e.g.
 * "conv_igemm_p8<1, 1, 256>"; the fused stage-1 blocks "bottleneck_kernel<64>" / "bottleneck_ring_kernel"): static
 * strings owned by the library.  Returns the count (round 6: bench.py's per-kernel in-bench roofline table). */
int cbw_kws_profile_kernels(cbw_kws* h, const char** kernel, int max_records);

/* decision (model.py:782-799, :804-813): prob = softmax(logits)[:,1] * ghost;
 * mode 0: idx = sorted {k : prob >= thr}; mode 1: argmax(logits) == 1
 * (cb_whisper.py:128).  prob (optional) f32 [K]; idx int32 [K]; n int32 [1].   */
int cbw_kws_spot(const float* logits, const float* ghost, int K, float thr, int mode, float* prob, int32_t* idx,
                 int32_t* n, cbw_stream_t stream);
/* 64-bit content checksum of a device byte range (16-byte aligned; position-dependent, not cryptographic): the
 * key of the keyword-database projection cache (efficient_kws.model.KWSModel re-projects the database when its
 * content changed, where the reference re-projects every group on every call, efficient_kws/model.py:767-780).
 * out: device uint64 [1]; ws >= cbw_checksum_workspace_bytes().                                             */
int64_t cbw_checksum_workspace_bytes(void);
int cbw_checksum(const void* data, int64_t bytes, uint64_t* out, void* ws, int64_t ws_bytes, cbw_stream_t stream);
/* the near-threshold band of the bf16 scores (the pairs cbw_kws_rescore re-runs in fp32 so the decision of
 * model.py:810-813 follows the reference's fp32 evaluation, eval-*-comp-*.yaml:8 `32-true`):
 * idx = sorted {k : |softmax(logits[k])[1] * ghost[k] - thr| <= band}, n = count (device int32).      */
int cbw_kws_band(const float* logits, const float* ghost, int K, float thr, float band, int32_t* idx, int32_t* n,
                 cbw_stream_t stream);
/* the same band with a half-width proportional to the pair's logit magnitude:
 * idx = sorted {k : |p[k] - thr| <= coef * max(|logits[k][0]|, |logits[k][1]|)} (the bf16 rounding error of a
 * pair's decision variable scales with its activations).                                  */
int cbw_kws_band_scaled(const float* logits, const float* ghost, int K, float thr, float coef, int32_t* idx,
                        int32_t* n, cbw_stream_t stream);

/* ---------------------------------------------------------------- Whisper front end
 * Replaces WhisperFeatureExtractor(padding='max_length') (utils.py:186-187).
 * pcm f32 [n] (16 kHz) -> out f32 [n_mel][3000]; packed (optional) bf16 [3000][cpad]
 * time-major copy for cbw_encoder_hs (cpad >= n_mel, multiple of 64).
 * ws: >= 64 bytes.                                                              */
int cbw_mel(const float* pcm, int64_t n, int n_mel, float* out, uint16_t* packed, int cpad, void* ws,
            cbw_stream_t stream);
/* long-form features (the input of PBAWhisper.generate beyond 30 s, pba_whisper.py:343-475):
 * WhisperFeatureExtractor(padding='longest', truncation=False) of one waveform -- reflect padding at the
 * audio's ends, no zero padding, out f32 [n_mel][n / 160], the max - 8 floor over the whole audio.
 * ws >= 1 KB (partial maxima).                                                                        */
int cbw_mel_long(const float* pcm, int64_t n, int n_mel, float* out, void* ws, cbw_stream_t stream);

/* ---------------------------------------------------------------- Whisper encoder
 * Replaces WhisperModel.encoder(input_features, output_hidden_states=True)
 * (cb_whisper.py:100-104, utils.py:188-192).                                    */
typedef struct {
    int n_mel, d_model, n_layers, n_heads, ffn_dim;
} cbw_encoder_config;
int cbw_encoder_create(const cbw_encoder_config* cfg, cbw_encoder** out);
int cbw_encoder_destroy(cbw_encoder* h);
int cbw_encoder_set_param(cbw_encoder* h, const char* name, const float* host, int64_t numel);
int cbw_encoder_finalize(cbw_encoder* h);
int64_t cbw_encoder_workspace_bytes(cbw_encoder* h, int B);
/* mel bf16 [B][3000][cpad] (cpad = n_mel rounded up to 64) -> hs f32 [B][n_ids][1500][D]
 * = hidden_states[layer_ids[i]] (0 = embeddings, i = layer i output, n_layers = post-LN),
 * layer_ids is a HOST int32 array.  flags bit 0: divide by the per-frame L2 norm
 * (cb_whisper.py:106, utils.py:195); bit 1: stop after the last requested state
 * (same outputs, skips the layers no requested state depends on).               */
int cbw_encoder_hs(cbw_encoder* h, const uint16_t* mel, int B, const int32_t* layer_ids, int n_ids, int normalize,
                   float* hs, void* ws, int64_t ws_bytes, cbw_stream_t stream);

/* ---------------------------------------------------------------- Whisper decoder
 * Replaces the per-step WhisperDecoder forward that PBAWhisper.generate drives through
 * HF beam search (pba_whisper.py:323-331 short-form, :425-442 long-form).  B decoding
 * rows (= batch x beams) share Benc encoder items (row r reads item r / (B/Benc)).
 * `state` (size cbw_decoder_state_bytes) holds the self-attention KV cache
 * [L][B][max_len][D] and the cross-attention KV [L][Benc][1500][D] (bf16) plus scratch. */
typedef struct {
    int vocab, d_model, n_layers, n_heads, ffn_dim, max_len;   /* max_len <= 448 (max_target_positions) */
} cbw_decoder_config;
typedef struct cbw_decoder cbw_decoder;
int cbw_decoder_create(const cbw_decoder_config* cfg, cbw_decoder** out);
int cbw_decoder_destroy(cbw_decoder* h);
/* HF WhisperDecoder names without the `model.decoder.` prefix (embed_tokens is also proj_out) */
int cbw_decoder_set_param(cbw_decoder* h, const char* name, const float* host, int64_t numel);
int cbw_decoder_finalize(cbw_decoder* h);
int cbw_decoder_vocab_padded(cbw_decoder* h);   /* logits row pitch: vocab rounded up to 128 */
int64_t cbw_decoder_state_bytes(cbw_decoder* h, int B, int Benc);
/* cross-attention K/V from the post-LN encoder output f32 [Benc][1500][D] (once per window) */
int cbw_decoder_cross_kv(cbw_decoder* h, const float* enc_out, int Benc, void* state, int64_t state_bytes, int B,
                         cbw_stream_t stream);
/* one token per row at position pos (tokens int32 [B], device) -> logits f32 [B][vocab_padded] */
int cbw_decoder_step(cbw_decoder* h, const int32_t* tokens, int pos, int B, int Benc, void* state, int64_t state_bytes,
                     float* logits, cbw_stream_t stream);
/* the same step with the position read from device memory (pos_dev: one int32): every launch argument is then
 * independent of the position, so a caller can capture one step into a hipGraph and replay it for every
 * position (write *pos_dev, replay).  Needs the fused GEMV path (B <= 16, the defaults).                   */
int cbw_decoder_step_dev(cbw_decoder* h, const int32_t* tokens, const int32_t* pos_dev, int B, int Benc, void* state,
                         int64_t state_bytes, float* logits, cbw_stream_t stream);
/* beam reorder of the self-attention cache: row r <- row src_rows[r] for positions [0, len) */
/* Prefill of a forced prefix (replaces stepping the forced decoder_input_ids one token at a time): the T
 * prefix tokens (device int32 [T]) run as T rows at positions 0..T-1 with causal self-attention; their K/V
 * go to positions 0..T-1 of all B beam rows (identical through a forced prefix, HF beam search); logits
 * (f32 [vocab_padded]) receives the last token's logits.  Benc must be 1.  The next cbw_decoder_step is at
 * pos = T. */
int cbw_decoder_prefill(cbw_decoder* h, const int32_t* tokens, int T, int B, int Benc, void* state,
                        int64_t state_bytes, float* logits, cbw_stream_t stream);
/* Several windows in one decode step (rows = windows x beams, Benc = windows; no reference counterpart: the
 * reference decodes one audio per generate call, pba_whisper.py:343-475 -- this batches the long-form windows of
 * several audios so each step streams the decoder weights once for all of them).  Window w's beams are rows
 * [w nb, (w + 1) nb) and attend to encoder slot w.
 * cross_kv_slot: slot `slot`'s cross-attention K/V from enc_out f32 [1500][D] (the other slots untouched).
 * prefill_rows: cbw_decoder_prefill into rows [r0, r0 + nb) against slot `slot` (the other rows untouched);
 *   logits (f32 [vocab_padded]) receives the last token's logits.
 * step_rows: cbw_decoder_step_dev with one position per row (pos_rows: device int32 [B]); each row's logits
 *   equal those of a step over its window alone (bit for bit: the rows' arithmetic does not depend on B). */
int cbw_decoder_cross_kv_slot(cbw_decoder* h, const float* enc_out, int slot, int Benc, void* state,
                              int64_t state_bytes, int B, cbw_stream_t stream);
int cbw_decoder_prefill_rows(cbw_decoder* h, const int32_t* tokens, int T, int slot, int r0, int nb, int B, int Benc,
                             void* state, int64_t state_bytes, float* logits, cbw_stream_t stream);
int cbw_decoder_step_rows(cbw_decoder* h, const int32_t* tokens, const int32_t* pos_rows, int B, int Benc, void* state,
                          int64_t state_bytes, float* logits, cbw_stream_t stream);
/* Cross-attention probabilities for token-level timestamps (transformers WhisperGenerationMixin.
 * _extract_token_timestamps, reached from pba_whisper.py:333-336 and the long-form return_token_timestamps path,
 * :425-442): the decoder runs teacher-forced over tokens[0..T) (device int32) against encoder slot 0 of `state`
 * (cbw_decoder_cross_kv first), writing its K/V into cache row 0, and for each (layer, head) pair i of `heads`
 * (host int32 [2 n]) probs[i][t][j] = softmax_j(q_t . k_j) over the 1500 encoder frames (device f32 [n][T][1500]):
 * the weights generate's cross_attentions carry for the alignment heads, one query row per decoder position. */
int cbw_decoder_cross_attn_probs(cbw_decoder* h, const int32_t* tokens, int T, const int32_t* heads, int n, int B,
                                 int Benc, void* state, int64_t state_bytes, float* probs, cbw_stream_t stream);
/* Dynamic time warping for token-level timestamps (host code, transformers' _dynamic_time_warping): matrix f64
 * [rows][cols] (host, row-major; the negated, normalised, median-filtered mean alignment weights); writes the
 * warping path as text_idx / time_idx (host int32, >= rows + cols entries) and its length to *len. */
int cbw_dtw(const double* matrix, int rows, int cols, int32_t* text_idx, int32_t* time_idx, int* len);
int cbw_decoder_reorder(cbw_decoder* h, const int32_t* src_rows, int B, int Benc, int len, void* state,
                        int64_t state_bytes, cbw_stream_t stream);
/* HF beam-search scores: log_softmax(logits) + bias, and their top-k (k <= 16, ties -> lower id) per
 * row.  bias = the logits processors as additive -inf masks, f32 [V] shared (bias_ld = 0) or per row
 * [B][bias_ld] (the timestamp rules), or NULL; the normaliser is the RAW logits' logsumexp
 * (next_token_scores = log_softmax(logits) before the processors).  lp f32 [B][k], idx int32 [B][k]. */
int cbw_logprob_topk(const float* logits, int B, int V, int ld, const float* bias, int64_t bias_ld, int k, float* lp,
                     int32_t* idx, cbw_stream_t stream);
/* WhisperTimeStampLogitsProcessor (long-form, return_timestamps; pba_whisper.py:425-442 runs it through
 * HF generate): per row r, bias_out[r][V] = bias (shared [V] suppression or NULL) + the timestamp masks
 * for that row's state[r] = {last_was_timestamp, penultimate_was_timestamp, lowest allowed timestamp
 * id, at_begin}; max_initial < 0 disables max_initial_timestamp_index.                             */
int cbw_timestamp_rules(const float* logits, int B, int V, int ld, const float* bias, const int32_t* state,
                        int timestamp_begin, int no_timestamps, int eos, int max_initial, float* bias_out,
                        cbw_stream_t stream);

/* One beam-search step's bookkeeping on the GPU (HF 4.37 BeamSearchScorer.process's next-beam choice,
 * generate/beam_search.py as pinned by cbw/generate.py), so a decode loop needs no host round trip per
 * token: candidates beam_scores[r] (f64 [B], in/out) + lp[r][j] (cbw_logprob_topk, [B][k]) sorted by
 * (score desc, row, token), top k logged to cand_score f64 [k], cand_row / cand_tok int32 [k] (the host
 * replays the EOS candidates into its finished hypotheses and detects the end); the first B non-EOS
 * candidates become the next beams: tokens / parents int32 [B] (parents feed cbw_decoder_reorder), *ok = 1
 * when B were found.  ts_state int32 [B][4] = {n, last, second last, last timestamp (-1)} of each row's
 * tokens at positions >= the rules' begin index, advanced by this step's token when count != 0 and gathered
 * from the parent rows; st_out int32 [B][4] = the cbw_timestamp_rules state for the next position. */
int cbw_beam_select(const float* lp, const int32_t* idx, int B, int k, int eos, double* beam_scores,
                    double* cand_score, int32_t* cand_row, int32_t* cand_tok, int32_t* tokens, int32_t* parents,
                    int32_t* ok, int32_t* ts_state, int32_t* st_out, int timestamp_begin, int count,
                    cbw_stream_t stream);

/* ---------------------------------------------------------------- building blocks (tests, tools)
 * NHWC bf16 implicit-GEMM convolution, y = act(conv(x, w) + bias (+ res)).
 * x [N][H][W][Cin], w [Cout][KH][KW][Cin], res/y [N][Ho][Wo][Cout]; Cin % 64 == 0, Cout % 64 == 0.
 * flags: 1 ReLU, 2 GELU, 4 res is f32, 8 y is f32, 16 add res after the activation. */
int cbw_conv2d(const uint16_t* x, const uint16_t* w, const float* bias, const void* res, void* y, int N, int H, int W,
               int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int flags, cbw_stream_t stream);
/* the fp8 tier's conv (building block, exposed for the parity tests): x e4m3 NHWC [N][H][W][Cin], w e4m3
 * [Cout][k][k][Cin], y[m][n] = act(alpha[n] * sum x.w + bias[n] (+ res[m][n] * res_scale)) stored as e4m3 of
 * y / y_scale (saturated at 448) or bf16 (out_bf16); res e4m3 [M][Cout] or NULL; pad k / 2; k 1 or 3;
 * Cin % 128 == 0, Cout % 128 == 0; relu 0/1. */
int cbw_conv2d_fp8(const uint8_t* x, const uint8_t* w, const float* alpha, const float* bias, const uint8_t* res,
                   float res_scale, void* y, float y_scale, int out_bf16, int relu, int N, int H, int W, int Cin,
                   int Cout, int k, int stride, cbw_stream_t stream);
/* test probes of the fp8 instructions: what 0..3 = one v_mfma_scale_f32_16x16x128_f8f6f4 with A [16][128] (a) and
 * B^T [16][128] (b) e4m3 loaded under operand lane map `what` -> out f32 C [16][16]; what 4 = the conversions,
 * a f32 [n] -> out e4m3 [n] (saturating) and out2 f32 [n] decoded back (n % 8 == 0). */
int cbw_fp8_probe(int what, const void* a, const void* b, void* out, void* out2, int n, cbw_stream_t stream);

/* 1x1 convolution over two K-sources (a ResNet expand conv with its shortcut conv folded in):
 * y = act([x | x2 sampled at (h*s2, w*s2)] . w + bias (+ res)); x [N][H][W][Cin], x2 [N][H2][W2][Cin2],
 * w [Cout][Cin + Cin2], res/y [N][H][W][Cout]; Cin, Cin2 % 64 == 0, Cout % 128 == 0; flags 1 ReLU. */
int cbw_conv1x1_dual(const uint16_t* x, const uint16_t* x2, const uint16_t* w, const float* bias, const void* res,
                     void* y, int N, int H, int W, int Cin, int H2, int W2, int Cin2, int s2, int Cout, int flags,
                     cbw_stream_t stream);
/* Plain bf16 GEMM on the implicit-GEMM tile kernel, y[M][N] = act(x[M][K] . w[N][K]^T + bias (+ res)), the
 * encoder's Linear layers (out-projection / fc2 run split-K: replaces the nn.Linear calls of HF
 * WhisperEncoderLayer under src/model/cb_whisper.py:100-104).  flags as cbw_conv2d.  ksplit: 0 = the factor
 * the encoder picks (cbw_gemm_splitk_factor), 1 = unsplit, S > 1 = S K-slices into fp32 partials
 * (partial: >= S * M * N floats) reduced in slice order by the split-K epilogue (deterministic). */
int cbw_gemm_splitk_factor(int M, int K, int N);
int cbw_gemm(const uint16_t* x, const uint16_t* w, const float* bias, const void* res, void* y, int M, int K, int N,
             int flags, int ksplit, float* partial, int64_t partial_floats, cbw_stream_t stream);
/* The encoder's self-attention (HF WhisperAttention under src/model/cb_whisper.py:100-104, non-causal, head dim
 * 64): qkv bf16 [B][T][3][H][64] with q pre-scaled by 1/8 -> out bf16 [B][T][H * 64], softmax in fp32. */
int cbw_encoder_attention(const uint16_t* qkv, uint16_t* out, int B, int T, int H, cbw_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CBW_H */
