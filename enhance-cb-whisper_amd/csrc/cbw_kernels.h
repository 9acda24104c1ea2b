// Internal launcher declarations (host side) for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <initializer_list>
#include <string>

typedef __bf16 bf16;

enum {
    CBW_EPI_RELU = 1,
    CBW_EPI_GELU = 2,
    CBW_EPI_RES_F32 = 4,       // residual operand is fp32 (else bf16)
    CBW_EPI_OUT_F32 = 8,       // output is fp32 (else bf16)
    CBW_EPI_RES_AFTER_ACT = 16, // y = act(acc + bias) + res   (else act(acc + bias + res))
    // compensated bf16 output (the 3-term split re-scoring tier): y is bf16 [M][2*Cout] = [hi | lo] with
    // hi = bf16(v), lo = bf16(v - hi); a following conv reads it with xfold = Cout as the three K-segments
    // [hi | hi | lo] against weights [w_hi | w_lo | w_hi], summing x_hi.w_hi + x_hi.w_lo + x_lo.w_hi in
    // fp32; y32 (optional) receives v in fp32 [M][Cout].  Tile kernels only.
    CBW_EPI_SPLIT3 = 32,
    // residual given as such a [hi | lo] tensor (res_ld = 2*Cout): res = hi + lo
    CBW_EPI_RES_SPLIT = 64
};

struct ConvArgs {
    const void* x;      // [N][H][W][Cin] bf16
    const void* w;      // [Cout][KH][KW][Cin] bf16
    const float* bias;  // [Cout] or null
    const void* res;    // [M][res_ld] or null
    void* y;            // [M][y_ld]
    const void* zero;   // >= 16 bytes of zeros in device memory
    int N, H, W, Cin, Ho, Wo, Cout, KH, KW;
    int sh, sw, ph, pw;
    int M;              // N*Ho*Wo
    int res_ld, y_ld;
    int flags;
    // optional second K-source (1x1 convs only): y = act([x | x2(strided)] . w + bias) with
    // w [Cout][Cin + Cin2]; x2 is [N][H2][W2][Cin2] sampled at (oh*s2, ow*s2).  Used to fold a
    // ResNet shortcut conv into the expand conv of the same block (no shortcut tensor in HBM).
    const void* x2;
    int Cin2, H2, W2, s2;
    // split-K (conv_igemm_kernel only, set by cbw_conv_igemm_splitk): block z of grid.y accumulates K-steps
    // [z nsteps / ksplit, (z + 1) nsteps / ksplit) and stores raw fp32 sums to partial[z][M][Cout]
    int ksplit;
    float* partial;
    float* y32;         // CBW_EPI_SPLIT3: optional fp32 copy of the output, [M][Cout]
    // folded input (tile kernels only): x holds x_ld channels per pixel (0 = Cin); with xfold = C > 0 the K
    // channels [0, Cin = 3C) read physical channels c < C ? c : c - C, i.e. a [hi | lo] tensor (x_ld = 2C)
    // seen as [hi | hi | lo]
    int x_ld, xfold;
};

hipError_t cbw_conv_igemm(const ConvArgs& a, hipStream_t st);
// the kernel (rocprofv3's short name, template arguments included) the last conv dispatch on this host thread
// launched: a string literal or a per-instantiation static, so the runtime's profile records keep the pointer
extern thread_local const char* cbw_last_conv_kernel;
// the CUs cbw_conv_stream sizes its persistent grid for (0: all): set by the KWS runtime while keyword chunks run on
// several streams, so the HBM-bound streaming convs leave CUs to the other streams' MFMA-bound convs
extern thread_local int cbw_cs_grid_cus;
inline std::string kernel_name(const char* base, std::initializer_list<int> targs) {   // "base<a, b, c>"
    std::string s = std::string(base) + "<";
    bool first = true;
    for (int t : targs) {
        s += (first ? "" : ", ") + std::to_string(t);
        first = false;
    }
    return s + ">";
}
// split-K for few-tile GEMMs (the Whisper encoder's out-projection and fc2 at M = 1500): the K-split factor
// that fills the GPU (1 = no split), and the split launch + a deterministic fixed-order reduction with the
// epilogue (bias, residual, activation, output type); partial holds ksplit * M * Cout floats.
int cbw_conv_splitk_factor(const ConvArgs& a);
hipError_t cbw_conv_igemm_splitk(const ConvArgs& a, int ksplit, float* partial, hipStream_t st);
// skinny GEMM for M <= 16 rows (gemv.hip): y = act(x . W^T + bias (+ res)); x [M][ldx], W [N][K] bf16;
// one workgroup per 16 output columns, K split over its waves and reduced in LDS (deterministic)
struct GemvArgs {
    const bf16* x;
    int ldx;
    const bf16* w;
    const float* bias;
    const void* res;
    int res_ld;
    void* y;
    int ldy;
    int M, N, K, flags;
    // LayerNorm prologue (optional): x = LN(xf) over K with ln_g / ln_b (eps ln_eps), xf f32 rows of
    // stride ldx, computed exactly as layernorm_kernel does; x is then ignored
    const float* xf;
    const float* ln_g;
    const float* ln_b;
    float ln_eps;
    // K/V cache append (optional): output columns [kv_D, 2 kv_D) also go to kv_k + m kv_ld + (n - kv_D),
    // [2 kv_D, 3 kv_D) to kv_v (the decode step's fused qkv projection)
    bf16* kv_k;
    bf16* kv_v;
    int64_t kv_ld;
    int kv_D;
    const int* kv_pos;   // optional: the append position read on the device (kv_k/kv_v then point at position 0)
    int kv_pos_rows;     // with kv_pos: 1 = one position per row (kv_pos[m], a step over several windows)
};
int cbw_gemv_waves(int K);
bool cbw_gemv_ln_ok(int M, int K);   // whether the LayerNorm prologue applies to this shape
hipError_t cbw_gemv(const GemvArgs& a, hipStream_t st);

// fp8 (OCP e4m3) implicit-GEMM conv (conv_fp8.hip): the first tier of the exact-decision cascade.  x / res / y
// e4m3 NHWC with one static scale per tensor (folded into the weights / res_scale / y_inv_scale); w e4m3
// [Cout][KH][KW][Cin] quantized per output channel; y = act(acc * alpha + bias (+ res * res_scale)) as e4m3
// (value * y_inv_scale, saturated) or bf16 (out_bf16).  1x1 / 3x3, Cin % 128 == 0, Cout % 128 == 0.
struct F8ConvArgs {
    const uint8_t* x;
    const uint8_t* w;
    const float* alpha;
    const float* bias;
    const uint8_t* res;
    float res_scale;
    void* y;
    float y_inv_scale;
    int out_bf16;
    const void* zero;
    int N, H, W, Cin, Ho, Wo, Cout, KH, KW, sh, sw, ph, pw, M;
    int relu;
};
bool cbw_conv_fp8_supported(const F8ConvArgs& a);
// the fp8 streaming 1x1 kernel (conv_fp8_stream.hip): stride 1, Cin in {128, 256, 512}; cbw_conv_fp8 routes to it
bool cbw_conv_fp8_stream_supported(const F8ConvArgs& a);
hipError_t cbw_conv_fp8_stream(const F8ConvArgs& a, hipStream_t st);
hipError_t cbw_conv_fp8(const F8ConvArgs& a, hipStream_t st);
hipError_t cbw_quant_fp8(const uint16_t* x, uint8_t* y, int64_t n, float inv_scale, hipStream_t st);   // bf16 -> e4m3
int cbw_absmax_groups();
hipError_t cbw_absmax_f32(const float* x, int64_t n, float* part, hipStream_t st);   // part[cbw_absmax_groups()]
hipError_t cbw_mfma_fp8_probe(const uint8_t* A, const uint8_t* Bt, float* C, int mode, hipStream_t st);
hipError_t cbw_cvt_fp8_probe(const float* x, uint8_t* q, float* back, int n, hipStream_t st);

// persistent 8-wave ring kernel (conv_ring.hip): Cout % 128 == 0, Cin % 64 == 0, 1x1 / 3x3, bf16
// residual/output, ReLU or none; hipErrorNotSupported otherwise
bool cbw_conv_ring_supported(const ConvArgs& a);
hipError_t cbw_conv_ring(const ConvArgs& a, hipStream_t st);
// row-stationary streaming 1x1 kernel (conv_stream.hip): stride-1 1x1, K = Cin (+ Cin2) in {128, 256, 384, 512}
// (K 512 on 16-pixel units; CBW_CS_K512=0 sends K 512 back to the tile kernels), weights stationary in LDS,
// rows in registers; for the HBM-bound expand convs and the K 256 / 512 reduces
bool cbw_conv_stream_supported(const ConvArgs& a);
bool cbw_conv_stream_wanted(const ConvArgs& a);
hipError_t cbw_conv_stream(const ConvArgs& a, hipStream_t st);

// fused ResNet-50 stage-1 identity bottleneck (bottleneck.hip): x, y NHWC bf16 [N][H][W][256];
// wr [64][256], wm [64][3][3][64], we [256][64] bf16 (BN folded), biases f32
hipError_t cbw_bottleneck_s1(const uint16_t* x, uint16_t* y, const uint16_t* wr, const float* br, const uint16_t* wm,
                             const float* bm, const uint16_t* we, const float* be, const void* zero, int N, int H,
                             int W, hipStream_t st);
// the same block with its output quantized for the fp8 tier: y e4m3 [N][H][W][256] = e4m3(bf16 block output *
// inv_scale) (cbw_quant_fp8's arithmetic)
hipError_t cbw_bottleneck_s1_q8(const uint16_t* x, uint8_t* y, const uint16_t* wr, const float* br, const uint16_t* wm,
                                const float* bm, const uint16_t* we, const float* be, float inv_scale, int N, int H,
                                int W, hipStream_t st);
// the stage's first block: x [N][H][W][64]; wr [64][64], wm [64][3][3][64], wcat [256][64 + 64] = [W_expand |
// W_shortcut] (BN folded), bcat = b_expand + b_shortcut (load_fused_expand_shortcut)
hipError_t cbw_bottleneck_s1_first(const uint16_t* x, uint16_t* y, const uint16_t* wr, const float* br,
                                   const uint16_t* wm, const float* bm, const uint16_t* wcat, const float* bcat,
                                   const void* zero, int N, int H, int W, hipStream_t st);

// ---- KWS path (kws_kernels.hip) ----
// f32 [B][L][T][D] -> bf16 [L][B][T][D] (layer-major so each layer's rows are contiguous)
hipError_t cbw_cast_permute_lbtd(const float* x, uint16_t* y, int B, int L, int T, int D, hipStream_t st);
// rows of E floats (fp32 or bf16 in) -> L2-normalised bf16 rows with clamp(norm, eps); optional output
// row permutation from [L][B][T] to [B][L][T]
hipError_t cbw_normalize_rows(const void* x, int x_is_f32, void* y, int y_is_f32, int L, int B, int T, int E,
                              float eps, int permute_lb, hipStream_t st);
hipError_t cbw_nchw_to_nhwc4(const float* x, uint16_t* y, int K, int L, int H, int W, hipStream_t st);
hipError_t cbw_l2norm_rows_f32(float* x, int64_t rows, int E, hipStream_t st);
// LEF time projector: conv1d(U->U,k3,p1) (BN folded) + MaxPool1d(3,2,1) + L2-normalise, fp32 math.
// x: f32 [L][B][T][U] (GEMM2 output), w: f32 [L][U][3][U] (o, k, i), b: f32 [L][U]
// y: bf16 [B][L][To][U];  mask_in f32 [B][L][T] -> mask_out f32 [B][L][To] (max-pooled)
hipError_t cbw_lef_time_project(const float* x, const float* w, const float* b, void* y, int y_is_f32,
                                const float* mask_in, float* mask_out,
                                int L, int B, int T, int U, float eps, hipStream_t st);
// masked cosine-similarity maps, NHWC [K][Tk][Tu][4] bf16 (channel l < L, rest zero), L <= 4.
// kwd: bf16 [K][L][Tk][E] normalised; utt: bf16 [L][Tu][E] normalised; masks f32.
hipError_t cbw_sim_maps(const uint16_t* kwd, const float* kwd_mask, const uint16_t* utt, const float* utt_mask,
                        uint16_t* out, int K, int L, int Tk, int Tu, int E, hipStream_t st);
// same maps as fp32 NCHW [K][L][Tk][Tu] (KWSOutput.features on request)
hipError_t cbw_sim_to_nchw(const uint16_t* maps, float* out, int K, int L, int Tk, int Tu, hipStream_t st);
// ResNet stem conv7x7 s2 p3 over NHWC4 input, BN folded, ReLU. w: bf16 [64][7][8][4] (kw padded to 8)
hipError_t cbw_stem_conv(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y,
                         int N, int H, int W, int Ho, int Wo, hipStream_t st);
// stem conv + BN + ReLU + MaxPool2d(3,2,1) in one kernel (no stem tensor in HBM); y: bf16 NHWC [N][Hp][Wp][64]
hipError_t cbw_stem_pool(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H, int W,
                         int Hs, int Ws, int Hp, int Wp, hipStream_t st);
// the same over NHWC16 input (12-layer maps of the original CB-Whisper CNN), w: bf16 [64][7][8][16]
hipError_t cbw_stem16_pool(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H,
                           int W, int Hs, int Ws, int Hp, int Wp, hipStream_t st);
// the compensated tier's stem: NHWC16 [hi | hi | lo | 0] input, [w_hi | w_lo | w_hi | 0] weights, fp32 stem tile and
// max-pool, output [N][Hp][Wp][128] bf16 = [hi | lo] of the pooled fp32 value
hipError_t cbw_stem16_pool_x3(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H,
                              int W, int Hs, int Ws, int Hp, int Wp, hipStream_t st);
hipError_t cbw_maps_split16(const float* x, uint16_t* y, int K, int L, int H, int W, hipStream_t st);
// bilinear (align_corners=False, no antialias) resize of per-keyword similarity matrices to NHWC16
// bf16 [K][Ho][Wo][16]: sim f32, layer l row r at sim + l*layer_stride + r*ld; keyword k rows
// [off[k0+k], off[k0+k+1]) relative to off[k0]
hipError_t cbw_sim_resize(const float* sim, int64_t layer_stride, int ld, const int* off_dev, int k0, int K, int L,
                          int Tu, int Ho, int Wo, uint16_t* out, hipStream_t st);
hipError_t cbw_nchw_to_nhwc16(const float* x, uint16_t* y, int K, int L, int H, int W, hipStream_t st);
// MaxPool2d(3,2,1) NHWC bf16, C % 8 == 0
hipError_t cbw_maxpool3s2(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, int Ho, int Wo, hipStream_t st);
// AdaptiveAvgPool(1) + Linear(C -> 2): logits f32 [N][2]
hipError_t cbw_pool_fc(const uint16_t* x, const float* w, const float* b, float* logits, int N, int HW, int C,
                       hipStream_t st);
// prob = softmax(logits)[:,1] * ghost; idx_out = sorted {i : prob >= thr}; n_out = count.  mode 1 = argmax rule,
// mode 2 = the near-threshold band {i : |prob - thr| <= band} (the pairs the fp32 re-scoring re-runs)
// 64-bit content checksum of a 16-byte aligned device byte range (kws_kernels.hip); scratch: cbw_checksum_scratch_bytes()
int cbw_checksum_scratch_bytes();
hipError_t cbw_checksum64(const void* data, int64_t bytes, uint64_t* out, uint64_t* scratch, hipStream_t st);
hipError_t cbw_spot(const float* logits, const float* ghost, int K, float thr, float band, int mode, float* prob_out,
                    int* idx_out, int* n_out, hipStream_t st);

// ---- fp32 re-scoring path (kws_exact.hip) ----
struct F32ConvArgs {
    const float* x;     // [N][H][W][Cin]
    const float* w;     // [Cout][KH][KW][Cin]
    const float* bias;  // [Cout] or null
    const float* res;   // [M][Cout] or null
    float* y;           // [M][Cout]
    int N, H, W, Cin, Ho, Wo, Cout, KH, KW, sh, sw, ph, pw, M, relu;
};
hipError_t cbw_conv_f32(const F32ConvArgs& a, hipStream_t st);   // Cout % 64 == 0
hipError_t cbw_sim_f32(const float* kwd, const float* kwd_mask, const float* utt, const float* utt_mask, const int* sel,
                       int p0, int P, float* out, int L, int Tk, int Tu, int E, hipStream_t st);
hipError_t cbw_maxpool_f32(const float* x, float* y, int N, int H, int W, int C, int Ho, int Wo, hipStream_t st);
hipError_t cbw_pool_fc_f32(const float* x, const float* w, const float* b, const int* sel, int p0, int P, float* logits,
                           int HW, int C, hipStream_t st);
hipError_t cbw_permute_lbtd_f32(const float* x, float* y, int B, int L, int T, int D, hipStream_t st);
// fp32 [M][C] -> bf16 [M][2C] = [hi | lo] (input of the 3-term split convs, CBW_EPI_SPLIT3)
hipError_t cbw_split3(const float* x, uint16_t* y, int64_t M, int C, hipStream_t st);
// part[g][c] += sum of x[r][c] over workgroup g's rows (g < cbw_channel_sum_groups()); bias-correction statistics
hipError_t cbw_channel_sum_f32(const float* x, int64_t M, int C, float* part, hipStream_t st);
int cbw_channel_sum_groups();

// ---- Whisper front end / encoder (whisper_kernels.hip) ----
constexpr int CBW_MEL_LONG_PARTS = 256;   // long-form: partial maxima in the scratch (>= 1 KB)
// frames <= 0 / L_pad <= 0: the 30 s window (3000 frames, zero padding to 480000 samples); else long-form
// features of the whole audio (L_pad = n_samples, frames = n_samples / 160)
hipError_t cbw_mel_frames(const float* pcm, int n_samples, const float* filters, const float* twiddle,
                          float* logmel, int n_mel, hipStream_t st, int L_pad = 0, int frames = 0);
hipError_t cbw_mel_finish(float* logmel, int n_mel, float* scratch, uint16_t* packed, int cpad, hipStream_t st,
                          int frames = 0);
hipError_t cbw_layernorm(const float* x, const float* g, const float* b, uint16_t* y, float* y32, int rows, int D,
                         float eps, hipStream_t st);
hipError_t cbw_attention(const uint16_t* qkv, uint16_t* out, int B, int T, int H, int hd, hipStream_t st);

// ---- Whisper decoder step (whisper_kernels.hip) ----
// pos_inc 0: every row at pos (decode step); 1: row r at pos + r (prefill of a prefix)
hipError_t cbw_dec_embed(const int* tok, const uint16_t* E, const float* P, int pos, float* h, int B, int D,
                         hipStream_t st, int pos_inc = 0, const int* pos_dev = nullptr, int pos_rows = 0);
hipError_t cbw_dec_kv_append(const uint16_t* qkv, uint16_t* kc, uint16_t* vc, int B, int D, int maxlen, int pos,
                             hipStream_t st);
// prefill: the k, v of T prefix tokens (fused qkv rows) -> positions 0..T-1 of all B cache rows
hipError_t cbw_dec_kv_prefill(const uint16_t* qkv, uint16_t* kc, uint16_t* vc, int T, int B, int D, int maxlen,
                              hipStream_t st);
// causal 1 (prefill): query row r sees keys 0..r
hipError_t cbw_dec_attention(const uint16_t* q, int ldq, const uint16_t* kc, const uint16_t* vc, int64_t kv_bstride,
                             int n_keys, int rows_per_kv, uint16_t* out, int B, int H, int D, hipStream_t st,
                             int causal = 0);
// cross-attention probabilities of head `head` for T query rows (q row pitch ldq, pre-scaled) against n_keys cross
// keys (row pitch D): out f32 [T][n_keys] (token-level timestamps)
hipError_t cbw_dec_cross_probs(const uint16_t* q, int ldq, const uint16_t* kc, int n_keys, int T, int D, int head,
                               float* out, hipStream_t st);
hipError_t cbw_dec_reorder_kv(uint16_t* ks, uint16_t* vs, const int* rows, int B, int n_layers, int64_t layer_elems,
                              int64_t row_elems, int64_t copy_elems, hipStream_t st);
// decode-step self-attention in one launch: row r (its own K/V batch r) over min(n_keys, n_keys_pos[nk_rows ? r : 0]
// + 1) keys when n_keys_pos is given, else n_keys; n_keys <= 448
hipError_t cbw_dec_self_attn(const uint16_t* q, int ldq, const uint16_t* kc, const uint16_t* vc, int64_t kv_bstride,
                             int n_keys, uint16_t* out, int B, int H, int D, hipStream_t st, const int* n_keys_pos,
                             int nk_rows);
// split-key decode attention; part = cbw_dec_attn_split_floats(B, H) floats of scratch
int cbw_dec_attn_split_floats(int B, int H);
// n_keys_pos (optional): the key count is *n_keys_pos + 1, read on the device; n_keys then bounds it (the grid
// covers ceil(n_keys / 64) chunks; chunks past the live count contribute nothing) -- graph-replayable steps
hipError_t cbw_dec_attn_split(const uint16_t* q, int ldq, const uint16_t* kc, const uint16_t* vc, int64_t kv_bstride,
                              int n_keys, int rows_per_kv, uint16_t* out, int B, int H, int D, float* part,
                              hipStream_t st, const int* n_keys_pos = nullptr, int nk_rows = 0);
hipError_t cbw_dec_gather_rows(const uint16_t* src, uint16_t* dst, const int* rows, int B, int64_t row_elems,
                               int64_t copy_elems, hipStream_t st);
hipError_t cbw_beam_select_launch(const float* lp, const int* idx, int B, int k, int eos, double* beam_scores,
                                  double* cand_score, int* cand_row, int* cand_tok, int* tokens, int* parents, int* ok,
                                  int* ts_state, int* st_out, int ts_begin, int count, hipStream_t st);
hipError_t cbw_logprob_topk_launch(const float* logits, int B, int V, int ld, const float* bias, int64_t bias_ld,
                                   int k, float* lp, int* idx, hipStream_t st);
hipError_t cbw_timestamp_rules_launch(const float* logits, int B, int V, int ld, const float* bias, const int* state,
                                      int ts_begin, int no_ts, int eos, int max_initial, float* bias_out,
                                      hipStream_t st);
