// Whisper front end and encoder kernels for gfx950: log-mel spectrogram,
// LayerNorm, and non-causal flash attention (hd = 64).
//
// Reference semantics: HF WhisperFeatureExtractor (called at src/utils.py:186-187,
// src/data/dataset.py:332-339) and HF WhisperEncoder (called at
// src/model/cb_whisper.py:100-104, src/utils.py:188-192); see oracle/mel.py and
// oracle/encoder.py for the restated algorithms these kernels are checked against.
#include <algorithm>
#include <cstdlib>
#include <map>

#include "cbw_common.h"
#include "cbw_kernels.h"

namespace {

constexpr int N_FFT = 400, HOP = 160, N_SAMPLES = 480000, N_FRAMES = 3000, N_FREQ = 201;

// ---------------------------------------------------------------- log-mel
// one block per frame: windowed frame -> direct 400-point real DFT (exact twiddle
// table) -> |X|^2 -> mel projection -> log10(max(., 1e-10)).  Input is the raw
// clip; zero-pad/truncate to 30 s and the reflect padding of torch.stft(center=True)
// are applied on the fly.
// L_pad: the length the reflect padding of torch.stft(center=True) mirrors at (480000 for the 30 s window,
// the audio length for long-form features); frames: output frames = the row pitch of logmel
__global__ __launch_bounds__(256) void mel_frames_kernel(const float* __restrict__ pcm, int n_samples,
                                                         const float* __restrict__ filters,
                                                         const float* __restrict__ twiddle,
                                                         float* __restrict__ logmel, int n_mel, int L_pad, int frames) {
    __shared__ float xw[N_FFT];
    __shared__ float tw[2 * N_FFT];
    __shared__ float pw[N_FREQ + 7];
    const int t = blockIdx.x;
    for (int i = threadIdx.x; i < 2 * N_FFT; i += blockDim.x) tw[i] = twiddle[i];
    for (int n = threadIdx.x; n < N_FFT; n += blockDim.x) {
        int j = t * HOP + n - N_FFT / 2;
        if (j < 0) j = -j;
        if (j >= L_pad) j = 2 * (L_pad - 1) - j;
        const float v = j < n_samples ? pcm[j] : 0.f;
        const float win = 0.5f - 0.5f * tw[n];    // cos(2*pi*n/400) = twiddle[n]
        xw[n] = v * win;
    }
    __syncthreads();
    for (int f = threadIdx.x; f < N_FREQ; f += blockDim.x) {
        float re = 0.f, im = 0.f;
        int idx = 0;
        for (int n = 0; n < N_FFT; ++n) {
            re = fmaf(xw[n], tw[idx], re);
            im = fmaf(xw[n], tw[N_FFT + idx], im);
            idx += f;
            if (idx >= N_FFT) idx -= N_FFT;
        }
        pw[f] = re * re + im * im;
    }
    __syncthreads();
    for (int m = threadIdx.x; m < n_mel; m += blockDim.x) {
        float s = 0.f;
        for (int f = 0; f < N_FREQ; ++f) s = fmaf(filters[f * n_mel + m], pw[f], s);
        logmel[(int64_t)m * frames + t] = log10f(fmaxf(s, 1e-10f));
    }
}

// block b writes the max of its grid-strided share to out[b] (mel_finish_kernel reduces the gridDim.x partials)
__global__ __launch_bounds__(1024) void max_reduce_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
    __shared__ float red[16];
    float m = -INFINITY;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, x[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
        out[blockIdx.x] = r;
    }
}

// (max(x, gmax - 8) + 4) / 4, in place, + time-major bf16 copy [3000][cpad] for the encoder
__global__ void mel_finish_kernel(float* __restrict__ logmel, int n_mel, const float* __restrict__ gmax, int n_part,
                                  bf16* __restrict__ packed, int cpad, int frames) {
    float mx = gmax[0];
    for (int i = 1; i < n_part; ++i) mx = fmaxf(mx, gmax[i]);
    const float floor_v = mx - 8.0f;
    const int C = packed ? cpad : n_mel;
    const int64_t total = (int64_t)frames * C;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const int64_t t = i / C;
        float v = 0.f;
        if (c < n_mel) {
            v = (fmaxf(logmel[(int64_t)c * frames + t], floor_v) + 4.0f) * 0.25f;
            logmel[(int64_t)c * frames + t] = v;
        }
        if (packed) packed[i] = f2bf(v);
    }
}

// ---------------------------------------------------------------- LayerNorm (one wave per row)
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                        const float* __restrict__ b, bf16* __restrict__ y,
                                                        float* __restrict__ y32, int rows, int D, float eps) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + (int64_t)row * D;
    float s = 0.f;
    for (int i = lane * 4; i < D; i += 256) {
        const f32x4 v = *(const f32x4*)(xr + i);
        s += v[0] + v[1] + v[2] + v[3];
    }
    const float mean = wave_sum(s) / D;
    float ss = 0.f;
    for (int i = lane * 4; i < D; i += 256) {
        const f32x4 v = *(const f32x4*)(xr + i);
#pragma unroll
        for (int q = 0; q < 4; ++q) ss += (v[q] - mean) * (v[q] - mean);
    }
    const float rstd = rsqrtf(wave_sum(ss) / D + eps);
    for (int i = lane * 4; i < D; i += 256) {
        const f32x4 v = *(const f32x4*)(xr + i);
        const f32x4 gg = *(const f32x4*)(g + i), bb = *(const f32x4*)(b + i);
        f32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (v[q] - mean) * rstd * gg[q] + bb[q];
        if (y) {
            bf16x4 ob;
#pragma unroll
            for (int q = 0; q < 4; ++q) ob[q] = f2bf(o[q]);
            *(bf16x4*)(y + (int64_t)row * D + i) = ob;
        }
        if (y32) *(f32x4*)(y32 + (int64_t)row * D + i) = o;
    }
}

// ---------------------------------------------------------------- attention
// Non-causal softmax(Q K^T) V with Q pre-scaled by hd^-1/2 (folded into q_proj).
// qkv: bf16 [B][T][3][H][64]; out: bf16 [B][T][H*64].
// Block = 4 waves x 16 queries of one (b, h); 64-key tiles staged in LDS.
// S^T = K Q^T puts the query on the MFMA lane (lane & 15) so the online-softmax
// state is lane-local; P^T feeds O^T = V^T P^T directly from the accumulator
// with a permuted key order that the V^T operand reads in the same order.
constexpr int AT_KT = 64;
__global__ __launch_bounds__(256) void attention_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out, int T,
                                                        int H) {
    constexpr int HD = 64;
    constexpr int VT_PITCH = 136;    // bytes per d-row of V^T (64 keys * 2 B + 8 pad)
    __shared__ __attribute__((aligned(16))) char Ks[AT_KT * 128];
    __shared__ __attribute__((aligned(16))) char Vt[HD * VT_PITCH];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int bh = blockIdx.y;
    const int b = bh / H, h = bh % H;
    const int D = H * HD;
    const int64_t row_stride = 3 * (int64_t)D;
    const bf16* base = qkv + (int64_t)b * T * row_stride;
    const int q = blockIdx.x * 64 + wid * 16 + fr;
    const int qld = min(q, T - 1);
    bf16x8 qf[2];
    qf[0] = *(const bf16x8*)(base + qld * row_stride + h * HD + fq * 8);
    qf[1] = *(const bf16x8*)(base + qld * row_stride + h * HD + 32 + fq * 8);

    f32x4 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;

    for (int k0 = 0; k0 < T; k0 += AT_KT) {
        __syncthreads();
        // stage K (swizzled rows) and V^T
        for (int c = tid; c < AT_KT * 8; c += 256) {
            const int key = c >> 3, ch = c & 7;
            const int kg = k0 + key;
            bf16x8 kv, vv;
            if (kg < T) {
                kv = *(const bf16x8*)(base + kg * row_stride + D + h * HD + ch * 8);
                vv = *(const bf16x8*)(base + kg * row_stride + 2 * D + h * HD + ch * 8);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) { kv[j] = f2bf(0.f); vv[j] = f2bf(0.f); }
            }
            *(bf16x8*)(Ks + key * 128 + ((ch ^ ((key >> 1) & 7)) * 16)) = kv;
#pragma unroll
            for (int j = 0; j < 8; ++j) *(bf16*)(Vt + (ch * 8 + j) * VT_PITCH + key * 2) = vv[j];
        }
        __syncthreads();
        // S^T tile: 4 key-subtiles x 16 queries
        f32x4 s[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            s[st] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int key = st * 16 + fr;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int ch = ks * 4 + fq;
                const bf16x8 kf = *(const bf16x8*)(Ks + key * 128 + ((ch ^ ((key >> 1) & 7)) * 16));
                s[st] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[st], 0, 0, 0);
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int kg = k0 + st * 16 + fq * 4 + i;
                if (kg >= T) s[st][i] = -INFINITY;
                mx = fmaxf(mx, s[st][i]);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float m_new = fmaxf(m_run, mx);
        const float alpha = __expf(m_run - m_new);
        float rs = 0.f;
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                s[st][i] = __expf(s[st][i] - m_new);
                rs += s[st][i];
            }
        rs += __shfl_xor(rs, 16, 64);
        rs += __shfl_xor(rs, 32, 64);
        l_run = l_run * alpha + rs;
        m_run = m_new;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[dt][i] *= alpha;
        // O^T += V^T P^T ; k-step ks covers keys 32ks + {4fq..4fq+3, 16+4fq..16+4fq+3}
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 pf;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pf[j] = f2bf(s[2 * ks][j]);
                pf[4 + j] = f2bf(s[2 * ks + 1][j]);
            }
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int d = dt * 16 + fr;
                const char* vr = Vt + d * VT_PITCH + (ks * 32 + fq * 4) * 2;
                const bf16x4 v0 = *(const bf16x4*)vr;
                const bf16x4 v1 = *(const bf16x4*)(vr + 32);
                bf16x8 vf;
#pragma unroll
                for (int j = 0; j < 4; ++j) { vf[j] = v0[j]; vf[4 + j] = v1[j]; }
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
            }
        }
    }
    if (q >= T) return;
    const float inv = 1.0f / l_run;
    bf16* orow = out + ((int64_t)b * T + q) * D + h * HD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
        bf16x4 ov;
#pragma unroll
        for (int i = 0; i < 4; ++i) ov[i] = f2bf(o[dt][i] * inv);
        *(bf16x4*)(orow + dt * 16 + fq * 4) = ov;
    }
}

// ---------------------------------------------------------------- decoder step kernels
// h[r] = E[token[r]] + P[pos]  (fp32 residual stream)
__global__ void dec_embed_kernel(const int* __restrict__ tok, const bf16* __restrict__ E, const float* __restrict__ P,
                                 int pos, int pos_inc, float* __restrict__ h, int D, const int* __restrict__ pos_dev,
                                 int pos_rows) {
    const int r = blockIdx.x;
    const int t = tok[r];
    if (pos_dev) pos = pos_dev[pos_rows ? r : 0];   // pos_rows: one position per row (several windows in one step)
    const int pr = pos + pos_inc * r;   // decode step: every row at pos; prefill: row r is token r at pos + r
    for (int d = threadIdx.x; d < D; d += blockDim.x) h[(int64_t)r * D + d] = bf2f(E[(int64_t)t * D + d]) + P[(int64_t)pr * D + d];
}

// prefill: k, v of prefix token t (fused qkv row t) -> position t of every beam row's self-attention cache
__global__ void dec_kv_prefill_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ kc, bf16* __restrict__ vc, int D,
                                      int maxlen) {
    const int t = blockIdx.x, b = blockIdx.y;
    for (int d = threadIdx.x * 8; d < D; d += blockDim.x * 8) {
        *(bf16x8*)(kc + ((int64_t)b * maxlen + t) * D + d) = *(const bf16x8*)(qkv + (int64_t)t * 3 * D + D + d);
        *(bf16x8*)(vc + ((int64_t)b * maxlen + t) * D + d) = *(const bf16x8*)(qkv + (int64_t)t * 3 * D + 2 * D + d);
    }
}

// k, v of the fused qkv rows -> self-attention cache at position pos
__global__ void dec_kv_append_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ kc, bf16* __restrict__ vc, int D,
                                     int maxlen, int pos) {
    const int r = blockIdx.x;
    for (int d = threadIdx.x * 8; d < D; d += blockDim.x * 8) {
        *(bf16x8*)(kc + ((int64_t)r * maxlen + pos) * D + d) = *(const bf16x8*)(qkv + (int64_t)r * 3 * D + D + d);
        *(bf16x8*)(vc + ((int64_t)r * maxlen + pos) * D + d) = *(const bf16x8*)(qkv + (int64_t)r * 3 * D + 2 * D + d);
    }
}

// one query row per (row, head) against n_keys cached keys (decode step); q pre-scaled.
// K/V element (key j, dim c) of kv batch b at kv + b*kv_bstride + j*D + c; row r reads kv batch r / rows_per_kv.
constexpr int DA_MAXK = 1536;
__global__ __launch_bounds__(256) void dec_attention_kernel(const bf16* __restrict__ q, int ldq,
                                                            const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                            int64_t kv_bstride, int n_keys_all, int rows_per_kv,
                                                            bf16* __restrict__ out, int D, int causal) {
    __shared__ float qs[64];
    __shared__ float ps[DA_MAXK];
    __shared__ float red[8];
    __shared__ float pv[32][65];
    const int r = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
    const int b = r / rows_per_kv;
    // causal (prefill): query row r is prefix token r and sees keys 0..r
    const int n_keys = causal ? min(n_keys_all, r + 1) : n_keys_all;
    if (tid < 64) qs[tid] = bf2f(q[(int64_t)r * ldq + h * 64 + tid]);
    __syncthreads();
    const bf16* kb = kc + b * kv_bstride + h * 64;
    const bf16* vb = vc + b * kv_bstride + h * 64;
    float mx = -INFINITY;
    for (int j = tid; j < n_keys; j += 256) {
        const bf16* kr = kb + (int64_t)j * D;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 64; c += 8) {
            const bf16x8 kv = *(const bf16x8*)(kr + c);
#pragma unroll
            for (int e = 0; e < 8; ++e) s = fmaf(qs[c + e], bf2f(kv[e]), s);
        }
        ps[j] = s;
        mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float sum = 0.f;
    for (int j = tid; j < n_keys; j += 256) {
        const float e = __expf(ps[j] - mx);
        ps[j] = e;
        sum += e;
    }
    sum = wave_sum(sum);
    if ((tid & 63) == 0) red[4 + (tid >> 6)] = sum;
    __syncthreads();
    const float inv = 1.0f / (red[4] + red[5] + red[6] + red[7]);
    // P.V: thread = 8 dims (one 16-byte load per key) x every 32nd key, four keys in flight per step;
    // the 32 key groups meet in LDS (fixed order)
    const int dg = tid & 7, kg = tid >> 3;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bf16* vd = vb + dg * 8;
    int j = kg;
    for (; j + 96 < n_keys; j += 128) {
        bf16x8 v4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v4[u] = *(const bf16x8*)(vd + (int64_t)(j + 32 * u) * D);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float p = ps[j + 32 * u];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(p, bf2f(v4[u][e]), acc[e]);
        }
    }
    for (; j < n_keys; j += 32) {
        const bf16x8 vv = *(const bf16x8*)(vd + (int64_t)j * D);
        const float p = ps[j];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(p, bf2f(vv[e]), acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) pv[kg][dg * 8 + e] = acc[e];
    __syncthreads();
    if (tid < 64) {
        float o = 0.f;
        for (int k = 0; k < 32; ++k) o += pv[k][tid];
        out[(int64_t)r * D + h * 64 + tid] = f2bf(o * inv);
    }
}

// Cross-attention probabilities of one head (token-level timestamps: the alignment heads' weights that
// transformers' _extract_token_timestamps reads from generate's cross_attentions): row r = softmax_j(q_r . k_j)
// over the n_keys encoder frames, the same scores, max and exponentials as dec_attention_kernel; out f32 [T][n_keys].
__global__ __launch_bounds__(256) void dec_cross_probs_kernel(const bf16* __restrict__ q, int ldq,
                                                              const bf16* __restrict__ kc, int n_keys, int D, int h,
                                                              float* __restrict__ out) {
    __shared__ float qs[64];
    __shared__ float ps[DA_MAXK];
    __shared__ float red[8];
    const int r = blockIdx.x, tid = threadIdx.x;
    if (tid < 64) qs[tid] = bf2f(q[(int64_t)r * ldq + h * 64 + tid]);
    __syncthreads();
    const bf16* kb = kc + h * 64;
    float mx = -INFINITY;
    for (int j = tid; j < n_keys; j += 256) {
        const bf16* kr = kb + (int64_t)j * D;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 64; c += 8) {
            const bf16x8 kv = *(const bf16x8*)(kr + c);
#pragma unroll
            for (int e = 0; e < 8; ++e) s = fmaf(qs[c + e], bf2f(kv[e]), s);
        }
        ps[j] = s;
        mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float sum = 0.f;
    for (int j = tid; j < n_keys; j += 256) {
        const float e = __expf(ps[j] - mx);
        ps[j] = e;
        sum += e;
    }
    sum = wave_sum(sum);
    if ((tid & 63) == 0) red[4 + (tid >> 6)] = sum;
    __syncthreads();
    const float inv = 1.0f / (red[4] + red[5] + red[6] + red[7]);
    for (int j = tid; j < n_keys; j += 256) out[(int64_t)r * n_keys + j] = ps[j] * inv;
}

// Split-key decode attention (flash-decoding): workgroup = (key chunk of DS_CHUNK keys, head, kv batch)
// serving ALL the R query rows that share the kv batch (the beams of a window against its cross K/V: K/V
// read once, not once per beam).  With one chunk the workgroup writes the output; otherwise each writes
// its chunk's unnormalised P.V and (max, sum) per query row and dec_attn_combine_kernel merges the S
// partials in chunk order (deterministic).  (A last-arriver combine inside this kernel needs an
// agent-scope release per workgroup -- an L2 writeback on gfx950 -- and measured 1.7x slower than the
// second launch.)
// R <= RMAX rows per kv batch (1 for self-attention, beams for cross-attention); q pre-scaled.
constexpr int DS_CHUNK = 64;
constexpr int DS_MAXS = 24;   // 1536 keys

template <int RMAX>
__global__ __launch_bounds__(256) void dec_attn_split_kernel(const bf16* __restrict__ q, int ldq,
                                                             const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                             int64_t kv_bstride, int n_keys, int R,
                                                             bf16* __restrict__ out, int D, float* __restrict__ part,
                                                             const int* __restrict__ n_keys_pos, int nk_rows) {
    __shared__ float qs[RMAX][64];
    __shared__ float ps[RMAX][DS_CHUNK];
    __shared__ float st[2][RMAX];
    constexpr int NQ = 8;   // partial P.V sums per (row, dim): 4 waves x 2 half-waves
    __shared__ float red[NQ][RMAX][64];
    const int s = blockIdx.x, h = blockIdx.y, b = blockIdx.z, S = gridDim.x, H = gridDim.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r0 = b * R;
    const int j0 = s * DS_CHUNK;
    const bf16* kb = kc + b * kv_bstride + (int64_t)j0 * D + h * 64;
    const bf16* vb = vc + b * kv_bstride + (int64_t)j0 * D + h * 64;
    if (n_keys_pos) n_keys = min(n_keys, n_keys_pos[nk_rows ? b : 0] + 1);   // nk_rows: a key count per kv batch
    const int nk = min(DS_CHUNK, n_keys - j0);
    if (nk <= 0) {   // a chunk past the live keys (device-side count): a neutral partial (m = -inf, l = 0, o = 0)
        float* pp = part + ((int64_t)(b * H + h) * S + s) * (RMAX * 66);
        for (int i = tid; i < R * 64; i += 256) pp[i] = 0.f;
        if (tid < R) { pp[RMAX * 64 + tid] = -INFINITY; pp[RMAX * 65 + tid] = 0.f; }
        return;
    }
    // every global load of the chunk in flight before the first wait: the R query rows first (their LDS
    // staging then waits only for them), then K for the scores and V for P.V
    const int j = tid >> 2, p = tid & 3;          // scores: 4 threads per key, 16 dims each
    const int dg = tid & 7, kg = tid >> 3;        // P.V: 8 dims x keys kg, kg + 32
    static_assert(RMAX * 64 <= 2 * 256, "query staging: two elements per thread");
    // unconditional loads of clamped elements (a conditionally loaded value made the compiler wait for it at the
    // branch join: the two query loads and then K / V went out one round trip after another); rows past nk are
    // read as row nk - 1 and carry score -inf / weight p = 0 below (0 x a finite value adds nothing)
    const int qi0 = min(tid, R * 64 - 1), qi1 = min(tid + 256, R * 64 - 1);
    const unsigned short qv0 = ((const unsigned short*)q)[(int64_t)(r0 + (qi0 >> 6)) * ldq + h * 64 + (qi0 & 63)];
    const unsigned short qv1 = ((const unsigned short*)q)[(int64_t)(r0 + (qi1 >> 6)) * ldq + h * 64 + (qi1 & 63)];
    const int jc = min(j, nk - 1), kg0 = min(kg, nk - 1), kg1 = min(kg + 32, nk - 1);
    const bf16x8 k0 = *(const bf16x8*)(kb + (int64_t)jc * D + p * 16);
    const bf16x8 k1 = *(const bf16x8*)(kb + (int64_t)jc * D + p * 16 + 8);
    const bf16x8 v0 = *(const bf16x8*)(vb + (int64_t)kg0 * D + dg * 8);
    const bf16x8 v1 = *(const bf16x8*)(vb + (int64_t)kg1 * D + dg * 8);
    if (tid < R * 64) qs[tid >> 6][tid & 63] = bf2f(__builtin_bit_cast(bf16, qv0));
    if (tid + 256 < R * 64) qs[(tid + 256) >> 6][tid & 63] = bf2f(__builtin_bit_cast(bf16, qv1));
    __syncthreads();
    {
#pragma unroll
        for (int i = 0; i < RMAX; ++i) {
            if (i < R) {
                float d = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    d = fmaf(qs[i][p * 16 + e], bf2f(k0[e]), d);
                    d = fmaf(qs[i][p * 16 + 8 + e], bf2f(k1[e]), d);
                }
                d += xor_lane<1>(d);
                d += xor_lane<2>(d);
                if (p == 0) ps[i][j] = j < nk ? d : -INFINITY;
            }
        }
    }
    __syncthreads();
    // chunk softmax statistics: wave w takes rows w, w + 4, ...
    for (int i = w; i < R; i += 4) {
        const float v = ps[i][lane];
        const float m = wave_max_x(v);
        const float e = lane < nk ? __expf(v - m) : 0.f;
        ps[i][lane] = e;
        const float l = wave_sum_x(e);
        if (lane == 0) { st[0][i] = m; st[1][i] = l; }
    }
    __syncthreads();
    // P.V: key groups reduced by shuffles within the wave, LDS across waves (keys past nk carry p = 0, v = 0)
    float acc[RMAX][8];
#pragma unroll
    for (int i = 0; i < RMAX; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[i][e] = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bf16x8 v = u ? v1 : v0;
        const int jj = kg + 32 * u;
#pragma unroll
        for (int i = 0; i < RMAX; ++i)
            if (i < R) {
                const float pr = ps[i][jj];
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[i][e] = fmaf(pr, bf2f(v[e]), acc[i][e]);
            }
    }
#pragma unroll
    for (int i = 0; i < RMAX; ++i)
        if (i < R)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                // the two half-waves' key groups stay separate (no xor-32 round trip): 8 partials per output
                float a = acc[i][e];
                a += xor_lane<8>(a);
                a += xor_lane<16>(a);
                if ((lane & 31) < 8) red[2 * w + (lane >> 5)][i][dg * 8 + e] = a;
            }
    __syncthreads();
    auto osum = [&](int r, int d) {   // the NQ partial sums of output (r, d), in a fixed order
        float o = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q) o += red[q][r][d];
        return o;
    };
    if (S == 1 && !n_keys_pos) {
        for (int i = tid; i < R * 64; i += 256) {
            const int r = i >> 6, d = i & 63;
            out[(int64_t)(r0 + r) * D + h * 64 + d] = f2bf(osum(r, d) / st[1][r]);
        }
        return;
    }
    // partial of this chunk: o[R][64], m[R], l[R]
    float* pp = part + ((int64_t)(b * H + h) * S + s) * (RMAX * 66);
    for (int i = tid; i < R * 64; i += 256) {
        const int r = i >> 6, d = i & 63;
        pp[i] = osum(r, d);
    }
    if (tid < R) { pp[RMAX * 64 + tid] = st[0][tid]; pp[RMAX * 65 + tid] = st[1][tid]; }
}

// the S chunk partials of a (kv batch, head) combined in chunk order: thread = (row, dim)
template <int RMAX>
__global__ __launch_bounds__(512) void dec_attn_combine_kernel(const float* __restrict__ part, int S, int R,
                                                               bf16* __restrict__ out, int D) {
    const int h = blockIdx.x, b = blockIdx.y, H = gridDim.x, i = threadIdx.x;
    if (i >= R * 64) return;
    const int r = i >> 6, d = i & 63;
    const float* base = part + (int64_t)(b * H + h) * S * (RMAX * 66);
    float mv[DS_MAXS], lv[DS_MAXS], ov[DS_MAXS];   // every partial load in flight at once (clamped chunk index:
    // unconditional loads, the chunks past S are never used)
#pragma unroll
    for (int c = 0; c < DS_MAXS; ++c) {
        const float* pc = base + min(c, S - 1) * (RMAX * 66);
        mv[c] = pc[RMAX * 64 + r];
        lv[c] = pc[RMAX * 65 + r];
        ov[c] = pc[i];
    }
    float M = -INFINITY;
#pragma unroll
    for (int c = 0; c < DS_MAXS; ++c)
        if (c < S) M = fmaxf(M, mv[c]);
    float o = 0.f, L = 0.f;
#pragma unroll
    for (int c = 0; c < DS_MAXS; ++c)
        if (c < S && lv[c] > 0.f) {
            const float f = __expf(mv[c] - M);
            o = fmaf(f, ov[c], o);
            L = fmaf(f, lv[c], L);
        }
    out[(int64_t)(b * R + r) * D + h * 64 + d] = f2bf(o / L);
}

// Decode-step self-attention in one launch (round 6): workgroup = (row, head) over the row's <= DSA_MAXK cached keys,
// every load of the row issued before the first wait -- the query's 16 dims per lane straight from global (no LDS
// staging), K as NP passes of 64 keys (4 lanes per key, 16 dims each), V as 2 NP groups of 32 keys (8 dims per lane)
// -- so the softmax, P.V and the normalisation need no second launch (the split kernel's combine).  NP = ceil(n_keys
// / 64) is uniform per workgroup and selects a fully unrolled body (unconditional, clamped loads: keys past n_keys
// read key n_keys - 1 and carry weight 0).  Reductions in a fixed order (deterministic).
constexpr int DSA_MAXP = 7;
constexpr int DSA_MAXK = DSA_MAXP * 64;   // 448 = Whisper's max_target_positions
template <int NP>
__device__ __forceinline__ void dec_self_attn_body(const bf16* __restrict__ qr, const bf16* __restrict__ kb,
                                                   const bf16* __restrict__ vb, int nk, int D, bf16* __restrict__ out,
                                                   float* ps, float* red, float (*pv)[64]) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int j = tid >> 2, p = tid & 3;     // scores: key j + 64 u, dims 16 p .. 16 p + 15
    const int dg = tid & 7, kg = tid >> 3;   // P.V: dims 8 dg .. 8 dg + 7, keys kg + 32 u
    const bf16x8 qa = *(const bf16x8*)(qr + p * 16);
    const bf16x8 qb = *(const bf16x8*)(qr + p * 16 + 8);
    bf16x8 ka[NP], kb2[NP], vv[2 * NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        const int jj = min(j + 64 * u, nk - 1);
        ka[u] = *(const bf16x8*)(kb + (int64_t)jj * D + p * 16);
        kb2[u] = *(const bf16x8*)(kb + (int64_t)jj * D + p * 16 + 8);
    }
#pragma unroll
    for (int u = 0; u < 2 * NP; ++u) vv[u] = *(const bf16x8*)(vb + (int64_t)min(kg + 32 * u, nk - 1) * D + dg * 8);
    float sc[NP];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            d = fmaf(bf2f(qa[e]), bf2f(ka[u][e]), d);
            d = fmaf(bf2f(qb[e]), bf2f(kb2[u][e]), d);
        }
        d += xor_lane<1>(d);
        d += xor_lane<2>(d);
        sc[u] = j + 64 * u < nk ? d : -INFINITY;
        mx = fmaxf(mx, sc[u]);
    }
    mx = wave_max_x(mx);
    if (lane == 0) red[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float l = 0.f;
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        const float e = j + 64 * u < nk ? __expf(sc[u] - mx) : 0.f;
        if (p == 0) { ps[j + 64 * u] = e; l += e; }
    }
    l = wave_sum_x(l);
    if (lane == 0) red[4 + w] = l;
    __syncthreads();
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2 * NP; ++u) {
        const float pr = ps[kg + 32 * u];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(pr, bf2f(vv[u][e]), acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {   // the wave's 8 key groups (lane bits 3-5), then the 4 waves in LDS
        float a = acc[e];
        a += xor_lane<8>(a);
        a += xor_lane<16>(a);
        a += __shfl_xor(a, 32, 64);
        if (lane < 8) pv[w][dg * 8 + e] = a;
    }
    __syncthreads();
    if (tid < 64) {
        const float L = (red[4] + red[5]) + (red[6] + red[7]);
        out[tid] = f2bf(((pv[0][tid] + pv[1][tid]) + (pv[2][tid] + pv[3][tid])) / L);
    }
}
__global__ __launch_bounds__(256) void dec_self_attn_kernel(const bf16* __restrict__ q, int ldq,
                                                            const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                            int64_t kv_bstride, int n_keys, bf16* __restrict__ out,
                                                            int D, const int* __restrict__ n_keys_pos, int nk_rows) {
    __shared__ float ps[DSA_MAXK];
    __shared__ float red[8];
    __shared__ float pv[4][64];
    const int r = blockIdx.x, h = blockIdx.y;
    if (n_keys_pos) n_keys = min(n_keys, n_keys_pos[nk_rows ? r : 0] + 1);
    const int nk = max(1, min(n_keys, DSA_MAXK));
    const bf16* qr = q + (int64_t)r * ldq + h * 64;
    const bf16* kb = kc + r * kv_bstride + h * 64;
    const bf16* vb = vc + r * kv_bstride + h * 64;
    bf16* o = out + (int64_t)r * D + h * 64;
    switch ((nk + 63) >> 6) {
        case 1: dec_self_attn_body<1>(qr, kb, vb, nk, D, o, ps, red, pv); break;
        case 2: dec_self_attn_body<2>(qr, kb, vb, nk, D, o, ps, red, pv); break;
        case 3: dec_self_attn_body<3>(qr, kb, vb, nk, D, o, ps, red, pv); break;
        case 4: dec_self_attn_body<4>(qr, kb, vb, nk, D, o, ps, red, pv); break;
        case 5: dec_self_attn_body<5>(qr, kb, vb, nk, D, o, ps, red, pv); break;
        case 6: dec_self_attn_body<6>(qr, kb, vb, nk, D, o, ps, red, pv); break;
        default: dec_self_attn_body<7>(qr, kb, vb, nk, D, o, ps, red, pv); break;
    }
}

// beam reorder: dst[r] = src[src_rows[r]] for the first len positions of every cache row
__global__ void dec_gather_rows_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst, const int* __restrict__ rows,
                                       int64_t row_elems, int64_t copy_elems) {
    const int r = blockIdx.y;
    const bf16* s = src + (int64_t)rows[r] * row_elems;
    bf16* d = dst + (int64_t)r * row_elems;
    for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 8; i < copy_elems; i += (int64_t)gridDim.x * blockDim.x * 8)
        *(bf16x8*)(d + i) = *(const bf16x8*)(s + i);
}

// beam reorder of the whole self-attention K/V cache in place, every layer in one launch: a thread owns
// one 16-byte column (layer, K or V, position chunk) of all B <= 16 rows, loads the B source rows of it,
// then writes the rows whose source differs -- no other thread touches those bytes, so no staging copy
__global__ __launch_bounds__(256) void dec_reorder_kv_kernel(bf16* __restrict__ ks, bf16* __restrict__ vs,
                                                             const int* __restrict__ rows, int B, int64_t layer_elems,
                                                             int64_t row_elems, int64_t chunks) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= chunks) return;
    bf16* base = (blockIdx.z ? vs : ks) + blockIdx.y * layer_elems + i * 8;
    bf16x8 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)   // rows that keep their own history are neither read nor written
        if (r < B && rows[r] != r) v[r] = *(const bf16x8*)(base + min(max(rows[r], 0), B - 1) * row_elems);
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (r < B && rows[r] != r) *(bf16x8*)(base + r * row_elems) = v[r];
}

// log_softmax(logits + bias) and the top-k (k <= 16) per row; ties keep the lower token id
constexpr int TK_MAX = 16;
__global__ __launch_bounds__(1024) void logprob_topk_kernel(const float* __restrict__ logits, int V, int ld,
                                                            const float* __restrict__ bias, int64_t bias_ld, int k,
                                                            float* __restrict__ out_lp, int* __restrict__ out_idx) {
    __shared__ float red[16];
    __shared__ float cand_v[16][TK_MAX];
    __shared__ int cand_i[16][TK_MAX];
    const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const float* x = logits + (int64_t)r * ld;
    if (bias) bias += (int64_t)r * bias_ld;
    // log_softmax over the RAW logits, the logits processors' additive masks after it: HF beam search
    // normalises first (next_token_scores = log_softmax(logits); processed = processors(scores)), so a
    // suppressed token's mass stays in the normaliser
    // two passes over the row, eight loads in flight per thread in each
    constexpr int TK_U = 8;
    float mx = -INFINITY;
    for (int i0 = tid; i0 < V; i0 += 1024 * TK_U) {
        float v[TK_U];
#pragma unroll
        for (int u = 0; u < TK_U; ++u) v[u] = i0 + u * 1024 < V ? x[i0 + u * 1024] : -INFINITY;
#pragma unroll
        for (int u = 0; u < TK_U; ++u) mx = fmaxf(mx, v[u]);
    }
    mx = wave_max(mx);
    if (lane == 0) red[wid] = mx;
    __syncthreads();
    mx = red[0];
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, red[i]);
    __syncthreads();
    // second pass: the normaliser and, per thread, the top-k of its strided slice of logits + bias as a
    // sorted register list (insertion by compare-and-swap down the list: static indices only, so the list
    // stays in VGPRs -- a data-dependent insertion index put it in scratch memory)
    float tv[TK_MAX];
    int ti[TK_MAX];
#pragma unroll
    for (int j = 0; j < TK_MAX; ++j) { tv[j] = -INFINITY; ti[j] = 0x7fffffff; }
    float kth_v = -INFINITY;
    int kth_i = 0x7fffffff;
    float s = 0.f;
    for (int i0 = tid; i0 < V; i0 += 1024 * TK_U) {
        float v[TK_U], bv[TK_U];
#pragma unroll
        for (int u = 0; u < TK_U; ++u) {
            const int i = i0 + u * 1024;
            v[u] = i < V ? x[i] : -INFINITY;
            bv[u] = (bias && i < V) ? bias[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < TK_U; ++u) {
            const int i = i0 + u * 1024;
            if (i >= V) continue;
            s += __expf(v[u] - mx);
            float cv = v[u] + bv[u];
            int ci = i;
            if (cv > kth_v || (cv == kth_v && ci < kth_i)) {
#pragma unroll
                for (int q = 0; q < TK_MAX; ++q) {
                    if (q < k) {
                        const bool b = cv > tv[q] || (cv == tv[q] && ci < ti[q]);
                        const float ov = tv[q];
                        const int oi = ti[q];
                        tv[q] = b ? cv : ov;
                        ti[q] = b ? ci : oi;
                        cv = b ? ov : cv;
                        ci = b ? oi : ci;
                    }
                }
#pragma unroll
                for (int q = 0; q < TK_MAX; ++q)
                    if (q == k - 1) { kth_v = tv[q]; kth_i = ti[q]; }
            }
        }
    }
    s = wave_sum(s);
    if (lane == 0) red[wid] = s;
    __syncthreads();
    float tot = 0.f;
    for (int i = 0; i < 16; ++i) tot += red[i];
    const float lse = mx + logf(tot);
    // wave merge: k rounds of (max value, min index) over the 64 list heads
    int head = 0;
    for (int j = 0; j < k; ++j) {
        float v = head < k ? tv[0] : -INFINITY;
        int id = head < k ? ti[0] : 0x7fffffff;
        float bv = v;
        int bi = id;
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if (lane == 0) { cand_v[wid][j] = bv; cand_i[wid][j] = bi; }
        if (id == bi && head < k) {   // the owner pops its head
#pragma unroll
            for (int q = 0; q < TK_MAX - 1; ++q) { tv[q] = tv[q + 1]; ti[q] = ti[q + 1]; }
            tv[TK_MAX - 1] = -INFINITY;
            ti[TK_MAX - 1] = 0x7fffffff;
            ++head;
        }
    }
    __syncthreads();
    if (wid == 0) {
        // merge the 16 wave lists (each sorted) with the same rule
        int pos = 0;   // lane < 16 owns wave list `lane`
        for (int j = 0; j < k; ++j) {
            float v = (lane < 16 && pos < k) ? cand_v[lane][pos] : -INFINITY;
            int id = (lane < 16 && pos < k) ? cand_i[lane][pos] : 0x7fffffff;
            float bv = v;
            int bi = id;
            for (int o = 32; o > 0; o >>= 1) {
                const float ov = __shfl_xor(bv, o, 64);
                const int oi = __shfl_xor(bi, o, 64);
                if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
            }
            if (lane < 16 && pos < k && id == bi) ++pos;
            if (lane == 0) {
                out_lp[(int64_t)r * k + j] = bv - lse;
                out_idx[(int64_t)r * k + j] = bi;
            }
        }
    }
}


// ---- two-stage top-k: the row split into TK_CHUNKS chunks so ~B x 32 workgroups share the pass
constexpr int TK_CHUNKS = 32;

CBW_DEV bool tk_better(float v, int i, float ov, int oi) { return v > ov || (v == ov && i < oi); }

// insert (v, i) into a lane's sorted register list of k entries (compare-and-swap down: static indices)
CBW_DEV void tk_insert(float (&tv)[TK_MAX], int (&ti)[TK_MAX], int k, float v, int i) {
#pragma unroll
    for (int q = 0; q < TK_MAX; ++q) {
        if (q < k) {
            const bool b = tk_better(v, i, tv[q], ti[q]);
            const float ov = tv[q];
            const int oi = ti[q];
            tv[q] = b ? v : ov;
            ti[q] = b ? i : oi;
            v = b ? ov : v;
            i = b ? oi : i;
        }
    }
}

// k rounds of (max value, min index) over the 64 lanes' list heads; lane 0 receives the merged list
CBW_DEV void tk_wave_merge(float (&tv)[TK_MAX], int (&ti)[TK_MAX], int k, float* mv, int* mi) {
    const int lane = threadIdx.x & 63;
    for (int j = 0; j < k; ++j) {
        float bv = tv[0];
        int bi = ti[0];
        for (int o = 32; o > 0; o >>= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (tk_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
        }
        if (lane == 0) { mv[j] = bv; mi[j] = bi; }
        if (ti[0] == bi && tv[0] == bv) {   // the owner pops its head (ids are unique across lanes)
#pragma unroll
            for (int q = 0; q < TK_MAX - 1; ++q) { tv[q] = tv[q + 1]; ti[q] = ti[q + 1]; }
            tv[TK_MAX - 1] = -INFINITY;
            ti[TK_MAX - 1] = 0x7fffffff;
        }
    }
}

// stage 1: chunk c of row r -> its max m_c, sum exp(x - m_c), and top-k of x + bias.
// part layout per (r, c): [k values | k ids (int bits) | m_c | s_c], stride 2 * TK_MAX + 2 floats
__global__ __launch_bounds__(256) void topk_chunk_kernel(const float* __restrict__ logits, int V, int ld,
                                                         const float* __restrict__ bias, int64_t bias_ld, int k,
                                                         int chunk, float* __restrict__ part) {
    __shared__ float red[4];
    __shared__ float cv[4][TK_MAX];
    __shared__ int ci[4][TK_MAX];
    const int c = blockIdx.x, r = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const float* x = logits + (int64_t)r * ld;
    if (bias) bias += (int64_t)r * bias_ld;
    const int lo = c * chunk, hi = min(V, lo + chunk);
    constexpr int U = 8;
    float tv[TK_MAX];
    int ti[TK_MAX];
#pragma unroll
    for (int j = 0; j < TK_MAX; ++j) { tv[j] = -INFINITY; ti[j] = 0x7fffffff; }
    float mx = -INFINITY, sm = 0.f;
    for (int i0 = lo + tid; i0 < hi; i0 += 256 * U) {
        float v[U], bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * 256;
            v[u] = i < hi ? x[i] : -INFINITY;
            bv[u] = (bias && i < hi) ? bias[i] : 0.f;
        }
        float m2 = mx;
#pragma unroll
        for (int u = 0; u < U; ++u) m2 = fmaxf(m2, v[u]);
        if (m2 > -INFINITY) {
            sm *= __expf(mx - m2);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (i0 + u * 256 < hi) sm += __expf(v[u] - m2);
            mx = m2;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * 256 < hi) {
                const float t = v[u] + bv[u];
                float kv = -INFINITY;
                int ki = 0x7fffffff;
#pragma unroll
                for (int q = 0; q < TK_MAX; ++q)
                    if (q == k - 1) { kv = tv[q]; ki = ti[q]; }
                if (tk_better(t, i0 + u * 256, kv, ki)) tk_insert(tv, ti, k, t, i0 + u * 256);
            }
    }
    // (max, sum) of the chunk: wave then block, rescaled to the chunk max
    float wm = wave_max(mx);
    float ws = wave_sum(mx > -INFINITY ? sm * __expf(mx - wm) : 0.f);
    __shared__ float red_s[4];
    if (lane == 0) { red[wid] = wm; red_s[wid] = ws; }
    tk_wave_merge(tv, ti, k, cv[wid], ci[wid]);
    __syncthreads();
    if (wid != 0) return;
    float lv[TK_MAX];
    int li[TK_MAX];
#pragma unroll
    for (int q = 0; q < TK_MAX; ++q) {   // lane < 4 owns wave list `lane`
        lv[q] = (lane < 4 && q < k) ? cv[lane & 3][q] : -INFINITY;
        li[q] = (lane < 4 && q < k) ? ci[lane & 3][q] : 0x7fffffff;
    }
    float* pp = part + ((int64_t)r * gridDim.x + c) * (2 * TK_MAX + 2);
    __shared__ float outv[TK_MAX];
    __shared__ int outi[TK_MAX];
    tk_wave_merge(lv, li, k, outv, outi);
    if (lane < k) {
        pp[lane] = outv[lane];
        pp[TK_MAX + lane] = __int_as_float(outi[lane]);
    }
    if (lane == 0) {
        float M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        float S = 0.f;
        for (int w = 0; w < 4; ++w) S += red[w] > -INFINITY ? red_s[w] * __expf(red[w] - M) : 0.f;
        pp[2 * TK_MAX] = M;
        pp[2 * TK_MAX + 1] = S;
    }
}

// stage 2: one wave per row merges the chunks (lane c owns chunk c's sorted list) and the normaliser
__global__ __launch_bounds__(64) void topk_merge_kernel(const float* __restrict__ part, int C, int k,
                                                        float* __restrict__ out_lp, int* __restrict__ out_idx) {
    __shared__ float mv[TK_MAX];
    __shared__ int mi[TK_MAX];
    const int r = blockIdx.x, lane = threadIdx.x;
    const float* pp = part + ((int64_t)r * C + min(lane, C - 1)) * (2 * TK_MAX + 2);
    const bool own = lane < C;
    float tv[TK_MAX];
    int ti[TK_MAX];
#pragma unroll
    for (int q = 0; q < TK_MAX; ++q) {
        tv[q] = (own && q < k) ? pp[q] : -INFINITY;
        ti[q] = (own && q < k) ? __float_as_int(pp[TK_MAX + q]) : 0x7fffffff;
    }
    const float m = own ? pp[2 * TK_MAX] : -INFINITY;
    const float sc = own ? pp[2 * TK_MAX + 1] : 0.f;
    const float M = wave_max(m);
    const float S = wave_sum(m > -INFINITY ? sc * __expf(m - M) : 0.f);
    const float lse = M + logf(S);
    tk_wave_merge(tv, ti, k, mv, mi);
    __syncthreads();
    if (lane < k) {
        out_lp[(int64_t)r * k + lane] = mv[lane] - lse;
        out_idx[(int64_t)r * k + lane] = mi[lane];
    }
}

// WhisperTimeStampLogitsProcessor (transformers 4.37.2, generation/logits_process.py; installed 5.15
// copy is identical) for one decoding row per block, as an additive mask on top of the shared
// suppression bias: bias_out[r][i] = bias[i] + (masked ? -inf : 0).
// st[r] = {last_was_timestamp, penultimate_was_timestamp, first allowed timestamp id (timestamps
// below it are masked; = timestamp_begin when none was sampled), at_begin (no token sampled yet)}.
// The "timestamp mass beats every text token" test compares logsumexp over the timestamp tokens with
// the max over text tokens of the masked logits (log_softmax is a common shift of both).
__global__ __launch_bounds__(1024) void timestamp_rules_kernel(const float* __restrict__ logits, int V, int ld,
                                                               const float* __restrict__ bias,
                                                               const int* __restrict__ st, int ts_begin, int no_ts,
                                                               int eos, int max_initial,
                                                               float* __restrict__ bias_out) {
    __shared__ float red[16];
    const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const float* x = logits + (int64_t)r * ld;
    float* o = bias_out + (int64_t)r * V;
    const int last_ts = st[4 * r], penult_ts = st[4 * r + 1], ts_floor = st[4 * r + 2], at_begin = st[4 * r + 3];
    auto mask = [&](int i) -> float {
        float b = bias ? bias[i] : 0.f;
        bool m = i == no_ts;
        if (last_ts) m = m || (penult_ts ? i >= ts_begin : i < eos);
        m = m || (i >= ts_begin && i < ts_floor);
        if (at_begin) m = m || i < ts_begin || (max_initial >= 0 && i > ts_begin + max_initial);
        return m ? -INFINITY : b;
    };
    float mt = -INFINITY, mts = -INFINITY;
    // eight logits and biases in flight per thread: unconditional loads of clamped indices (a load inside the bound
    // check made the compiler wait for each before the next); max is order-independent
    const float* bsrc = bias ? bias : x;
    for (int i0 = tid; i0 < V; i0 += 8 * 1024) {
        float xv[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int ii = min(i0 + u * 1024, V - 1);
            xv[u] = x[ii];
            bv[u] = bsrc[ii];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 1024;
            if (i >= V) break;
            bool m = i == no_ts;
            if (last_ts) m = m || (penult_ts ? i >= ts_begin : i < eos);
            m = m || (i >= ts_begin && i < ts_floor);
            if (at_begin) m = m || i < ts_begin || (max_initial >= 0 && i > ts_begin + max_initial);
            const float v = xv[u] + (m ? -INFINITY : (bias ? bv[u] : 0.f));
            if (i < ts_begin) mt = fmaxf(mt, v);
            else mts = fmaxf(mts, v);
        }
    }
    mt = wave_max(mt);
    mts = wave_max(mts);
    if (lane == 0) red[wid] = mts;
    __syncthreads();
    float m_ts = red[0];
    for (int i = 1; i < 16; ++i) m_ts = fmaxf(m_ts, red[i]);
    __syncthreads();
    if (lane == 0) red[wid] = mt;
    __syncthreads();
    float m_text = red[0];
    for (int i = 1; i < 16; ++i) m_text = fmaxf(m_text, red[i]);
    __syncthreads();
    float s = 0.f;
    if (m_ts > -INFINITY)
        for (int i = ts_begin + tid; i < V; i += 1024) s += __expf(x[i] + mask(i) - m_ts);
    s = wave_sum(s);
    if (lane == 0) red[wid] = s;
    __syncthreads();
    float tot = 0.f;
    for (int i = 0; i < 16; ++i) tot += red[i];
    const float lse_ts = m_ts > -INFINITY ? m_ts + logf(tot) : -INFINITY;
    const bool force_ts = lse_ts > m_text;
    for (int i0 = tid; i0 < V; i0 += 8 * 1024) {   // the biases again, eight in flight (as above)
        float bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) bv[u] = bsrc[min(i0 + u * 1024, V - 1)];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 1024;
            if (i >= V) break;
            bool m = i == no_ts;
            if (last_ts) m = m || (penult_ts ? i >= ts_begin : i < eos);
            m = m || (i >= ts_begin && i < ts_floor);
            if (at_begin) m = m || i < ts_begin || (max_initial >= 0 && i > ts_begin + max_initial);
            o[i] = ((force_ts && i < ts_begin) || m) ? -INFINITY : (bias ? bv[u] : 0.f);
        }
    }
}
}  // namespace

hipError_t cbw_dec_embed(const int* tok, const uint16_t* E, const float* P, int pos, float* h, int B, int D,
                         hipStream_t st, int pos_inc, const int* pos_dev, int pos_rows) {
    hipLaunchKernelGGL(dec_embed_kernel, dim3(B), dim3(256), 0, st, tok, (const bf16*)E, P, pos, pos_inc, h, D, pos_dev,
                       pos_rows);
    return hipGetLastError();
}

hipError_t cbw_dec_kv_prefill(const uint16_t* qkv, uint16_t* kc, uint16_t* vc, int T, int B, int D, int maxlen,
                              hipStream_t st) {
    hipLaunchKernelGGL(dec_kv_prefill_kernel, dim3(T, B), dim3(64), 0, st, (const bf16*)qkv, (bf16*)kc, (bf16*)vc, D,
                       maxlen);
    return hipGetLastError();
}

hipError_t cbw_dec_kv_append(const uint16_t* qkv, uint16_t* kc, uint16_t* vc, int B, int D, int maxlen, int pos,
                             hipStream_t st) {
    hipLaunchKernelGGL(dec_kv_append_kernel, dim3(B), dim3(64), 0, st, (const bf16*)qkv, (bf16*)kc, (bf16*)vc, D, maxlen,
                       pos);
    return hipGetLastError();
}

hipError_t cbw_dec_attention(const uint16_t* q, int ldq, const uint16_t* kc, const uint16_t* vc, int64_t kv_bstride,
                             int n_keys, int rows_per_kv, uint16_t* out, int B, int H, int D, hipStream_t st,
                             int causal) {
    if (n_keys > DA_MAXK || n_keys <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dec_attention_kernel, dim3(B, H), dim3(256), 0, st, (const bf16*)q, ldq, (const bf16*)kc,
                       (const bf16*)vc, kv_bstride, n_keys, rows_per_kv, (bf16*)out, D, causal);
    return hipGetLastError();
}

hipError_t cbw_dec_self_attn(const uint16_t* q, int ldq, const uint16_t* kc, const uint16_t* vc, int64_t kv_bstride,
                             int n_keys, uint16_t* out, int B, int H, int D, hipStream_t st, const int* n_keys_pos,
                             int nk_rows) {
    if (n_keys <= 0 || n_keys > DSA_MAXK || B <= 0 || H * 64 > D) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dec_self_attn_kernel, dim3(B, H), dim3(256), 0, st, (const bf16*)q, ldq, (const bf16*)kc,
                       (const bf16*)vc, kv_bstride, n_keys, (bf16*)out, D, n_keys_pos, nk_rows);
    return hipGetLastError();
}

hipError_t cbw_dec_cross_probs(const uint16_t* q, int ldq, const uint16_t* kc, int n_keys, int T, int D, int head,
                               float* out, hipStream_t st) {
    if (n_keys > DA_MAXK || n_keys <= 0 || T <= 0 || head < 0 || (head + 1) * 64 > D) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dec_cross_probs_kernel, dim3(T), dim3(256), 0, st, (const bf16*)q, ldq, (const bf16*)kc, n_keys,
                       D, head, out);
    return hipGetLastError();
}

int cbw_dec_attn_split_floats(int B, int H) { return B * H * DS_MAXS * 8 * 66; }

hipError_t cbw_dec_attn_split(const uint16_t* q, int ldq, const uint16_t* kc, const uint16_t* vc, int64_t kv_bstride,
                              int n_keys, int rows_per_kv, uint16_t* out, int B, int H, int D, float* part,
                              hipStream_t st, const int* n_keys_pos, int nk_rows) {
    const int S = (n_keys + DS_CHUNK - 1) / DS_CHUNK;
    if (n_keys <= 0 || S > DS_MAXS || rows_per_kv < 1 || rows_per_kv > 8 || B % rows_per_kv) return hipErrorInvalidValue;
    const dim3 grid(S, H, B / rows_per_kv);
#define DS_LAUNCH(RM)                                                                                                 \
    hipLaunchKernelGGL((dec_attn_split_kernel<RM>), grid, dim3(256), 0, st, (const bf16*)q, ldq, (const bf16*)kc,      \
                       (const bf16*)vc, kv_bstride, n_keys, rows_per_kv, (bf16*)out, D, part, n_keys_pos, nk_rows)
    if (rows_per_kv == 1) DS_LAUNCH(1);
    else DS_LAUNCH(8);
#undef DS_LAUNCH
    if (S > 1 || n_keys_pos) {
        const dim3 cgrid(H, B / rows_per_kv);
        if (rows_per_kv == 1)
            hipLaunchKernelGGL(dec_attn_combine_kernel<1>, cgrid, dim3(64), 0, st, part, S, 1, (bf16*)out, D);
        else
            hipLaunchKernelGGL(dec_attn_combine_kernel<8>, cgrid, dim3(64 * rows_per_kv), 0, st, part, S, rows_per_kv,
                               (bf16*)out, D);
    }
    return hipGetLastError();
}

hipError_t cbw_dec_gather_rows(const uint16_t* src, uint16_t* dst, const int* rows, int B, int64_t row_elems,
                               int64_t copy_elems, hipStream_t st) {
    hipLaunchKernelGGL(dec_gather_rows_kernel, dim3(64, B), dim3(256), 0, st, (const bf16*)src, (bf16*)dst, rows,
                       row_elems, copy_elems);
    return hipGetLastError();
}

hipError_t cbw_dec_reorder_kv(uint16_t* ks, uint16_t* vs, const int* rows, int B, int n_layers, int64_t layer_elems,
                              int64_t row_elems, int64_t copy_elems, hipStream_t st) {
    if (B < 1 || B > 16 || copy_elems % 8 || row_elems % 8) return hipErrorInvalidValue;
    const int64_t chunks = copy_elems / 8;
    if (chunks == 0) return hipSuccess;
    hipLaunchKernelGGL(dec_reorder_kv_kernel, dim3((unsigned)((chunks + 255) / 256), n_layers, 2), dim3(256), 0, st,
                       (bf16*)ks, (bf16*)vs, rows, B, layer_elems, row_elems, chunks);
    return hipGetLastError();
}

// ---------------------------------------------------------------- beam bookkeeping on the GPU
// One HF 4.37 beam-search step's next-beam choice (cbw/generate.py BeamProcess.process; transformers
// BeamSearchScorer.process): the B*k candidates beam_scores[r] + lp[r][j] (f64, the host's Python floats),
// sorted by (score desc, row, token), truncated to k; EOS candidates are left to the host's hypotheses (it
// replays this step from the logged candidates); the first B non-EOS candidates become the next beams.  One
// thread: at most 16 x 16 candidates.  Timestamp-rule state per row {n, t1, t2, last_ts} of the tokens at
// positions >= begin (count != 0), gathered from the parent rows, and the cbw_timestamp_rules state derived
// from it.
// One workgroup of 256 threads: candidate c = (row c / k, slot c % k) is ranked by comparing it with every other
// candidate under the total order (score desc, row asc, token asc) -- the ranks < k are exactly the top k the
// bounded insertion sort of the previous single-thread version produced (the order is total: a row's top-k tokens
// are distinct) -- then thread 0 walks those <= 16 entries from LDS.  (The single-thread version indexed private
// arrays dynamically, i.e. through scratch: 43 us per decode step at 5 beams.)
__global__ __launch_bounds__(256) void beam_select_kernel(const float* __restrict__ lp, const int* __restrict__ idx,
                                                          int B, int k, int eos, double* __restrict__ beam_scores,
                                                          double* __restrict__ cand_score, int* __restrict__ cand_row,
                                                          int* __restrict__ cand_tok, int* __restrict__ tokens,
                                                          int* __restrict__ parents, int* __restrict__ ok,
                                                          int* __restrict__ ts_state, int* __restrict__ st_out,
                                                          int ts_begin, int count) {
    __shared__ double c_sc[256];
    __shared__ int c_r[256], c_t[256];
    __shared__ double s_cs[16];
    __shared__ int s_cr[16], s_ct[16], s_st[16][4];
    const int tid = threadIdx.x, nall = B * k;
    if (tid < nall) {
        const int r = tid / k;
        c_sc[tid] = beam_scores[r] + (double)lp[tid];
        c_r[tid] = r;
        c_t[tid] = idx[tid];
    }
    if (tid < 4 * B) s_st[tid >> 2][tid & 3] = ts_state[tid];
    __syncthreads();
    if (tid < nall) {
        const double sc = c_sc[tid];
        const int r = c_r[tid], tok = c_t[tid];
        int rank = 0;
        for (int j = 0; j < nall; ++j) {
            const double sj = c_sc[j];
            const int rj = c_r[j], tj = c_t[j];
            rank += (sj > sc || (sj == sc && (rj < r || (rj == r && tj < tok)))) ? 1 : 0;
        }
        if (rank < k) {
            s_cs[rank] = sc;
            s_cr[rank] = r;
            s_ct[rank] = tok;
        }
    }
    __syncthreads();
    if (tid != 0) return;
    const int n = nall < k ? nall : k;
    int nb = 0;
    double nscore[16];
    int ntok[16], nrow[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {   // fixed trip count: the arrays stay in registers
        if (i < n && nb < B && s_ct[i] != eos) {
#pragma unroll
            for (int b = 0; b < 16; ++b)
                if (b == nb) { nscore[b] = s_cs[i]; ntok[b] = s_ct[i]; nrow[b] = s_cr[i]; }
            ++nb;
        }
    }
    for (int i = 0; i < n; ++i) { cand_score[i] = s_cs[i]; cand_row[i] = s_cr[i]; cand_tok[i] = s_ct[i]; }
    *ok = nb == B ? 1 : 0;
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        if (b >= B) break;
        const int pr = b < nb ? nrow[b] : 0, t = b < nb ? ntok[b] : eos;
        beam_scores[b] = b < nb ? nscore[b] : -1e9;
        tokens[b] = t;
        parents[b] = pr;
        int sn = s_st[pr][0], t1 = s_st[pr][1], t2 = s_st[pr][2], lts = s_st[pr][3];
        if (count) {
            ++sn;
            t2 = t1;
            t1 = t;
            if (t >= ts_begin) lts = t;
        }
        ts_state[4 * b] = sn; ts_state[4 * b + 1] = t1; ts_state[4 * b + 2] = t2; ts_state[4 * b + 3] = lts;
        const int last = sn >= 1 && t1 >= ts_begin, penult = sn < 2 || t2 >= ts_begin;
        st_out[4 * b] = last;
        st_out[4 * b + 1] = penult;
        st_out[4 * b + 2] = lts < 0 ? ts_begin : ((last && !penult) ? lts : lts + 1);
        st_out[4 * b + 3] = sn == 0;
    }
}

hipError_t cbw_beam_select_launch(const float* lp, const int* idx, int B, int k, int eos, double* beam_scores,
                                  double* cand_score, int* cand_row, int* cand_tok, int* tokens, int* parents, int* ok,
                                  int* ts_state, int* st_out, int ts_begin, int count, hipStream_t st) {
    if (B < 1 || B > 16 || k < 1 || k > 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(beam_select_kernel, dim3(1), dim3(256), 0, st, lp, idx, B, k, eos, beam_scores, cand_score,
                       cand_row, cand_tok, tokens, parents, ok, ts_state, st_out, ts_begin, count);
    return hipGetLastError();
}

hipError_t cbw_logprob_topk_launch(const float* logits, int B, int V, int ld, const float* bias, int64_t bias_ld,
                                   int k, float* lp, int* idx, hipStream_t st) {
    if (k < 1 || k > TK_MAX || B < 1 || V < 1) return hipErrorInvalidValue;
    static const bool one_pass = [] { const char* e = getenv("CBW_TOPK_SPLIT"); return e && atoi(e) == 0; }();
    if (one_pass) {
        hipLaunchKernelGGL(logprob_topk_kernel, dim3(B), dim3(1024), 0, st, logits, V, ld, bias, bias_ld, k, lp, idx);
        return hipGetLastError();
    }
    // chunk partials in a per-device scratch owned by the library (grow-only, stream-ordered reuse)
    static thread_local std::map<int, std::pair<float*, size_t>> scratch;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const int C = std::min(TK_CHUNKS, V);
    const int chunk = (V + C - 1) / C;
    const size_t need = (size_t)B * C * (2 * TK_MAX + 2) * sizeof(float);
    auto& sc = scratch[dev];
    if (sc.second < need) {
        if (sc.first) {
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            (void)hipFree(sc.first);
            sc = {nullptr, 0};
        }
        if ((e = hipMalloc((void**)&sc.first, need)) != hipSuccess) return e;
        sc.second = need;
    }
    hipLaunchKernelGGL(topk_chunk_kernel, dim3(C, B), dim3(256), 0, st, logits, V, ld, bias, bias_ld, k, chunk,
                       sc.first);
    hipLaunchKernelGGL(topk_merge_kernel, dim3(B), dim3(64), 0, st, sc.first, C, k, lp, idx);
    return hipGetLastError();
}

hipError_t cbw_timestamp_rules_launch(const float* logits, int B, int V, int ld, const float* bias, const int* state,
                                      int ts_begin, int no_ts, int eos, int max_initial, float* bias_out,
                                      hipStream_t st) {
    hipLaunchKernelGGL(timestamp_rules_kernel, dim3(B), dim3(1024), 0, st, logits, V, ld, bias, state, ts_begin, no_ts,
                       eos, max_initial, bias_out);
    return hipGetLastError();
}

hipError_t cbw_mel_frames(const float* pcm, int n_samples, const float* filters, const float* twiddle, float* logmel,
                          int n_mel, hipStream_t st, int L_pad, int frames) {
    if (L_pad <= 0) L_pad = N_SAMPLES;
    if (frames <= 0) frames = N_FRAMES;
    hipLaunchKernelGGL(mel_frames_kernel, dim3(frames), dim3(256), 0, st, pcm, n_samples, filters, twiddle, logmel,
                       n_mel, L_pad, frames);
    return hipGetLastError();
}

hipError_t cbw_mel_finish(float* logmel, int n_mel, float* scratch, uint16_t* packed, int cpad, hipStream_t st,
                          int frames) {
    const int parts = frames > 0 ? CBW_MEL_LONG_PARTS : 1;   // the 30 s window keeps its single-block max
    if (frames <= 0) frames = N_FRAMES;
    hipLaunchKernelGGL(max_reduce_kernel, dim3(parts), dim3(1024), 0, st, logmel, (int64_t)n_mel * frames, scratch);
    hipLaunchKernelGGL(mel_finish_kernel, dim3(1024), dim3(256), 0, st, logmel, n_mel, scratch, parts, (bf16*)packed,
                       cpad, frames);
    return hipGetLastError();
}

hipError_t cbw_layernorm(const float* x, const float* g, const float* b, uint16_t* y, float* y32, int rows, int D,
                         float eps, hipStream_t st) {
    if (D % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, g, b, (bf16*)y, y32, rows, D, eps);
    return hipGetLastError();
}

hipError_t cbw_attention(const uint16_t* qkv, uint16_t* out, int B, int T, int H, int hd, hipStream_t st) {
    if (hd != 64 || T <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(attention_kernel, dim3((T + 63) / 64, B * H), dim3(256), 0, st, (const bf16*)qkv, (bf16*)out,
                       T, H);
    return hipGetLastError();
}
