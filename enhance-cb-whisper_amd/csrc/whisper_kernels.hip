// Whisper front end and encoder kernels for gfx950: log-mel spectrogram,
// LayerNorm, and non-causal flash attention (hd = 64).
//
// Reference semantics: HF WhisperFeatureExtractor (called at src/utils.py:186-187,
// src/data/dataset.py:332-339) and HF WhisperEncoder (called at
// src/model/cb_whisper.py:100-104, src/utils.py:188-192); see oracle/mel.py and
// oracle/encoder.py for the restated algorithms these kernels are checked against.
#include "cbw_common.h"
#include "cbw_kernels.h"

namespace {

constexpr int N_FFT = 400, HOP = 160, N_SAMPLES = 480000, N_FRAMES = 3000, N_FREQ = 201;

// ---------------------------------------------------------------- log-mel
// one block per frame: windowed frame -> direct 400-point real DFT (exact twiddle
// table) -> |X|^2 -> mel projection -> log10(max(., 1e-10)).  Input is the raw
// clip; zero-pad/truncate to 30 s and the reflect padding of torch.stft(center=True)
// are applied on the fly.
__global__ __launch_bounds__(256) void mel_frames_kernel(const float* __restrict__ pcm, int n_samples,
                                                         const float* __restrict__ filters,
                                                         const float* __restrict__ twiddle,
                                                         float* __restrict__ logmel, int n_mel) {
    __shared__ float xw[N_FFT];
    __shared__ float tw[2 * N_FFT];
    __shared__ float pw[N_FREQ + 7];
    const int t = blockIdx.x;
    for (int i = threadIdx.x; i < 2 * N_FFT; i += blockDim.x) tw[i] = twiddle[i];
    for (int n = threadIdx.x; n < N_FFT; n += blockDim.x) {
        int j = t * HOP + n - N_FFT / 2;
        if (j < 0) j = -j;
        if (j >= N_SAMPLES) j = 2 * (N_SAMPLES - 1) - j;
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
        logmel[(int64_t)m * N_FRAMES + t] = log10f(fmaxf(s, 1e-10f));
    }
}

__global__ __launch_bounds__(1024) void max_reduce_kernel(const float* __restrict__ x, int n, float* __restrict__ out) {
    __shared__ float red[16];
    float m = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, x[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
        out[0] = r;
    }
}

// (max(x, gmax - 8) + 4) / 4, in place, + time-major bf16 copy [3000][cpad] for the encoder
__global__ void mel_finish_kernel(float* __restrict__ logmel, int n_mel, const float* __restrict__ gmax,
                                  bf16* __restrict__ packed, int cpad) {
    const float floor_v = gmax[0] - 8.0f;
    const int C = packed ? cpad : n_mel;
    const int total = N_FRAMES * C;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int c = i % C, t = i / C;
        float v = 0.f;
        if (c < n_mel) {
            v = (fmaxf(logmel[(int64_t)c * N_FRAMES + t], floor_v) + 4.0f) * 0.25f;
            logmel[(int64_t)c * N_FRAMES + t] = v;
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

}  // namespace

hipError_t cbw_mel_frames(const float* pcm, int n_samples, const float* filters, const float* twiddle, float* logmel,
                          int n_mel, hipStream_t st) {
    hipLaunchKernelGGL(mel_frames_kernel, dim3(N_FRAMES), dim3(256), 0, st, pcm, n_samples, filters, twiddle, logmel,
                       n_mel);
    return hipGetLastError();
}

hipError_t cbw_mel_finish(float* logmel, int n_mel, float* scratch, uint16_t* packed, int cpad, hipStream_t st) {
    hipLaunchKernelGGL(max_reduce_kernel, dim3(1), dim3(1024), 0, st, logmel, n_mel * N_FRAMES, scratch);
    hipLaunchKernelGGL(mel_finish_kernel, dim3(1024), dim3(256), 0, st, logmel, n_mel, scratch, (bf16*)packed, cpad);
    return hipGetLastError();
}

hipError_t cbw_layernorm(const float* x, const float* g, const float* b, uint16_t* y, float* y32, int rows, int D,
                         float eps, hipStream_t st) {
    if (D % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x, g, b, (bf16*)y, y32, rows, D, eps);
    return hipGetLastError();
}

hipError_t cbw_attention(const uint16_t* qkv, uint16_t* out, int B, int T, int H, int hd, hipStream_t st) {
    if (hd != 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(attention_kernel, dim3((T + 63) / 64, B * H), dim3(256), 0, st, (const bf16*)qkv, (bf16*)out,
                       T, H);
    return hipGetLastError();
}
