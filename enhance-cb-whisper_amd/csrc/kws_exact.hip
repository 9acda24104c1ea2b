// fp32 re-scoring path of the KWS classifier (gfx950): the efficient_kws forward tail in fp32 for a
// selected set of (keyword, utterance) pairs -- the pairs whose bf16 probability lies within a band
// around the decision threshold -- so the spotted-keyword indices follow the reference's fp32
// evaluation (eval-*-comp-*.yaml: precision 32-true) and not bf16 rounding.
//
// Kernels: an fp32 implicit-GEMM conv on the fp32-input MFMA (v_mfma_f32_16x16x4_f32: exact fp32
// products, k-ordered fp32 accumulation; cdna_hip_programming.md §3 "FP32-input MFMA"), the masked
// similarity maps, MaxPool2d(3,2,1), AdaptiveAvgPool + Linear with a scatter into the logits, and the
// projector's layout permute.  Reference: efficient_kws/model.py:143-193 (projector, time projector,
// sim_matrix, masks) and resnet.py:51-58 + HF ResNetModel (the ResNet).
#include <algorithm>

#include "cbw_common.h"
#include "cbw_kernels.h"

namespace {

constexpr int F_BM = 64, F_BN = 64, F_BK = 16, F_PAD = 4;

// A tile: 64 pixels x 16 K (im2col gather), B tile: 64 channels x 16 K, both stored K-major in LDS
// ([k][m] / [k][n]) so each lane's fragment element is one float.  VEC: Cin % 16 == 0, so a K-step
// lies inside one tap and rows load as float4; otherwise (the stem, Cin = L) element-wise.
template <bool VEC>
__global__ __launch_bounds__(256) void conv_f32_kernel(F32ConvArgs a) {
    __shared__ float As[2][F_BK][F_BM + F_PAD];
    __shared__ float Bs[2][F_BK][F_BN + F_PAD];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int nt_n = a.Cout / F_BN;
    const int tm = blockIdx.x / nt_n, tn = blockIdx.x % nt_n;
    const int m0 = tm * F_BM, n0 = tn * F_BN;
    const int K = a.KH * a.KW * a.Cin;
    const int nk = (K + F_BK - 1) / F_BK;
    const int HoWo = a.Ho * a.Wo;

    float ra[4], rb[4];
    auto pix = [&](int m, int& n, int& ih0, int& iw0) {
        n = m / HoWo;
        const int rem = m - n * HoWo;
        const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
        ih0 = oh * a.sh - a.ph;
        iw0 = ow * a.sw - a.pw;
    };
    auto load = [&](int kt) {
        const int k0 = kt * F_BK;
        if constexpr (VEC) {
            const int m = m0 + (tid >> 2), kq = (tid & 3) * 4;
            const int tap = k0 / a.Cin, c0 = k0 - tap * a.Cin;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (m < a.M) {
                int n, ih0, iw0;
                pix(m, n, ih0, iw0);
                const int ih = ih0 + kh, iw = iw0 + kw;
                if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                    v = *(const f32x4*)(a.x + (((int64_t)n * a.H + ih) * a.W + iw) * a.Cin + c0 + kq);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) ra[j] = v[j];
            const int nn = n0 + (tid >> 2);
            const f32x4 w = *(const f32x4*)(a.w + (int64_t)nn * K + k0 + kq);
#pragma unroll
            for (int j = 0; j < 4; ++j) rb[j] = w[j];
        } else {
            const int m = m0 + (tid & 63);
            int n = 0, ih0 = 0, iw0 = 0;
            if (m < a.M) pix(m, n, ih0, iw0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = k0 + (tid >> 6) * 4 + j;
                float v = 0.f;
                if (m < a.M && k < K) {
                    const int tap = k / a.Cin, c = k - tap * a.Cin;
                    const int kh = tap / a.KW, kw = tap - kh * a.KW;
                    const int ih = ih0 + kh, iw = iw0 + kw;
                    if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                        v = a.x[(((int64_t)n * a.H + ih) * a.W + iw) * a.Cin + c];
                }
                ra[j] = v;
                const int nn = n0 + (tid & 63);
                rb[j] = k < K ? a.w[(int64_t)nn * K + k] : 0.f;
            }
        }
    };
    auto store = [&](int buf) {
        if constexpr (VEC) {
            const int m = tid >> 2, kq = (tid & 3) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                As[buf][kq + j][m] = ra[j];
                Bs[buf][kq + j][m] = rb[j];
            }
        } else {
            const int m = tid & 63, kb = (tid >> 6) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                As[buf][kb + j][m] = ra[j];
                Bs[buf][kb + j][m] = rb[j];
            }
        }
    };

    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    load(0);
    store(0);
    __syncthreads();
    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load(kt + 1);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            float av[2], bv[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) av[i] = As[buf][kk * 4 + fq][wm * 32 + i * 16 + fr];
#pragma unroll
            for (int j = 0; j < 2; ++j) bv[j] = Bs[buf][kk * 4 + fq][wn * 32 + j * 16 + fr];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
    // D[m][n]: lane holds rows 4*fq + q (pixels), column fr (channel) of each 16x16 tile
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 32 + j * 16 + fr;
            const float b = a.bias ? a.bias[n] : 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int m = m0 + wm * 32 + i * 16 + fq * 4 + q;
                if (m >= a.M) continue;
                float v = acc[i][j][q] + b;
                if (a.res) v += a.res[(int64_t)m * a.Cout + n];
                if (a.relu) v = fmaxf(v, 0.f);
                a.y[(int64_t)m * a.Cout + n] = v;
            }
        }
}

// maps NHWC f32 [P][Tk][Tu][L]: pair p = keyword sel[p0 + p]; block (p, i) = one keyword frame
__global__ __launch_bounds__(256) void sim_f32_kernel(const float* __restrict__ kwd, const float* __restrict__ kwd_mask,
                                                      const float* __restrict__ utt, const float* __restrict__ utt_mask,
                                                      const int* __restrict__ sel, int p0, float* __restrict__ out,
                                                      int L, int Tk, int Tu, int E) {
    extern __shared__ float kr[];   // [L][E]
    const int p = blockIdx.y, i = blockIdx.x;
    const int k = sel[p0 + p];
    for (int e = threadIdx.x; e < L * E; e += 256) {
        const int l = e / E;
        kr[e] = kwd[(((int64_t)k * L + l) * Tk + i) * E + (e - l * E)];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < Tu; j += 256) {
        for (int l = 0; l < L; ++l) {
            const float* u = utt + ((int64_t)l * Tu + j) * E;
            const float* q = kr + l * E;
            float s = 0.f;
            for (int e = 0; e < E; e += 4) {
                const f32x4 uv = *(const f32x4*)(u + e);
                s = fmaf(q[e], uv[0], s);
                s = fmaf(q[e + 1], uv[1], s);
                s = fmaf(q[e + 2], uv[2], s);
                s = fmaf(q[e + 3], uv[3], s);
            }
            s = s * kwd_mask[((int64_t)k * L + l) * Tk + i] * utt_mask[(int64_t)l * Tu + j];
            out[(((int64_t)p * Tk + i) * Tu + j) * L + l] = s;
        }
    }
}

// E = 64 fast path: one block per (keyword pair, 256 utterance frames); the keyword's [L][Tk][64] rows sit
// in LDS, each thread keeps its utterance frame's 64 floats of one layer in registers and runs the Tk dot
// products against broadcast LDS reads (the utterance is read once per block, not once per keyword frame)
__global__ __launch_bounds__(256) void sim_f32_e64_kernel(const float* __restrict__ kwd, const float* __restrict__ kwd_mask,
                                                          const float* __restrict__ utt, const float* __restrict__ utt_mask,
                                                          const int* __restrict__ sel, int p0, float* __restrict__ out,
                                                          int L, int Tk, int Tu) {
    extern __shared__ float kr[];   // [L][Tk][64], then the keyword mask [L][Tk]
    const int p = blockIdx.y;
    const int k = sel[p0 + p];
    const int n = L * Tk * 64;
    const float* ksrc = kwd + (int64_t)k * n;
    for (int e = threadIdx.x * 4; e < n; e += 256 * 4) *(f32x4*)(kr + e) = *(const f32x4*)(ksrc + e);
    float* km = kr + n;
    for (int e = threadIdx.x; e < L * Tk; e += 256) km[e] = kwd_mask[(int64_t)k * L * Tk + e];
    __syncthreads();
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= Tu) return;
    for (int l = 0; l < L; ++l) {
        f32x4 u[16];
        const float* up = utt + ((int64_t)l * Tu + j) * 64;
#pragma unroll
        for (int q = 0; q < 16; ++q) u[q] = *(const f32x4*)(up + 4 * q);
        const float um = utt_mask[(int64_t)l * Tu + j];
        for (int i = 0; i < Tk; ++i) {
            const float* q = kr + ((int64_t)l * Tk + i) * 64;
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                const f32x4 kv = *(const f32x4*)(q + 4 * c);
                s = fmaf(kv[0], u[c][0], s);
                s = fmaf(kv[1], u[c][1], s);
                s = fmaf(kv[2], u[c][2], s);
                s = fmaf(kv[3], u[c][3], s);
            }
            out[(((int64_t)p * Tk + i) * Tu + j) * L + l] = s * km[l * Tk + i] * um;
        }
    }
}

__global__ void maxpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int H, int W, int C,
                                   int Ho, int Wo) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)N * Ho * Wo * C;
    if (idx >= total) return;
    const int c = idx % C;
    int64_t r = idx / C;
    const int ow = r % Wo;
    r /= Wo;
    const int oh = r % Ho;
    const int n = r / Ho;
    float m = -INFINITY;
    for (int dh = 0; dh < 3; ++dh)
        for (int dw = 0; dw < 3; ++dw) {
            const int ih = oh * 2 - 1 + dh, iw = ow * 2 - 1 + dw;
            if (ih >= 0 && ih < H && iw >= 0 && iw < W) m = fmaxf(m, x[(((int64_t)n * H + ih) * W + iw) * C + c]);
        }
    y[idx] = m;
}

// per pair: mean over HW, Linear(C -> 2); logits row sel[p0 + p]
__global__ __launch_bounds__(256) void pool_fc_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, const int* __restrict__ sel,
                                                          int p0, float* __restrict__ logits, int HW, int C) {
    __shared__ float red[2][4];
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    float s0 = 0.f, s1 = 0.f;
    for (int c = tid; c < C; c += 256) {
        float m = 0.f;
        for (int t0 = 0; t0 < HW; t0 += 8) {   // eight loads in flight, summed in pixel order
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (t0 + u < HW) v[u] = x[((int64_t)p * HW + t0 + u) * C + c];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (t0 + u < HW) m += v[u];
        }
        m /= (float)HW;
        s0 = fmaf(m, w[c], s0);
        s1 = fmaf(m, w[C + c], s1);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (lane == 0) { red[0][wid] = s0; red[1][wid] = s1; }
    __syncthreads();
    if (tid == 0) {
        const int k = sel[p0 + p];
        logits[2 * (int64_t)k] = red[0][0] + red[0][1] + red[0][2] + red[0][3] + b[0];
        logits[2 * (int64_t)k + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3] + b[1];
    }
}

// f32 [B][L][T][D] -> [L][B][T][D]
__global__ void permute_lbtd_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int L, int T, int D) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)B * L * T * D;
    if (idx >= total) return;
    const int d = idx % D;
    int64_t r = idx / D;
    const int t = r % T;
    r /= T;
    const int l = r % L;
    const int b = r / L;
    y[(((int64_t)l * B + b) * T + t) * D + d] = x[idx];
}

unsigned grid1(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

// fp32 [M][C] -> compensated bf16 [M][2C] = [hi | lo] (the input layout of the 3-term split convs,
// CBW_EPI_SPLIT3); 4 channels per thread, C % 4 == 0
__global__ void split3_kernel(const float* __restrict__ x, bf16* __restrict__ y, int64_t M, int C) {
    const int64_t n4 = M * C / 4;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e * 4;
        const int64_t m = i / C;
        const int c = (int)(i - m * C);
        const f32x4 v = *(const f32x4*)(x + i);
        bf16x4 hi, lo;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            hi[q] = f2bf(v[q]);
            lo[q] = f2bf(v[q] - bf2f(hi[q]));
        }
        bf16* yp = y + m * 2 * C + c;
        *(bf16x4*)yp = hi;
        *(bf16x4*)(yp + C) = lo;
    }
}

// per-channel sums of an fp32 NHWC tensor [M][C] (bias-correction statistics, setup only): workgroup g adds the
// sum of its row range to part[g][c] (each (g, c) written by one thread; launches on one stream accumulate).
// C >= 256: one channel per thread, rows serial; C < 256: 256 / C row lanes per channel, reduced through LDS.
constexpr int CS_G = 64;
__global__ void __launch_bounds__(256) channel_sum_kernel(const float* __restrict__ x, int64_t M, int C,
                                                         float* __restrict__ part) {
    __shared__ float red[256];
    const int64_t rows = (M + CS_G - 1) / CS_G;
    const int64_t r0 = blockIdx.x * rows, r1 = r0 + rows < M ? r0 + rows : M;
    float* out = part + (size_t)blockIdx.x * C;
    if (C >= 256) {
        for (int c = threadIdx.x; c < C; c += 256) {
            float s = 0.f;
            for (int64_t r = r0; r < r1; ++r) s += x[r * C + c];
            out[c] += s;
        }
        return;
    }
    const int rl = 256 / C, tc = threadIdx.x % C, tr = threadIdx.x / C;
    float s = 0.f;
    if (tr < rl)
        for (int64_t r = r0 + tr; r < r1; r += rl) s += x[r * C + tc];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < C) {
        float t = 0.f;
        for (int i = 0; i < rl; ++i) t += red[i * C + threadIdx.x];
        out[threadIdx.x] += t;
    }
}

}  // namespace

hipError_t cbw_channel_sum_f32(const float* x, int64_t M, int C, float* part, hipStream_t st) {
    if (M <= 0 || C <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(channel_sum_kernel, dim3(CS_G), dim3(256), 0, st, x, M, C, part);
    return hipGetLastError();
}
int cbw_channel_sum_groups() { return CS_G; }

hipError_t cbw_conv_f32(const F32ConvArgs& a, hipStream_t st) {
    if (a.Cout % F_BN || a.M <= 0) return hipErrorInvalidValue;
    const int nt = ((a.M + F_BM - 1) / F_BM) * (a.Cout / F_BN);
    if (a.Cin % F_BK == 0)
        hipLaunchKernelGGL(conv_f32_kernel<true>, dim3(nt), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(conv_f32_kernel<false>, dim3(nt), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t cbw_sim_f32(const float* kwd, const float* kwd_mask, const float* utt, const float* utt_mask, const int* sel,
                       int p0, int P, float* out, int L, int Tk, int Tu, int E, hipStream_t st) {
    if (E % 4 || P <= 0) return hipErrorInvalidValue;
    const size_t lds64 = (size_t)L * Tk * (64 + 1) * 4;
    if (E == 64 && lds64 <= 128 * 1024) {
        hipLaunchKernelGGL(sim_f32_e64_kernel, dim3((Tu + 255) / 256, P), dim3(256), lds64, st, kwd, kwd_mask, utt,
                           utt_mask, sel, p0, out, L, Tk, Tu);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(sim_f32_kernel, dim3(Tk, P), dim3(256), (size_t)L * E * 4, st, kwd, kwd_mask, utt, utt_mask, sel,
                       p0, out, L, Tk, Tu, E);
    return hipGetLastError();
}

hipError_t cbw_maxpool_f32(const float* x, float* y, int N, int H, int W, int C, int Ho, int Wo, hipStream_t st) {
    hipLaunchKernelGGL(maxpool_f32_kernel, dim3(grid1((int64_t)N * Ho * Wo * C, 256)), dim3(256), 0, st, x, y, N, H, W, C,
                       Ho, Wo);
    return hipGetLastError();
}

hipError_t cbw_pool_fc_f32(const float* x, const float* w, const float* b, const int* sel, int p0, int P, float* logits,
                           int HW, int C, hipStream_t st) {
    hipLaunchKernelGGL(pool_fc_f32_kernel, dim3(P), dim3(256), 0, st, x, w, b, sel, p0, logits, HW, C);
    return hipGetLastError();
}

hipError_t cbw_permute_lbtd_f32(const float* x, float* y, int B, int L, int T, int D, hipStream_t st) {
    hipLaunchKernelGGL(permute_lbtd_f32_kernel, dim3(grid1((int64_t)B * L * T * D, 256)), dim3(256), 0, st, x, y, B, L,
                       T, D);
    return hipGetLastError();
}

hipError_t cbw_split3(const float* x, uint16_t* y, int64_t M, int C, hipStream_t st) {
    if (C % 4) return hipErrorInvalidValue;
    const int64_t n4 = M * C / 4;
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 4096);
    hipLaunchKernelGGL(split3_kernel, dim3(std::max(grid, 1)), dim3(256), 0, st, x, (bf16*)y, M, C);
    return hipGetLastError();
}
