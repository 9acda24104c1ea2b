// efficient_kws hot-path kernels for gfx950 other than the implicit-GEMM convs:
// projection helpers, masked cosine-similarity maps, ResNet stem / maxpool /
// pool+classifier, and the spotting decision.
//
// Reference semantics (paths relative to the reference src/):
//   projector / time projector     efficient_kws/model.py:87-124, :143-166
//   sim_matrix (eps clamp) + masks efficient_kws/model.py:174-191, :210-218
//   Resnet.forward                 efficient_kws/resnet.py:51-58 (HF ResNetModel)
//   decision                       efficient_kws/model.py:782-799 (softmax[:,1] * ghost >= thr)
//                                  model/cb_whisper.py:128 (argmax == 1)
#include "cbw_common.h"
#include "cbw_kernels.h"

namespace {

// ---------------------------------------------------------------- cast/permute
__global__ void cast_permute_kernel(const float* __restrict__ x, bf16* __restrict__ y, int B, int L, int T, int D) {
    const int64_t total8 = (int64_t)B * L * T * D / 8;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total8; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = i * 8;
        const int d = e % D;
        int64_t r = e / D;
        const int t = r % T; r /= T;
        const int l = r % L;
        const int b = r / L;
        const f32x4 v0 = *(const f32x4*)(x + e), v1 = *(const f32x4*)(x + e + 4);
        bf16x8 o;
        o[0] = f2bf(v0[0]); o[1] = f2bf(v0[1]); o[2] = f2bf(v0[2]); o[3] = f2bf(v0[3]);
        o[4] = f2bf(v1[0]); o[5] = f2bf(v1[1]); o[6] = f2bf(v1[2]); o[7] = f2bf(v1[3]);
        *(bf16x8*)(y + (((int64_t)l * B + b) * T + t) * D + d) = o;
    }
}

// ---------------------------------------------------------------- row L2 normalise
// one wave per row; input rows ordered [L][B][T]
CBW_DEV void store_out(bf16* p, float v) { *p = f2bf(v); }
CBW_DEV void store_out(float* p, float v) { *p = v; }

template <class OutT>
__global__ void normalize_rows_kernel(const void* __restrict__ x, int x_is_f32, OutT* __restrict__ y, int L, int B,
                                      int T, int E, float eps, int permute_lb) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t rows = (int64_t)L * B * T;
    if (row >= rows) return;
    const int t = row % T;
    const int b = (row / T) % B;
    const int l = row / ((int64_t)T * B);
    float ss = 0.f;
    for (int e = lane; e < E; e += 64) {
        const float v = x_is_f32 ? ((const float*)x)[row * E + e] : bf2f(((const bf16*)x)[row * E + e]);
        ss += v * v;
    }
    ss = wave_sum(ss);
    const float inv = 1.0f / fmaxf(sqrtf(ss), eps);
    const int64_t orow = permute_lb ? (((int64_t)b * L + l) * T + t) : row;
    for (int e = lane; e < E; e += 64) {
        const float v = x_is_f32 ? ((const float*)x)[row * E + e] : bf2f(((const bf16*)x)[row * E + e]);
        store_out(y + orow * E + e, v * inv);
    }
}

// ---------------------------------------------------------------- LEF time projector
// block = 64 threads (one wave), thread o = output channel; CH output frames per block.
constexpr int LEF_CH = 16;
template <class OutT>
__global__ __launch_bounds__(64) void lef_time_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ bias, OutT* __restrict__ y,
                                                      const float* __restrict__ mask_in, float* __restrict__ mask_out,
                                                      int L, int B, int T, float eps) {
    constexpr int U = 64;
    constexpr int NC = 2 * LEF_CH + 1;     // conv frames needed
    constexpr int NX = NC + 2;             // input frames needed
    __shared__ float xs[NX][U + 1];
    const int To = (T - 1) / 2 + 1;
    const int o = threadIdx.x;
    const int seq = blockIdx.y;            // l * B + b
    const int l = seq / B, b = seq % B;
    const int to0 = blockIdx.x * LEF_CH;
    if (to0 >= To) return;
    const int tc0 = 2 * to0 - 1;           // first conv frame
    const int tx0 = tc0 - 1;               // first input frame
    const float* xseq = x + (int64_t)seq * T * U;
    for (int f = 0; f < NX; ++f) {
        const int t = tx0 + f;
        xs[f][o] = (t >= 0 && t < T) ? xseq[(int64_t)t * U + o] : 0.f;
    }
    __syncthreads();
    float acc[NC];
    const float bo = bias[l * U + o];
#pragma unroll
    for (int f = 0; f < NC; ++f) acc[f] = bo;
    const float* wl = w + (int64_t)l * 3 * U * U;   // [k][i][o]
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < U; ++i) {
            const float wv = wl[(k * U + i) * U + o];
#pragma unroll
            for (int f = 0; f < NC; ++f) acc[f] = fmaf(wv, xs[f + k][i], acc[f]);
        }
    const int nout = min(LEF_CH, To - to0);
    for (int j = 0; j < nout; ++j) {
        float m = -INFINITY;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int tc = tc0 + 2 * j + d;
            if (tc >= 0 && tc < T) m = fmaxf(m, acc[2 * j + d]);
        }
        const float ss = wave_sum(m * m);
        const float inv = 1.0f / fmaxf(sqrtf(ss), eps);
        const int to = to0 + j;
        store_out(y + (((int64_t)b * L + l) * To + to) * U + o, m * inv);
        if (o == 0 && mask_in) {
            const float* mi = mask_in + ((int64_t)b * L + l) * T;
            float mm = -INFINITY;
            for (int d = -1; d <= 1; ++d) {
                const int t = 2 * to + d;
                if (t >= 0 && t < T) mm = fmaxf(mm, mi[t]);
            }
            mask_out[((int64_t)b * L + l) * To + to] = mm;
        }
    }
}

// ---------------------------------------------------------------- similarity maps
// one wave per 16x16 (tk, tu) tile, all L layers; block = 4 waves along tu.
__global__ __launch_bounds__(256) void sim_maps_kernel(const bf16* __restrict__ kwd, const float* __restrict__ kwd_mask,
                                                       const bf16* __restrict__ utt, const float* __restrict__ utt_mask,
                                                       bf16* __restrict__ out, int K, int L, int Tk, int Tu, int E) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ntu = (Tu + 15) / 16, ntk = (Tk + 15) / 16;
    const int tu_tile = blockIdx.x * 4 + wv;
    if (tu_tile >= ntu) return;
    const int tk_tile = blockIdx.y % ntk;
    const int k = blockIdx.y / ntk;
    const int fr = lane & 15, fq = lane >> 4;
    const int tk_ld = min(tk_tile * 16 + fr, Tk - 1);
    const int tu_ld = min(tu_tile * 16 + fr, Tu - 1);
    f32x4 acc[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) acc[l] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < L; ++l) {
        const bf16* ap = kwd + (((int64_t)k * L + l) * Tk + tk_ld) * E + fq * 8;
        const bf16* bp = utt + ((int64_t)l * Tu + tu_ld) * E + fq * 8;
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
        for (int e0 = 0; e0 < E; e0 += 32) {
            const bf16x8 av = *(const bf16x8*)(ap + e0);
            const bf16x8 bv = *(const bf16x8*)(bp + e0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
        }
        if (l == 0) acc[0] = c; else if (l == 1) acc[1] = c; else if (l == 2) acc[2] = c; else acc[3] = c;
    }
    const int tu = tu_tile * 16 + fr;
    if (tu >= Tu) return;
    float um[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) um[l] = l < L ? utt_mask[(int64_t)l * Tu + tu] : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int tk = tk_tile * 16 + fq * 4 + q;
        if (tk >= Tk) break;
        bf16x4 o;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const float km = l < L ? kwd_mask[((int64_t)k * L + l) * Tk + tk] : 0.f;
            o[l] = f2bf(acc[l][q] * um[l] * km);
        }
        *(bf16x4*)(out + (((int64_t)k * Tk + tk) * Tu + tu) * 4) = o;
    }
}

// Row-strip variant for E <= 64 (LE / LEF projected features): one block per (keyword, 16-row tk tile),
// its 4 waves walk the tu tiles 4 apart.  The keyword fragments and masks are loaded once per wave and
// the utterance fragments (shared by every keyword: L2-resident) once per tile, so a wave streams
// 16 x 16 x 4-channel output tiles back to back instead of paying a launch and a load chain per tile
// (LEF chunk of 500 pairs: 182 us for the one-tile-per-wave kernel above, which stays for large E).
template <int EC>
__global__ __launch_bounds__(256) void sim_maps_rows_kernel(const bf16* __restrict__ kwd,
                                                            const float* __restrict__ kwd_mask,
                                                            const bf16* __restrict__ utt,
                                                            const float* __restrict__ utt_mask,
                                                            bf16* __restrict__ out, int L, int Tk, int Tu) {
    constexpr int E = EC * 32;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int ntu = (Tu + 15) / 16;
    const int tk_tile = blockIdx.x, k = blockIdx.y;
    const int tk_ld = min(tk_tile * 16 + fr, Tk - 1);
    bf16x8 kf[4][EC];
    float km[4][4];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
#pragma unroll
        for (int ec = 0; ec < EC; ++ec)
            kf[l][ec] = l < L ? *(const bf16x8*)(kwd + (((int64_t)k * L + l) * Tk + tk_ld) * E + ec * 32 + fq * 8)
                              : bf16x8{};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int tk = tk_tile * 16 + fq * 4 + q;
            km[l][q] = (l < L && tk < Tk) ? kwd_mask[((int64_t)k * L + l) * Tk + tk] : 0.f;
        }
    }
    bf16* ok = out + (int64_t)k * Tk * Tu * 4;
    // the next tile's utterance fragments and mask are loaded while this tile's MFMAs and stores run
    bf16x8 uf[4][EC];
    float umn[4];
    auto load_tile = [&](int t) {
        const int tu_ld = min(t * 16 + fr, Tu - 1);
#pragma unroll
        for (int l = 0; l < 4; ++l) {
#pragma unroll
            for (int ec = 0; ec < EC; ++ec)
                uf[l][ec] = l < L ? *(const bf16x8*)(utt + ((int64_t)l * Tu + tu_ld) * E + ec * 32 + fq * 8) : bf16x8{};
            umn[l] = l < L ? utt_mask[(int64_t)l * Tu + tu_ld] : 0.f;
        }
    };
    if (wv < ntu) load_tile(wv);
    for (int t = wv; t < ntu; t += 4) {
        const int tu = t * 16 + fr;
        f32x4 c[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            c[l] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ec = 0; ec < EC; ++ec)
                if (l < L) c[l] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[l][ec], uf[l][ec], c[l], 0, 0, 0);
        }
        float um[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) um[l] = umn[l];
        if (t + 4 < ntu) load_tile(t + 4);
        if (tu >= Tu) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int tk = tk_tile * 16 + fq * 4 + q;
            if (tk >= Tk) break;
            bf16x4 o;
#pragma unroll
            for (int l = 0; l < 4; ++l) o[l] = f2bf(c[l][q] * um[l] * km[l][q]);
            *(bf16x4*)(ok + ((int64_t)tk * Tu + tu) * 4) = o;
        }
    }
}

__global__ void sim_to_nchw_kernel(const bf16* __restrict__ maps, float* __restrict__ out, int K, int L, int Tk, int Tu) {
    const int64_t total = (int64_t)K * Tk * Tu;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int tu = i % Tu;
        const int tk = (i / Tu) % Tk;
        const int k = i / ((int64_t)Tu * Tk);
        const bf16x4 v = *(const bf16x4*)(maps + i * 4);
        for (int l = 0; l < L; ++l) out[(((int64_t)k * L + l) * Tk + tk) * Tu + tu] = bf2f(v[l]);
    }
}

// ---------------------------------------------------------------- ResNet stem
// conv7x7 s2 p3, Cin = 4 (NHWC4), Cout = 64, BN folded, ReLU.  GEMM M = pixels, K = 7 kh x (8 kw x 4 c).
// Block 256 threads = 4 waves x 64 rows; per kh stage each thread gathers one row's 8 pixels (64 B).
constexpr int STEM_BM = 256;
constexpr int STEM_BPITCH = 464;   // bytes per weight row in LDS (448 + 16 pad: conflict-free b128 reads)
__global__ __launch_bounds__(256, 2) void stem_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                      const float* __restrict__ bias, bf16* __restrict__ y,
                                                      int N, int H, int W, int Ho, int Wo) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* As = smem;                               // [256][64 B] swizzled
    char* Bs = smem + STEM_BM * 64;                // [64][STEM_BPITCH]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int M = N * Ho * Wo;
    const int nwg = (M + STEM_BM - 1) / STEM_BM;
    const int m0 = xcd_remap(blockIdx.x, nwg) * STEM_BM;
    // weights -> LDS: 64 rows x 448 B = 28 chunks of 16 B per row
    for (int c = tid; c < 64 * 28; c += 256) {
        const int r = c / 28, q = c % 28;
        *(bf16x8*)(Bs + r * STEM_BPITCH + q * 16) = *(const bf16x8*)(w + r * 224 + q * 8);
    }
    // this thread's gather row
    const int m = m0 + tid;
    const bool mok = m < M;
    const int mm = mok ? m : 0;
    const int n = mm / (Ho * Wo), rem = mm % (Ho * Wo);
    const int oh = rem / Wo, ow = rem % Wo;
    const int ih0 = oh * 2 - 3, iw0 = ow * 2 - 3;
    const bf16* xn = x + (int64_t)n * H * W * 4;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
    for (int kh = 0; kh < 7; ++kh) {
        uint2 px[8];
        const int ih = ih0 + kh;
        const bool rok = mok && ih >= 0 && ih < H;
#pragma unroll
        for (int kw = 0; kw < 8; ++kw) {
            const int iw = iw0 + kw;
            px[kw] = (rok && kw < 7 && iw >= 0 && iw < W) ? *(const uint2*)(xn + ((int64_t)ih * W + iw) * 4)
                                                          : make_uint2(0u, 0u);
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int cs = c ^ ((tid >> 2) & 3);
            *(uint4*)(As + tid * 64 + cs * 16) = make_uint4(px[2 * c].x, px[2 * c].y, px[2 * c + 1].x, px[2 * c + 1].y);
        }
        __syncthreads();
        bf16x8 av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = wid * 64 + i * 16 + fr;
            av[i] = *(const bf16x8*)(As + r * 64 + ((fq ^ ((r >> 2) & 3)) * 16));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = *(const bf16x8*)(Bs + (j * 16 + fr) * STEM_BPITCH + kh * 64 + fq * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    constexpr int LD = 68;
    float* Ep = (float*)smem + wid * 64 * LD;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) Ep[(i * 16 + fq * 4 + q) * LD + j * 16 + fr] = acc[i][j][q];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    for (int it = 0; it < 8; ++it) {
        const int p = it * 64 + lane;
        const int r = p >> 3, cg = p & 7;
        const int mo = m0 + wid * 64 + r;
        if (mo >= M) continue;
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(fmaxf(Ep[r * LD + cg * 8 + q] + bias[cg * 8 + q], 0.f));
        *(bf16x8*)(y + (int64_t)mo * 64 + cg * 8) = o;
    }
}

// ---------------------------------------------------------------- fused stem + maxpool
// ResNetEmbeddings (HF modeling_resnet, called by efficient_kws/resnet.py:51-58): conv7x7/s2/p3
// + BN + ReLU followed by MaxPool2d(3, 2, 1), in one pass.  One workgroup = R pooled rows x
// SP_PW pooled columns of one pair:
//   1. the NHWC4 input patch it needs ((4R+7) rows x 24 pixels) is copied to LDS once;
//   2. the stem conv runs as C^T = W . X^T on bf16 MFMA 16x16x32 (output channels on the MFMA
//      rows, so each lane ends with 4 consecutive channels of one stem pixel); the X fragment
//      of stem pixel (sr, sc), tap row kh, k-chunk fq is the 16-byte pair of input pixels at
//      patch (2 sr + kh, 2 sc + 2 fq) -- read straight from the patch, no im2col image;
//   3. bias + ReLU -> bf16 stem tile in LDS, 0 outside the stem image.  That 0 stands in for
//      maxpool's -inf padding exactly: ReLU outputs are >= 0 and every 3x3/s2 window holds at
//      least one in-image pixel;
//   4. 3x3/s2 max over the tile, 16-byte stores of the pooled NHWC output.
// The stem tile never reaches HBM (the unfused path writes and re-reads 1.8 MB per pair).
constexpr int SP_PW = 4;                 // pooled columns per tile
constexpr int SP_SC = 2 * SP_PW + 1;     // stem columns per tile
constexpr int SP_IC = 4 * SP_PW + 8;     // input pixels per patch row (2 * (SP_SC - 1) + 8 taps)
constexpr int SP_SPITCH = 144;           // LDS bytes per stem pixel: 64 ch bf16 + 16 pad (2-px stride hits other banks)
constexpr int SP_RMAX = 19;

__host__ __device__ constexpr int sp_patch_bytes(int R) { return ((4 * R + 7) * SP_IC * 8 + 15) / 16 * 16; }
__host__ __device__ constexpr int sp_lds_bytes(int R) { return sp_patch_bytes(R) + (2 * R + 1) * SP_SC * SP_SPITCH; }

CBW_DEV uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 r = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b));
    return __builtin_bit_cast(uint32_t, r);
}

constexpr int SP_LOADS = ((4 * SP_RMAX + 7) * SP_IC + 255) / 256;   // patch pixels per thread (max)

// V2 (issue diet, SQ r05a: the stem's waves issue VALU 41 % of their cycles against 31 % MFMA busy): the stem tile's
// ReLU on the rounded bf16 pairs (v_cvt_pk_bf16_f32 + v_pk_max_i16: no negative and no -0 entries), so the max-pool
// needs no sign masks, and the pool walks two pooled rows per item (5 stem rows: 15 reads for 2 outputs instead of
// 18).  The pooled values equal V1's bit for bit: ReLU commutes with the round to bf16, and V1 masks the sign of -0.
template <bool V2>
__global__ __launch_bounds__(256, 2) void stem_pool_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                           const float* __restrict__ bias, bf16* __restrict__ y,
                                                           int N, int H, int W, int Hs, int Ws, int Hp, int Wp,
                                                           int R, int nrt, int nct) {
    // Persistent: the block walks tiles blockIdx.x, +G, ... keeping the stem weights in registers, and the next
    // tile's patch loads are in flight while the current tile computes.
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int SR = 2 * R + 1, IR = 4 * R + 7;
    const int npatch = IR * SP_IC;
    char* In = smem;
    char* S = smem + sp_patch_bytes(R);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ntiles = N * nrt * nct;
    const int fr = lane & 15, fq = lane >> 4;
    bf16x8 wv[7][4];
#pragma unroll
    for (int kh = 0; kh < 7; ++kh)
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) wv[kh][jn] = *(const bf16x8*)(w + (jn * 16 + fr) * 224 + kh * 32 + fq * 8);
    f32x4 bv[4];
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) bv[jn] = *(const f32x4*)(bias + jn * 16 + fq * 4);
    // r06: retire the weight / bias loads here.  Without this wait the compiler's counters treat them as possibly
    // pending at the loop header (merged with the preheader), so every tile's first fragment waited vmcnt(4) and its
    // epilogue vmcnt(0) -- i.e. for the NEXT tile's patch loads issued just before: the prefetch was exposed.
    __builtin_amdgcn_s_waitcnt(0);

    auto tile_origin = [&](int t, int& n, int& ph0, int& pw0) {
        t = xcd_remap(t, ntiles);
        n = t / (nrt * nct);
        const int rem = t - n * (nrt * nct);
        const int rt = rem / nct;
        ph0 = rt * R;
        pw0 = (rem - rt * nct) * SP_PW;
    };
    uint2 pv[SP_LOADS];
    auto load_patch = [&](int t) {
        int n, ph0, pw0;
        tile_origin(t, n, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;   // input origin: stem origin (2 p0 - 1) * 2 - 3
        const bf16* xn = x + (int64_t)n * H * W * 4;
#pragma unroll
        for (int j = 0; j < SP_LOADS; ++j) {
            const int i = j * 256 + tid;
            const int r = i / SP_IC, c = i - r * SP_IC;
            const int ih = ir0 + r, iw = ic0 + c;
            pv[j] = make_uint2(0u, 0u);
            if (i < npatch && ih >= 0 && ih < H && iw >= 0 && iw < W) pv[j] = *(const uint2*)(xn + ((int64_t)ih * W + iw) * 4);
        }
    };
    const int G = gridDim.x;
    if ((int)blockIdx.x < ntiles) load_patch(blockIdx.x);
    const int P = SR * SP_SC;
    for (int t = blockIdx.x; t < ntiles; t += G) {
#pragma unroll
        for (int j = 0; j < SP_LOADS; ++j) {
            const int i = j * 256 + tid;
            if (i < npatch) *(uint2*)(In + i * 8) = pv[j];
        }
        __syncthreads();
        if (t + G < ntiles) load_patch(t + G);
        int n, ph0, pw0;
        tile_origin(t, n, ph0, pw0);
        const int sr0 = 2 * ph0 - 1, sc0 = 2 * pw0 - 1;   // stem origin of the tile (maxpool pad row/col)
        // epilogue of fragment f: bias + ReLU -> bf16 stem tile in LDS, 0 outside the stem image
        auto epi = [&](int f, const f32x4 (&acc)[4]) {
            const int pp = f * 16 + fr;
            if (pp >= P) return;
            const int srr = pp / SP_SC, scc = pp - srr * SP_SC;
            const int gr = sr0 + srr, gc = sc0 + scc;
            const bool ok = gr >= 0 && gr < Hs && gc >= 0 && gc < Ws;
#pragma unroll
            for (int jn = 0; jn < 4; ++jn) {
                if constexpr (V2) {
                    typedef float f32x2 __attribute__((ext_vector_type(2)));
                    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
                    typedef short s16x2 __attribute__((ext_vector_type(2)));
                    uint32_t o[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        s16x2 v = __builtin_bit_cast(s16x2, __builtin_convertvector(
                            (f32x2{acc[jn][2 * h] + bv[jn][2 * h], acc[jn][2 * h + 1] + bv[jn][2 * h + 1]}), bf16x2));
                        o[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, s16x2{0, 0}));
                    }
                    *(uint2*)(S + pp * SP_SPITCH + (jn * 16 + fq * 4) * 2) = ok ? make_uint2(o[0], o[1])
                                                                                 : make_uint2(0u, 0u);
                } else {
                    bf16x4 o;
#pragma unroll
                    for (int q = 0; q < 4; ++q) o[q] = f2bf(ok ? fmaxf(acc[jn][q] + bv[jn][q], 0.f) : 0.f);
                    *(bf16x4*)(S + pp * SP_SPITCH + (jn * 16 + fq * 4) * 2) = o;
                }
            }
        };
        auto frag_addr = [&](int f) {
            const int p = min(f * 16 + fr, P - 1);
            const int sr = p / SP_SC, sc = p - sr * SP_SC;
            return In + ((2 * sr) * SP_IC + 2 * sc + 2 * fq) * 8;
        };
        for (int f = wid; f * 16 < P; f += 4) {
            const char* xa = frag_addr(f);
            f32x4 acc[4];
#pragma unroll
            for (int jn = 0; jn < 4; ++jn) acc[jn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kh = 0; kh < 7; ++kh) {
                const bf16x8 xv = *(const bf16x8*)(xa + kh * SP_IC * 8);
#pragma unroll
                for (int jn = 0; jn < 4; ++jn)
                    acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[kh][jn], xv, acc[jn], 0, 0, 0);
            }
            epi(f, acc);
        }
        __syncthreads();
        if constexpr (V2) {
            // item = (pooled row pair, column, 8-channel group): stem rows 4 pr2 .. + 4, each row's 3-column max once
            const int NR2 = (R + 1) / 2;
            for (int i = tid; i < NR2 * SP_PW * 8; i += 256) {
                const int cg = i & 7, pix = i >> 3;
                const int pr2 = pix / SP_PW, pc = pix - pr2 * SP_PW;
                const int pw = pw0 + pc;
                if (pw >= Wp) continue;
                uint4 cm[5];
#pragma unroll
                for (int dr = 0; dr < 5; ++dr) {
                    const int sr = 4 * pr2 + dr;
                    uint4 m = make_uint4(0u, 0u, 0u, 0u);
                    if (sr < SR) {
#pragma unroll
                        for (int dc = 0; dc < 3; ++dc) {
                            const uint4 v = *(const uint4*)(S + (sr * SP_SC + 2 * pc + dc) * SP_SPITCH + cg * 16);
                            m.x = pk_max_u16(m.x, v.x);
                            m.y = pk_max_u16(m.y, v.y);
                            m.z = pk_max_u16(m.z, v.z);
                            m.w = pk_max_u16(m.w, v.w);
                        }
                    }
                    cm[dr] = m;
                }
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int pr = 2 * pr2 + k, ph = ph0 + pr;
                    if (pr >= R || ph >= Hp) break;
                    uint4 m = cm[2 * k];
                    m.x = pk_max_u16(pk_max_u16(m.x, cm[2 * k + 1].x), cm[2 * k + 2].x);
                    m.y = pk_max_u16(pk_max_u16(m.y, cm[2 * k + 1].y), cm[2 * k + 2].y);
                    m.z = pk_max_u16(pk_max_u16(m.z, cm[2 * k + 1].z), cm[2 * k + 2].z);
                    m.w = pk_max_u16(pk_max_u16(m.w, cm[2 * k + 1].w), cm[2 * k + 2].w);
                    *(uint4*)(y + (((int64_t)n * Hp + ph) * Wp + pw) * 64 + cg * 8) = m;
                }
            }
            continue;
        }
        for (int i = tid; i < R * SP_PW * 8; i += 256) {
            const int cg = i & 7, pix = i >> 3;
            const int pr = pix / SP_PW, pc = pix - pr * SP_PW;
            const int ph = ph0 + pr, pw = pw0 + pc;
            if (ph >= Hp || pw >= Wp) continue;
            // every stem value is a ReLU output (>= 0, possibly -0): with the sign bit cleared the
            // bf16 bit patterns order like the values, so the max runs as packed u16 max
            uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int dr = 0; dr < 3; ++dr)
#pragma unroll
                for (int dc = 0; dc < 3; ++dc) {
                    const uint4 v = *(const uint4*)(S + ((2 * pr + dr) * SP_SC + 2 * pc + dc) * SP_SPITCH + cg * 16);
                    m.x = pk_max_u16(m.x, v.x & 0x7fff7fffu);
                    m.y = pk_max_u16(m.y, v.y & 0x7fff7fffu);
                    m.z = pk_max_u16(m.z, v.z & 0x7fff7fffu);
                    m.w = pk_max_u16(m.w, v.w & 0x7fff7fffu);
                }
            *(uint4*)(y + (((int64_t)n * Hp + ph) * Wp + pw) * 64 + cg * 8) = m;
        }
    }
}

// V3 (round 6, VERDICT r05 item 1: the stem at x2.35 of its roofline, VALU 41 % of its issue): V2's tiles, MFMAs,
// roundings, pool and pooled values (bit-identical), for the full-height case (one row tile: Hp <= SP_RMAX, so every
// tile's patch starts at input row -5 and its stem tile at stem row -1), with the per-tile index arithmetic hoisted:
//   * each thread's patch pixels (global offset relative to the tile's first column, row validity) are computed once
//     per launch; a tile adds one offset, and only the first / last column tile of a pair (uniform branch) tests
//     the columns;
//   * a fragment's stem pixel (row, column) steps by +64 pixels = +7 rows, +1 column from the previous fragment of
//     the wave (no divisions in the tile loop);
//   * the stem-image mask of the epilogue only where a fragment can hold an outside pixel (a wave-uniform branch:
//     the stem row -1, a last stem row past the image, the column-edge tiles).
__global__ __launch_bounds__(256, 2) void stem_pool_v3_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                              const float* __restrict__ bias, bf16* __restrict__ y,
                                                              int N, int H, int W, int Hs, int Ws, int Hp, int Wp,
                                                              int R, int nct) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int SR = 2 * R + 1, IR = 4 * R + 7;
    const int npatch = IR * SP_IC;
    char* In = smem;
    char* S = smem + sp_patch_bytes(R);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ntiles = N * nct;
    const int fr = lane & 15, fq = lane >> 4;
    bf16x8 wv[7][4];
#pragma unroll
    for (int kh = 0; kh < 7; ++kh)
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) wv[kh][jn] = *(const bf16x8*)(w + (jn * 16 + fr) * 224 + kh * 32 + fq * 8);
    f32x4 bv[4];
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) bv[jn] = *(const f32x4*)(bias + jn * 16 + fq * 4);
    __builtin_amdgcn_s_waitcnt(0);   // weights / bias retired before the tile loop (see stem_pool_kernel)

    // patch pixel j of this thread (i = 256 j + tid): row i / SP_IC (input row - 5), column (c0 + 16 j) mod SP_IC
    // (256 = 10 x 24 + 16); offset in elements from the tile's pixel (0, ic0); p_ok bit j: in the patch, row in image
    int p_off[SP_LOADS];
    unsigned p_ok = 0;
    const int c0 = tid % SP_IC;
#pragma unroll
    for (int j = 0; j < SP_LOADS; ++j) {
        const int i = j * 256 + tid;
        const int r = i / SP_IC, c = i - r * SP_IC;
        const int ih = r - 5;
        p_off[j] = (ih * W + c) * 4;
        if (i < npatch && ih >= 0 && ih < H) p_ok |= 1u << j;
    }
    const int P = SR * SP_SC;
    const int nfrag = (P + 15) / 16;
    const int sr_first = (wid * 16 + fr) / SP_SC, sc_first = (wid * 16 + fr) % SP_SC;
    // the wave's fragments that may hold a stem row outside the image (row -1, or a row >= Hs): bit per fragment
    unsigned rowmask_frags = 0;
    for (int f = wid, q = 0; f < nfrag; f += 4, ++q) {
        const int pr = min(f * 16 + 15, P - 1) / SP_SC;
        if (f * 16 / SP_SC == 0 || pr - 1 >= Hs) rowmask_frags |= 1u << q;
    }

    auto tile_origin = [&](int t, int& n, int& pw0) {
        t = xcd_remap(t, ntiles);
        n = t / nct;
        pw0 = (t - n * nct) * SP_PW;
    };
    // unconditional loads (an outside pixel reads the pair's first pixel) and a validity mask applied at the LDS
    // store: a load under a branch or a select had the compiler wait for each load right after issuing it
    uint2 pv[SP_LOADS];
    unsigned pv_ok = 0;
    auto load_patch = [&](int t) {
        int n, pw0;
        tile_origin(t, n, pw0);
        const int ic0 = 4 * pw0 - 5;
        const bf16* xn = x + (int64_t)n * H * W * 4;
        const bool edge = ic0 < 0 || ic0 + SP_IC > W;
        pv_ok = p_ok;
        if (edge) {
#pragma unroll
            for (int j = 0; j < SP_LOADS; ++j) {
                int c = c0 + (16 * j) % SP_IC;
                c = c >= SP_IC ? c - SP_IC : c;
                if (ic0 + c < 0 || ic0 + c >= W) pv_ok &= ~(1u << j);
            }
        }
#pragma unroll
        for (int j = 0; j < SP_LOADS; ++j) {
            const int off = ((pv_ok >> j) & 1u) ? p_off[j] + ic0 * 4 : 0;
            pv[j] = *(const uint2*)(xn + off);
        }
    };
    const int G = gridDim.x;
    if ((int)blockIdx.x < ntiles) load_patch(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += G) {
#pragma unroll
        for (int j = 0; j < SP_LOADS; ++j) {
            const int i = j * 256 + tid;
            if (i < npatch) *(uint2*)(In + i * 8) = ((pv_ok >> j) & 1u) ? pv[j] : make_uint2(0u, 0u);
        }
        __syncthreads();
        if (t + G < ntiles) load_patch(t + G);
        int n, pw0;
        tile_origin(t, n, pw0);
        const int sc0 = 2 * pw0 - 1;   // stem column of the tile's first stem column (maxpool pad column)
        const bool cedge = sc0 < 0 || sc0 + SP_SC > Ws;
        int sr = sr_first, sc = sc_first;
        for (int f = wid, q = 0; f < nfrag; f += 4, ++q) {
            const int pp = f * 16 + fr;
            const char* xa = In + ((2 * min(sr, SR - 1)) * SP_IC + 2 * sc + 2 * fq) * 8;
            f32x4 acc[4];
#pragma unroll
            for (int jn = 0; jn < 4; ++jn) acc[jn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kh = 0; kh < 7; ++kh) {
                const bf16x8 xv = *(const bf16x8*)(xa + kh * SP_IC * 8);
#pragma unroll
                for (int jn = 0; jn < 4; ++jn)
                    acc[jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[kh][jn], xv, acc[jn], 0, 0, 0);
            }
            // bias + ReLU on the rounded bf16 pairs (V2's epilogue), 0 outside the stem image
            bool ok = pp < P;
            if (cedge || ((rowmask_frags >> q) & 1u)) {
                const int gr = sr - 1, gc = sc0 + sc;
                ok = ok && gr >= 0 && gr < Hs && gc >= 0 && gc < Ws;
            }
            if (ok) {
                char* sw = S + pp * SP_SPITCH + fq * 8;
#pragma unroll
                for (int jn = 0; jn < 4; ++jn) {
                    typedef float f32x2 __attribute__((ext_vector_type(2)));
                    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
                    typedef short s16x2 __attribute__((ext_vector_type(2)));
                    uint32_t o[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        s16x2 v = __builtin_bit_cast(s16x2, __builtin_convertvector(
                            (f32x2{acc[jn][2 * h] + bv[jn][2 * h], acc[jn][2 * h + 1] + bv[jn][2 * h + 1]}), bf16x2));
                        o[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, s16x2{0, 0}));
                    }
                    *(uint2*)(sw + jn * 32) = make_uint2(o[0], o[1]);
                }
            } else if (pp < P) {
                char* sw = S + pp * SP_SPITCH + fq * 8;
#pragma unroll
                for (int jn = 0; jn < 4; ++jn) *(uint2*)(sw + jn * 32) = make_uint2(0u, 0u);
            }
            sr += 7;   // +64 pixels = 7 x 9 + 1
            if (++sc == SP_SC) {
                sc = 0;
                ++sr;
            }
        }
        __syncthreads();
        // V2's pool: item = (pooled row pair, column, 8-channel group), stem rows 4 pr2 .. + 4
        const int NR2 = (R + 1) / 2;
        for (int i = tid; i < NR2 * SP_PW * 8; i += 256) {
            const int cg = i & 7, pix = i >> 3;
            const int pr2 = pix / SP_PW, pc = pix - pr2 * SP_PW;
            const int pw = pw0 + pc;
            if (pw >= Wp) continue;
            uint4 cm[5];
#pragma unroll
            for (int dr = 0; dr < 5; ++dr) {
                const int srr = 4 * pr2 + dr;
                uint4 m = make_uint4(0u, 0u, 0u, 0u);
                if (srr < SR) {
#pragma unroll
                    for (int dc = 0; dc < 3; ++dc) {
                        const uint4 v = *(const uint4*)(S + (srr * SP_SC + 2 * pc + dc) * SP_SPITCH + cg * 16);
                        m.x = pk_max_u16(m.x, v.x);
                        m.y = pk_max_u16(m.y, v.y);
                        m.z = pk_max_u16(m.z, v.z);
                        m.w = pk_max_u16(m.w, v.w);
                    }
                }
                cm[dr] = m;
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int pr = 2 * pr2 + k, ph = pr;
                if (pr >= R || ph >= Hp) break;
                uint4 m = cm[2 * k];
                m.x = pk_max_u16(pk_max_u16(m.x, cm[2 * k + 1].x), cm[2 * k + 2].x);
                m.y = pk_max_u16(pk_max_u16(m.y, cm[2 * k + 1].y), cm[2 * k + 2].y);
                m.z = pk_max_u16(pk_max_u16(m.z, cm[2 * k + 1].z), cm[2 * k + 2].z);
                m.w = pk_max_u16(pk_max_u16(m.w, cm[2 * k + 1].w), cm[2 * k + 2].w);
                *(uint4*)(y + (((int64_t)n * Hp + ph) * Wp + pw) * 64 + cg * 8) = m;
            }
        }
    }
}

// ---------------------------------------------------------------- fused stem + maxpool, 16 channels
// The original CB-Whisper classifier (model/model.py:55-58: Resnet(num_channels=12)) reads 12 layers
// of similarity maps.  Input NHWC16 (channels 12..15 zero), weights [64][7][8][16] (kw padded to 8,
// BN folded): K per kernel row = 8 taps x 16 ch = 4 MFMA k-steps.  Same tile/pool scheme as
// stem_pool_kernel, but the weights (112 KB) live in LDS with a padded row pitch (conflict-free
// 16-lane A reads) and each wave computes two pixel fragments per weight read.
//
// X3 (the compensated re-scoring tier's stem): input channels [x_hi | x_hi | x_lo | 0] of the fp32 maps
// (maps_split16_kernel), weights [w_hi | w_lo | w_hi | 0] (load_stem16_x3), so one pass accumulates
// x_hi.w_hi + x_hi.w_lo + x_lo.w_hi in fp32; the stem tile stays fp32 in LDS, the max-pool runs on fp32 and
// the pooled value leaves split as [hi | lo] (128 bf16 per pixel, the tier's activation layout).
constexpr int S16_RMAX = 6;
constexpr int S16_RMAX_X3 = 5;                    // fp32 stem tile: 272-byte pixel pitch
constexpr int S16_WPITCH = 7 * 8 * 16 * 2 + 16;   // 1808 bytes per output channel
constexpr int S16_WBYTES = 64 * S16_WPITCH;       // 115712
constexpr int SP_SPITCH32 = 64 * 4 + 16;          // fp32 stem pixel pitch (X3)
__host__ __device__ constexpr int s16_patch_bytes(int R) { return (4 * R + 7) * SP_IC * 32; }
__host__ __device__ constexpr int s16_lds_bytes(int R, bool x3 = false) {
    return S16_WBYTES + s16_patch_bytes(R) + (2 * R + 1) * SP_SC * (x3 ? SP_SPITCH32 : SP_SPITCH);
}
static_assert(s16_lds_bytes(S16_RMAX) <= 163840 && s16_lds_bytes(S16_RMAX_X3, true) <= 163840, "LDS budget");
constexpr int S16_LOADS = ((4 * S16_RMAX + 7) * SP_IC * 2 + 255) / 256;   // 16-byte patch chunks per thread

template <bool X3>
__global__ __launch_bounds__(256, 1) void stem16_pool_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                             const float* __restrict__ bias, bf16* __restrict__ y,
                                                             int N, int H, int W, int Hs, int Ws, int Hp, int Wp,
                                                             int R, int nrt, int nct) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int SR = 2 * R + 1, IR = 4 * R + 7;
    const int nchunk = IR * SP_IC * 2;
    char* Wl = smem;
    char* In = smem + S16_WBYTES;
    char* S = In + s16_patch_bytes(R);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ntiles = N * nrt * nct;
    const int fr = lane & 15, fq = lane >> 4;
    for (int i = tid; i < 64 * 112; i += 256) {   // weights -> LDS: 112 chunks of 16 B per channel
        const int co = i / 112, c = i - co * 112;
        *(bf16x8*)(Wl + co * S16_WPITCH + c * 16) = *(const bf16x8*)(w + co * 896 + c * 8);
    }
    f32x4 bv[4];
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) bv[jn] = *(const f32x4*)(bias + jn * 16 + fq * 4);
    __builtin_amdgcn_s_waitcnt(0);   // bias retired before the loop (see stem_pool_kernel)

    auto tile_origin = [&](int t, int& n, int& ph0, int& pw0) {
        t = xcd_remap(t, ntiles);
        n = t / (nrt * nct);
        const int rem = t - n * (nrt * nct);
        const int rt = rem / nct;
        ph0 = rt * R;
        pw0 = (rem - rt * nct) * SP_PW;
    };
    uint4 pv[S16_LOADS];
    auto load_patch = [&](int t) {
        int n, ph0, pw0;
        tile_origin(t, n, ph0, pw0);
        const int ir0 = 4 * ph0 - 5, ic0 = 4 * pw0 - 5;
        const bf16* xn = x + (int64_t)n * H * W * 16;
#pragma unroll
        for (int j = 0; j < S16_LOADS; ++j) {
            const int i = j * 256 + tid;
            const int px = i >> 1, half = i & 1;
            const int r = px / SP_IC, c = px - r * SP_IC;
            const int ih = ir0 + r, iw = ic0 + c;
            pv[j] = make_uint4(0u, 0u, 0u, 0u);
            if (i < nchunk && ih >= 0 && ih < H && iw >= 0 && iw < W)
                pv[j] = *(const uint4*)(xn + ((int64_t)ih * W + iw) * 16 + half * 8);
        }
    };
    const int G = gridDim.x;
    if ((int)blockIdx.x < ntiles) load_patch(blockIdx.x);
    const int P = SR * SP_SC;
    const int F = (P + 15) / 16;
    for (int t = blockIdx.x; t < ntiles; t += G) {
#pragma unroll
        for (int j = 0; j < S16_LOADS; ++j) {
            const int i = j * 256 + tid;
            if (i < nchunk) *(uint4*)(In + i * 16) = pv[j];
        }
        __syncthreads();
        if (t + G < ntiles) load_patch(t + G);
        int n, ph0, pw0;
        tile_origin(t, n, ph0, pw0);
        const int sr0 = 2 * ph0 - 1, sc0 = 2 * pw0 - 1;
        for (int f0 = wid * 2; f0 < F; f0 += 8) {    // two fragments per pass
            f32x4 acc[2][4];
            const char* xa[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
#pragma unroll
                for (int jn = 0; jn < 4; ++jn) acc[u][jn] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int p = min((f0 + u) * 16 + fr, P - 1);
                const int sr = p / SP_SC, sc = p - sr * SP_SC;
                xa[u] = In + ((2 * sr) * SP_IC + 2 * sc + (fq >> 1)) * 32 + (fq & 1) * 16;
            }
            const char* wa = Wl + fr * S16_WPITCH + fq * 16;
            for (int kh = 0; kh < 7; ++kh) {
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    bf16x8 wv[4];
#pragma unroll
                    for (int jn = 0; jn < 4; ++jn) wv[jn] = *(const bf16x8*)(wa + jn * 16 * S16_WPITCH + (kh * 128 + ks * 32) * 2);
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const bf16x8 xv = *(const bf16x8*)(xa[u] + (kh * SP_IC + 2 * ks) * 32);
#pragma unroll
                        for (int jn = 0; jn < 4; ++jn)
                            acc[u][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[jn], xv, acc[u][jn], 0, 0, 0);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int pp = (f0 + u) * 16 + fr;
                if (f0 + u >= F || pp >= P) continue;
                const int srr = pp / SP_SC, scc = pp - srr * SP_SC;
                const int gr = sr0 + srr, gc = sc0 + scc;
                const bool ok = gr >= 0 && gr < Hs && gc >= 0 && gc < Ws;
#pragma unroll
                for (int jn = 0; jn < 4; ++jn) {
                    if (X3) {
                        f32x4 o;
#pragma unroll
                        for (int q = 0; q < 4; ++q) o[q] = ok ? fmaxf(acc[u][jn][q] + bv[jn][q], 0.f) : 0.f;
                        *(f32x4*)(S + pp * SP_SPITCH32 + (jn * 16 + fq * 4) * 4) = o;
                    } else {
                        bf16x4 o;
#pragma unroll
                        for (int q = 0; q < 4; ++q) o[q] = f2bf(ok ? fmaxf(acc[u][jn][q] + bv[jn][q], 0.f) : 0.f);
                        *(bf16x4*)(S + pp * SP_SPITCH + (jn * 16 + fq * 4) * 2) = o;
                    }
                }
            }
        }
        __syncthreads();
        if (X3) {   // fp32 3x3/s2 max (ReLU outputs >= 0, 0 = padding as above), then the [hi | lo] split
            for (int i = tid; i < R * SP_PW * 16; i += 256) {
                const int cg = i & 15, pix = i >> 4;
                const int pr = pix / SP_PW, pc = pix - pr * SP_PW;
                const int ph = ph0 + pr, pw = pw0 + pc;
                if (ph >= Hp || pw >= Wp) continue;
                f32x4 m = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int dr = 0; dr < 3; ++dr)
#pragma unroll
                    for (int dc = 0; dc < 3; ++dc) {
                        const f32x4 v = *(const f32x4*)(S + ((2 * pr + dr) * SP_SC + 2 * pc + dc) * SP_SPITCH32 + cg * 16);
#pragma unroll
                        for (int q = 0; q < 4; ++q) m[q] = fmaxf(m[q], v[q]);
                    }
                bf16x4 hi, lo;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    hi[q] = f2bf(m[q]);
                    lo[q] = f2bf(m[q] - bf2f(hi[q]));
                }
                bf16* yp = y + (((int64_t)n * Hp + ph) * Wp + pw) * 128 + cg * 4;
                *(bf16x4*)yp = hi;
                *(bf16x4*)(yp + 64) = lo;
            }
            __syncthreads();
            continue;
        }
        for (int i = tid; i < R * SP_PW * 8; i += 256) {
            const int cg = i & 7, pix = i >> 3;
            const int pr = pix / SP_PW, pc = pix - pr * SP_PW;
            const int ph = ph0 + pr, pw = pw0 + pc;
            if (ph >= Hp || pw >= Wp) continue;
            uint4 m = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (int dr = 0; dr < 3; ++dr)
#pragma unroll
                for (int dc = 0; dc < 3; ++dc) {
                    const uint4 v = *(const uint4*)(S + ((2 * pr + dr) * SP_SC + 2 * pc + dc) * SP_SPITCH + cg * 16);
                    m.x = pk_max_u16(m.x, v.x & 0x7fff7fffu);
                    m.y = pk_max_u16(m.y, v.y & 0x7fff7fffu);
                    m.z = pk_max_u16(m.z, v.z & 0x7fff7fffu);
                    m.w = pk_max_u16(m.w, v.w & 0x7fff7fffu);
                }
            *(uint4*)(y + (((int64_t)n * Hp + ph) * Wp + pw) * 64 + cg * 8) = m;
        }
        __syncthreads();   // S and In are rewritten by the next tile
    }
}

// ---------------------------------------------------------------- CB-Whisper similarity resize
// cb_whisper.py:189-210: per keyword k and layer l the similarity matrix sim[l][off_k + t][u]
// (t < len_k, u < Tu; rows of the per-layer GEMM keyword x utterance, fp32) is resized to
// (Ho, Wo) by torchvision resize(antialias=False) = bilinear, align_corners=False (PyTorch
// upsample_bilinear2d: scale = in/out, src = max(scale (dst + 0.5) - 0.5, 0), neighbour
// clamped to the last row/column).  Output NHWC16 bf16 [K][Ho][Wo][16], channels >= L zero.
__global__ void sim_resize_kernel(const float* __restrict__ sim, int64_t layer_stride, int ld,
                                  const int* __restrict__ off, int k0, int K, int L, int Tu, int Ho, int Wo,
                                  bf16* __restrict__ out) {
    const int64_t total = (int64_t)K * Ho * Wo;
    const float sx = (float)Tu / (float)Wo;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(i % Wo);
        const int64_t r = i / Wo;
        const int ii = (int)(r % Ho);
        const int k = (int)(r / Ho);
        const int row0 = off[k0 + k] - off[k0];
        const int Tk = off[k0 + k + 1] - off[k0 + k];
        const float sy = (float)Tk / (float)Ho;
        const float fy = fmaxf(sy * (ii + 0.5f) - 0.5f, 0.f);
        const float fx = fmaxf(sx * (j + 0.5f) - 0.5f, 0.f);
        const int y0 = (int)fy, x0 = (int)fx;
        const int y1 = y0 + (y0 < Tk - 1 ? 1 : 0), x1 = x0 + (x0 < Tu - 1 ? 1 : 0);
        const float ly1 = fy - y0, ly0 = 1.f - ly1, lx1 = fx - x0, lx0 = 1.f - lx1;
        bf16x8 o0, o1;
#pragma unroll
        for (int l = 0; l < 16; ++l) {
            float v = 0.f;
            if (l < L) {
                const float* s = sim + l * layer_stride + (int64_t)row0 * ld;
                v = ly0 * (lx0 * s[(int64_t)y0 * ld + x0] + lx1 * s[(int64_t)y0 * ld + x1]) +
                    ly1 * (lx0 * s[(int64_t)y1 * ld + x0] + lx1 * s[(int64_t)y1 * ld + x1]);
            }
            if (l < 8) o0[l] = f2bf(v); else o1[l - 8] = f2bf(v);
        }
        *(bf16x8*)(out + i * 16) = o0;
        *(bf16x8*)(out + i * 16 + 8) = o1;
    }
}

__global__ void nchw_to_nhwc16_kernel(const float* __restrict__ x, bf16* __restrict__ y, int K, int L, int H, int W) {
    const int64_t total = (int64_t)K * H * W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t hw = i % ((int64_t)H * W);
        const int64_t k = i / ((int64_t)H * W);
        bf16x8 o0, o1;
#pragma unroll
        for (int l = 0; l < 16; ++l) {
            const float v = l < L ? x[(k * L + l) * H * W + hw] : 0.f;
            if (l < 8) o0[l] = f2bf(v); else o1[l - 8] = f2bf(v);
        }
        *(bf16x8*)(y + i * 16) = o0;
        *(bf16x8*)(y + i * 16 + 8) = o1;
    }
}

// ---------------------------------------------------------------- maxpool 3x3 s2 p1
__global__ void maxpool3s2_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H, int W, int C, int Ho,
                                  int Wo) {
    const int cg = C / 8;
    const int64_t total = (int64_t)N * Ho * Wo * cg;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (i % cg) * 8;
        int64_t p = i / cg;
        const int ow = p % Wo; p /= Wo;
        const int oh = p % Ho;
        const int n = p / Ho;
        float m[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) m[q] = -INFINITY;
        for (int dh = -1; dh <= 1; ++dh) {
            const int ih = oh * 2 + dh;
            if (ih < 0 || ih >= H) continue;
            for (int dw = -1; dw <= 1; ++dw) {
                const int iw = ow * 2 + dw;
                if (iw < 0 || iw >= W) continue;
                const bf16x8 v = *(const bf16x8*)(x + (((int64_t)n * H + ih) * W + iw) * C + c);
#pragma unroll
                for (int q = 0; q < 8; ++q) m[q] = fmaxf(m[q], bf2f(v[q]));
            }
        }
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(m[q]);
        *(bf16x8*)(y + i * 8) = o;
    }
}

// ---------------------------------------------------------------- avgpool + classifier
template <int UNR>
__global__ __launch_bounds__(256) void pool_fc_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ b, float* __restrict__ logits, int HW,
                                                      int C) {
    __shared__ float red[2][4];
    const int n = blockIdx.x;
    float p0 = 0.f, p1 = 0.f;
    for (int c = threadIdx.x * 8; c < C; c += blockDim.x * 8) {
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        // UNR pixels' loads in flight per lane, summed in pixel order (the same bits as a serial loop)
        for (int t0 = 0; t0 < HW; t0 += UNR) {
            bf16x8 v[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u)
                if (t0 + u < HW) v[u] = *(const bf16x8*)(x + ((int64_t)n * HW + t0 + u) * C + c);
#pragma unroll
            for (int u = 0; u < UNR; ++u)
                if (t0 + u < HW)
#pragma unroll
                    for (int q = 0; q < 8; ++q) s[q] += bf2f(v[u][q]);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float mean = s[q] / (float)HW;
            p0 = fmaf(mean, w[c + q], p0);
            p1 = fmaf(mean, w[C + c + q], p1);
        }
    }
    p0 = wave_sum(p0);
    p1 = wave_sum(p1);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) { red[0][wid] = p0; red[1][wid] = p1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a0 = b[0], a1 = b[1];
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { a0 += red[0][i]; a1 += red[1][i]; }
        logits[n * 2] = a0;
        logits[n * 2 + 1] = a1;
    }
}

// ---------------------------------------------------------------- decision + ordered compaction
__global__ __launch_bounds__(1024) void spot_kernel(const float* __restrict__ logits, const float* __restrict__ ghost,
                                                    int K, float thr, float band, int mode,
                                                    float* __restrict__ prob_out, int* __restrict__ idx_out,
                                                    int* __restrict__ n_out) {
    __shared__ int wave_cnt[16];
    __shared__ int base_s;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) base_s = 0;
    __syncthreads();
    for (int k0 = 0; k0 < K; k0 += 1024) {
        const int k = k0 + tid;
        bool hit = false;
        if (k < K) {
            const float l0 = logits[2 * k], l1 = logits[2 * k + 1];
            float p = 1.0f / (1.0f + expf(l0 - l1));
            if (ghost) p *= ghost[k];
            if (prob_out) prob_out[k] = p;
            // mode 0: threshold decision; 1: argmax; 2: the near-threshold band |p - thr| <= band; 3: the band
            // scaled by the pair's logit magnitude, |p - thr| <= band max(|l0|, |l1|)
            hit = mode == 1   ? (l1 > l0)
                  : mode == 2 ? (fabsf(p - thr) <= band)
                  : mode == 3 ? (fabsf(p - thr) <= band * fmaxf(fabsf(l0), fabsf(l1)))
                              : (p >= thr);
        }
        const unsigned long long bal = __ballot(hit);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wave_cnt[wid] = __popcll(bal);
        __syncthreads();
        int off = base_s;
        for (int i = 0; i < wid; ++i) off += wave_cnt[i];
        if (hit) idx_out[off + before] = k;
        __syncthreads();
        if (tid == 0) {
            int s = 0;
            for (int i = 0; i < 16; ++i) s += wave_cnt[i];
            base_s += s;
        }
        __syncthreads();
    }
    if (tid == 0) *n_out = base_s;
}

// NCHW f32 [K][L][H][W] -> NHWC4 bf16 [K][H][W][4] (channels >= L zero)
__global__ void nchw_to_nhwc4_kernel(const float* __restrict__ x, bf16* __restrict__ y, int K, int L, int H, int W) {
    const int64_t total = (int64_t)K * H * W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t hw = i % ((int64_t)H * W);
        const int64_t k = i / ((int64_t)H * W);
        bf16x4 o;
#pragma unroll
        for (int l = 0; l < 4; ++l) o[l] = f2bf(l < L ? x[(k * L + l) * H * W + hw] : 0.f);
        *(bf16x4*)(y + i * 4) = o;
    }
}

// in-place x / ||x||_2 per row (no eps: cb_whisper.py:106, utils.py:195), one wave per row
__global__ __launch_bounds__(256) void l2norm_rows_f32_kernel(float* __restrict__ x, int64_t rows, int E) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    float* r = x + row * E;
    float ss = 0.f;
    for (int e = lane; e < E; e += 64) ss += r[e] * r[e];
    const float inv = 1.0f / sqrtf(wave_sum(ss));
    for (int e = lane; e < E; e += 64) r[e] *= inv;
}

inline int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

hipError_t cbw_cast_permute_lbtd(const float* x, uint16_t* y, int B, int L, int T, int D, hipStream_t st) {
    hipLaunchKernelGGL(cast_permute_kernel, dim3(grid_for((int64_t)B * L * T * D / 8, 256)), dim3(256), 0, st, x,
                       (bf16*)y, B, L, T, D);
    return hipGetLastError();
}

hipError_t cbw_normalize_rows(const void* x, int x_is_f32, void* y, int y_is_f32, int L, int B, int T, int E,
                              float eps, int permute_lb, hipStream_t st) {
    const int64_t rows = (int64_t)L * B * T;
    if (y_is_f32)
        hipLaunchKernelGGL(normalize_rows_kernel<float>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, x,
                           x_is_f32, (float*)y, L, B, T, E, eps, permute_lb);
    else
        hipLaunchKernelGGL(normalize_rows_kernel<bf16>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, x,
                           x_is_f32, (bf16*)y, L, B, T, E, eps, permute_lb);
    return hipGetLastError();
}

hipError_t cbw_nchw_to_nhwc4(const float* x, uint16_t* y, int K, int L, int H, int W, hipStream_t st) {
    if (L > 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nchw_to_nhwc4_kernel, dim3(grid_for((int64_t)K * H * W, 256)), dim3(256), 0, st, x, (bf16*)y,
                       K, L, H, W);
    return hipGetLastError();
}

hipError_t cbw_l2norm_rows_f32(float* x, int64_t rows, int E, hipStream_t st) {
    hipLaunchKernelGGL(l2norm_rows_f32_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, x, rows, E);
    return hipGetLastError();
}

hipError_t cbw_lef_time_project(const float* x, const float* w, const float* b, void* y, int y_is_f32,
                                const float* mask_in, float* mask_out, int L, int B, int T, int U, float eps,
                                hipStream_t st) {
    if (U != 64) return hipErrorInvalidValue;
    const int To = (T - 1) / 2 + 1;
    if (y_is_f32)
        hipLaunchKernelGGL(lef_time_kernel<float>, dim3((To + LEF_CH - 1) / LEF_CH, L * B), dim3(64), 0, st, x, w, b,
                           (float*)y, mask_in, mask_out, L, B, T, eps);
    else
        hipLaunchKernelGGL(lef_time_kernel<bf16>, dim3((To + LEF_CH - 1) / LEF_CH, L * B), dim3(64), 0, st, x, w, b,
                           (bf16*)y, mask_in, mask_out, L, B, T, eps);
    return hipGetLastError();
}

hipError_t cbw_sim_maps(const uint16_t* kwd, const float* kwd_mask, const uint16_t* utt, const float* utt_mask,
                        uint16_t* out, int K, int L, int Tk, int Tu, int E, hipStream_t st) {
    if (L > 4 || E % 32 != 0) return hipErrorInvalidValue;
    const int ntu = (Tu + 15) / 16, ntk = (Tk + 15) / 16;
    if (K <= 0 || Tk <= 0 || Tu <= 0) return hipSuccess;
    if ((E == 32 || E == 64) && K < 65536) {
        if (E == 64)
            hipLaunchKernelGGL(sim_maps_rows_kernel<2>, dim3(ntk, K), dim3(256), 0, st, (const bf16*)kwd, kwd_mask,
                               (const bf16*)utt, utt_mask, (bf16*)out, L, Tk, Tu);
        else
            hipLaunchKernelGGL(sim_maps_rows_kernel<1>, dim3(ntk, K), dim3(256), 0, st, (const bf16*)kwd, kwd_mask,
                               (const bf16*)utt, utt_mask, (bf16*)out, L, Tk, Tu);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(sim_maps_kernel, dim3((ntu + 3) / 4, ntk * K), dim3(256), 0, st, (const bf16*)kwd, kwd_mask,
                       (const bf16*)utt, utt_mask, (bf16*)out, K, L, Tk, Tu, E);
    return hipGetLastError();
}

hipError_t cbw_sim_to_nchw(const uint16_t* maps, float* out, int K, int L, int Tk, int Tu, hipStream_t st) {
    hipLaunchKernelGGL(sim_to_nchw_kernel, dim3(grid_for((int64_t)K * Tk * Tu, 256)), dim3(256), 0, st,
                       (const bf16*)maps, out, K, L, Tk, Tu);
    return hipGetLastError();
}

hipError_t cbw_stem_conv(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H, int W,
                         int Ho, int Wo, hipStream_t st) {
    const int64_t M = (int64_t)N * Ho * Wo;
    const int lds = 4 * 64 * 68 * 4;   // epilogue image >= A (16 KB) + B (29 KB)
    hipLaunchKernelGGL(stem_kernel, dim3((unsigned)((M + STEM_BM - 1) / STEM_BM)), dim3(256), lds, st,
                       (const bf16*)x, (const bf16*)w, bias, (bf16*)y, N, H, W, Ho, Wo);
    return hipGetLastError();
}

hipError_t cbw_stem_pool(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H, int W,
                         int Hs, int Ws, int Hp, int Wp, hipStream_t st) {
    if (N <= 0 || Hp <= 0 || Wp <= 0) return hipSuccess;
    const int nrt = (Hp + SP_RMAX - 1) / SP_RMAX;
    const int R = (Hp + nrt - 1) / nrt;
    const int nct = (Wp + SP_PW - 1) / SP_PW;
    const int64_t nt = (int64_t)N * nrt * nct;
    if (nt >= (1LL << 31)) return hipErrorInvalidValue;
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    const int64_t G = std::min<int64_t>(nt, 2 * (int64_t)ncu);
    const char* v1 = getenv("CBW_STEM_V1");   // A/B: the round-4 epilogue and pool (read per call)
    // round 6's V3 (default on full-height tiles; CBW_STEM_V3=0: V2): tools/stem_bench.py, 625 LEF pairs, alternating
    // runs 361.9 / 367.5 vs 373.2 / 377.3 us, bit-identical
    const char* v3 = getenv("CBW_STEM_V3");
    if (nrt == 1 && (!v3 || atoi(v3) != 0) && !(v1 && atoi(v1) == 1))
        hipLaunchKernelGGL(stem_pool_v3_kernel, dim3((unsigned)G), dim3(256), sp_lds_bytes(R), st, (const bf16*)x,
                           (const bf16*)w, bias, (bf16*)y, N, H, W, Hs, Ws, Hp, Wp, R, nct);
    else if (v1 && atoi(v1) == 1)
        hipLaunchKernelGGL(stem_pool_kernel<false>, dim3((unsigned)G), dim3(256), sp_lds_bytes(R), st, (const bf16*)x,
                           (const bf16*)w, bias, (bf16*)y, N, H, W, Hs, Ws, Hp, Wp, R, nrt, nct);
    else
        hipLaunchKernelGGL(stem_pool_kernel<true>, dim3((unsigned)G), dim3(256), sp_lds_bytes(R), st, (const bf16*)x,
                           (const bf16*)w, bias, (bf16*)y, N, H, W, Hs, Ws, Hp, Wp, R, nrt, nct);
    return hipGetLastError();
}

hipError_t cbw_stem16_pool(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H,
                           int W, int Hs, int Ws, int Hp, int Wp, hipStream_t st) {
    if (N <= 0 || Hp <= 0 || Wp <= 0) return hipSuccess;
    const int nrt = (Hp + S16_RMAX - 1) / S16_RMAX;
    const int R = (Hp + nrt - 1) / nrt;
    const int nct = (Wp + SP_PW - 1) / SP_PW;
    const int64_t nt = (int64_t)N * nrt * nct;
    if (nt >= (1LL << 31)) return hipErrorInvalidValue;
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    const int64_t G = std::min<int64_t>(nt, ncu);
    hipLaunchKernelGGL(stem16_pool_kernel<false>, dim3((unsigned)G), dim3(256), s16_lds_bytes(R), st, (const bf16*)x,
                       (const bf16*)w, bias, (bf16*)y, N, H, W, Hs, Ws, Hp, Wp, R, nrt, nct);
    return hipGetLastError();
}

hipError_t cbw_stem16_pool_x3(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H,
                              int W, int Hs, int Ws, int Hp, int Wp, hipStream_t st) {
    if (N <= 0 || Hp <= 0 || Wp <= 0) return hipSuccess;
    const int nrt = (Hp + S16_RMAX_X3 - 1) / S16_RMAX_X3;
    const int R = (Hp + nrt - 1) / nrt;
    const int nct = (Wp + SP_PW - 1) / SP_PW;
    const int64_t nt = (int64_t)N * nrt * nct;
    if (nt >= (1LL << 31)) return hipErrorInvalidValue;
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    const int64_t G = std::min<int64_t>(nt, ncu);
    hipLaunchKernelGGL(stem16_pool_kernel<true>, dim3((unsigned)G), dim3(256), s16_lds_bytes(R, true), st,
                       (const bf16*)x, (const bf16*)w, bias, (bf16*)y, N, H, W, Hs, Ws, Hp, Wp, R, nrt, nct);
    return hipGetLastError();
}

// fp32 maps NHWC [K][H][W][L] (sim_f32) -> NHWC16 bf16 [x_hi (L) | x_hi (L) | x_lo (L) | 0] (3 L <= 16): the
// compensated tier's stem input (cbw_stem16_pool_x3)
__global__ void maps_split16_kernel(const float* __restrict__ x, bf16* __restrict__ y, int K, int L, int HW) {
    const int64_t total = (int64_t)K * HW;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        bf16x8 o0 = {}, o1 = {};
        bf16 v[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) v[c] = f2bf(0.f);
        for (int l = 0; l < L; ++l) {
            const float f = x[i * L + l];
            const bf16 hi = f2bf(f);
            v[l] = hi;
            v[L + l] = hi;
            v[2 * L + l] = f2bf(f - bf2f(hi));
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            o0[c] = v[c];
            o1[c] = v[8 + c];
        }
        *(bf16x8*)(y + i * 16) = o0;
        *(bf16x8*)(y + i * 16 + 8) = o1;
    }
}

hipError_t cbw_maps_split16(const float* x, uint16_t* y, int K, int L, int H, int W, hipStream_t st) {
    if (3 * L > 16 || K <= 0) return K == 0 ? hipSuccess : hipErrorInvalidValue;
    hipLaunchKernelGGL(maps_split16_kernel, dim3(grid_for((int64_t)K * H * W, 256)), dim3(256), 0, st, x, (bf16*)y, K,
                       L, H * W);
    return hipGetLastError();
}

hipError_t cbw_sim_resize(const float* sim, int64_t layer_stride, int ld, const int* off_dev, int k0, int K, int L,
                          int Tu, int Ho, int Wo, uint16_t* out, hipStream_t st) {
    if (L > 16 || K <= 0) return K == 0 ? hipSuccess : hipErrorInvalidValue;
    hipLaunchKernelGGL(sim_resize_kernel, dim3(grid_for((int64_t)K * Ho * Wo, 256)), dim3(256), 0, st, sim,
                       layer_stride, ld, off_dev, k0, K, L, Tu, Ho, Wo, (bf16*)out);
    return hipGetLastError();
}

hipError_t cbw_nchw_to_nhwc16(const float* x, uint16_t* y, int K, int L, int H, int W, hipStream_t st) {
    if (L > 16) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nchw_to_nhwc16_kernel, dim3(grid_for((int64_t)K * H * W, 256)), dim3(256), 0, st, x, (bf16*)y,
                       K, L, H, W);
    return hipGetLastError();
}

hipError_t cbw_maxpool3s2(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, int Ho, int Wo, hipStream_t st) {
    if (C % 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(maxpool3s2_kernel, dim3(grid_for((int64_t)N * Ho * Wo * C / 8, 256)), dim3(256), 0, st,
                       (const bf16*)x, (bf16*)y, N, H, W, C, Ho, Wo);
    return hipGetLastError();
}

hipError_t cbw_pool_fc(const uint16_t* x, const float* w, const float* b, float* logits, int N, int HW, int C,
                       hipStream_t st) {
    if (C % 8) return hipErrorInvalidValue;
    const char* ue = getenv("CBW_POOL_UNROLL");   // pixels' loads in flight per lane (1 / 4 / 8), read per call
    const int unr = ue ? atoi(ue) : 8;
    if (unr == 8)
        hipLaunchKernelGGL(pool_fc_kernel<8>, dim3(N), dim3(256), 0, st, (const bf16*)x, w, b, logits, HW, C);
    else if (unr == 4)
        hipLaunchKernelGGL(pool_fc_kernel<4>, dim3(N), dim3(256), 0, st, (const bf16*)x, w, b, logits, HW, C);
    else
        hipLaunchKernelGGL(pool_fc_kernel<1>, dim3(N), dim3(256), 0, st, (const bf16*)x, w, b, logits, HW, C);
    return hipGetLastError();
}

hipError_t cbw_spot(const float* logits, const float* ghost, int K, float thr, float band, int mode, float* prob_out,
                    int* idx_out, int* n_out, hipStream_t st) {
    hipLaunchKernelGGL(spot_kernel, dim3(1), dim3(1024), 0, st, logits, ghost, K, thr, band, mode, prob_out, idx_out,
                       n_out);
    return hipGetLastError();
}

// ---------------------------------------------------------------- content checksum
// 64-bit position-dependent checksum of a byte range (the keyword-database cache key of efficient_kws.model.KWSModel,
// which re-projects the database only when its content changed): sum over 16-byte words w_i (wrapping) of
// splitmix64(lo(w_i) + C (2i + 1)) + splitmix64(hi(w_i) + C (2i + 2)); the tail bytes fold into one last word.  Not
// cryptographic: any change of a word changes its term, and two changed words cancel with probability ~2^-64.  One
// launch over grid-stride words into per-workgroup partials, a second sums the partials in order (no atomics).
namespace {
CBW_DEV uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
constexpr uint64_t CK_GOLD = 0x9e3779b97f4a7c15ull;
constexpr int CK_BLOCKS = 1024;

__global__ __launch_bounds__(256) void checksum_words_kernel(const uint4* __restrict__ p, int64_t n16,
                                                             uint64_t* __restrict__ part) {
    __shared__ uint64_t red[256];
    uint64_t s = 0;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const uint4 w = p[i];
        const uint64_t lo = ((uint64_t)w.y << 32) | w.x, hi = ((uint64_t)w.w << 32) | w.z;
        s += splitmix64(lo + CK_GOLD * (uint64_t)(2 * i + 1)) + splitmix64(hi + CK_GOLD * (uint64_t)(2 * i + 2));
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void checksum_finish_kernel(const uint64_t* __restrict__ part, int np,
                                                              const unsigned char* __restrict__ tail, int ntail,
                                                              int64_t n16, uint64_t* __restrict__ out) {
    __shared__ uint64_t red[256];
    uint64_t s = 0;
    for (int i = threadIdx.x; i < np; i += 256) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint64_t t = red[0];
        if (ntail > 0) {   // the last < 16 bytes, little-endian into two words (bytes 0-7, 8-15) hashed like a full word pair
            uint64_t w[2] = {0, 0};
            for (int b = 0; b < ntail; ++b) w[b >> 3] |= (uint64_t)tail[b] << (8 * (b & 7));
            t += splitmix64(w[0] + CK_GOLD * (uint64_t)(2 * n16 + 1) + (uint64_t)ntail) +
                 splitmix64(w[1] + CK_GOLD * (uint64_t)(2 * n16 + 2) + (uint64_t)ntail);
        }
        *out = t;
    }
}
}  // namespace

int cbw_checksum_scratch_bytes() { return CK_BLOCKS * 8; }

hipError_t cbw_checksum64(const void* data, int64_t bytes, uint64_t* out, uint64_t* scratch, hipStream_t st) {
    if (bytes < 0 || (bytes > 0 && !data) || !out || !scratch || ((uintptr_t)data & 15)) return hipErrorInvalidValue;
    const int64_t n16 = bytes / 16;
    const int ntail = (int)(bytes - n16 * 16);
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(CK_BLOCKS, (n16 + 255) / 256));
    hipLaunchKernelGGL(checksum_words_kernel, dim3(nb), dim3(256), 0, st, (const uint4*)data, n16, scratch);
    hipLaunchKernelGGL(checksum_finish_kernel, dim3(1), dim3(256), 0, st, scratch, nb,
                       (const unsigned char*)data + n16 * 16, ntail, n16, out);
    return hipGetLastError();
}
