// fp8 (OCP e4m3) implicit-GEMM convolution for the first tier of the exact-decision cascade (C5 of BASELINE.json:
// "fp8 MFMA"): ResNet-50 stages 2-4 of the efficient_kws classifier (src/efficient_kws/resnet.py:51-58, HF
// ResNetBottleNeckLayer) with both operands in e4m3 on the block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4
// at unit scales (2x the bf16 MFMA rate per clock, MI355X_MICROARCH.md "Matrix cores").
//
// Scaling: every activation tensor is stored as e4m3(v / s) with one static scale s per tensor (calibrated on the
// fp32 network's absolute maxima, cbw_kws_calibrate_fp8); a conv's weights are pre-multiplied by its input
// tensor's scale and quantized per output channel (w_q = e4m3(w s_in / alpha_n)), so the epilogue computes
// v = acc * alpha_n + bias_n (+ residual r_q * s_res), ReLU, and stores e4m3(v / s_out) or bf16.  The MFMA scale
// operands stay 127 (2^0); all scaling is in the fp32 epilogue.
//
// Structure: the bf16 4-wave tile kernel's (conv_igemm.hip) in bytes -- K-stage = 128 e4m3 channels = 128 B per
// row, glds im2col gather into a double-buffered XOR-swizzled LDS image, 4 waves x 64x64 outputs as 4x4 MFMA
// tiles (16x16x128: one MFMA per tile per stage), XCD-aware tile order, LDS-staged epilogue on 8-channel rows.
// Operands: lane l holds row l & 15 of A and column l & 15 of B, its 32 bytes the K-stage's channels
// 32 (l >> 4) .. + 31 for both (any k order shared by A and B gives the same product; checked on the GPU with exact
// integers, tests/test_gpu_fp8.py); C/D as every gfx950 16x16 MFMA (row 4 (l >> 4) + reg, col l & 15).
#include <algorithm>
#include <cstdlib>

#include "cbw_common.h"
#include "cbw_kernels.h"

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int F8_BK = 128;             // e4m3 channels per K-stage (128 B per row)
constexpr int F8_EPI_LD = 68;
constexpr int F8_EPI_BYTES = 4 * 64 * F8_EPI_LD * 4;
constexpr int F8_STAGE = (128 + 128) * 128;
constexpr int F8_LDS = 2 * F8_STAGE > F8_EPI_BYTES ? 2 * F8_STAGE : F8_EPI_BYTES;
constexpr float F8_MAX = 448.f;

CBW_DEV int swz8(int r) { return (r >> 1) & 7; }

CBW_DEV f32x4 mfma_f8(const i32x8& a, const i32x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// 8 floats -> 8 e4m3 bytes (value * inv, saturated to +-448)
CBW_DEV uint2 pack8_fp8(const float (&v)[8], float inv) {
    float q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = fminf(fmaxf(v[i] * inv, -F8_MAX), F8_MAX);
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[4], q[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[6], q[7], hi, true);
    return uint2{(unsigned)lo, (unsigned)hi};
}

CBW_DEV void unpack8_fp8(uint2 p, float scale, float (&v)[8]) {
    const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8((int)p.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)p.x, true);
    const f32x2 c = __builtin_amdgcn_cvt_pk_f32_fp8((int)p.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)p.y, true);
    v[0] = a[0] * scale; v[1] = a[1] * scale; v[2] = b[0] * scale; v[3] = b[1] * scale;
    v[4] = c[0] * scale; v[5] = c[1] * scale; v[6] = d[0] * scale; v[7] = d[1] * scale;
}

template <int KH, int KW>
__global__ __launch_bounds__(256, 2) void conv_fp8_kernel(F8ConvArgs a) {
    constexpr int BM = 128, BN = 128, WN = 2, AR = BM / 32, BR = BN / 32;
    static_assert(KH * KW <= 32, "tap mask");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int nt_n = a.Cout / BN;
    const int nt_m = (a.M + BM - 1) / BM;
    const int bid = xcd_remap(blockIdx.x, nt_m * nt_n);
    const int tm = bid / nt_n, tn = bid % nt_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int64_t Ktot = (int64_t)KH * KW * a.Cin;
    const int csteps = a.Cin / F8_BK;
    const int nsteps = KH * KW * csteps;
    const int HoWo = a.Ho * a.Wo;

    // per-lane A rows: window origin and in-image tap mask, computed once (as conv_igemm_kernel)
    const int sub_r = lane >> 3, chunk = lane & 7;
    const uint8_t* a_px[AR];
    unsigned a_tm[AR];
#pragma unroll
    for (int j = 0; j < AR; ++j) {
        const int r = (wid * AR + j) * 8 + sub_r;
        const int m = m0 + r;
        const bool okm = m < a.M;
        const int mm = okm ? m : 0;
        const int n = mm / HoWo, rem = mm - n * HoWo;
        const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
        const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
        unsigned tmask = 0;
#pragma unroll
        for (int kh = 0; kh < KH; ++kh)
#pragma unroll
            for (int kw = 0; kw < KW; ++kw) {
                const int ih = ih0 + kh, iw = iw0 + kw;
                if (okm && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) tmask |= 1u << (kh * KW + kw);
            }
        a_tm[j] = tmask;
        a_px[j] = a.x + (int64_t)n * a.H * a.W * a.Cin + ((int64_t)ih0 * a.W + iw0) * a.Cin + (chunk ^ swz8(r)) * 16;
    }
    const uint8_t* wrow[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int r = (wid * BR + j) * 8 + sub_r;
        wrow[j] = a.w + (int64_t)(n0 + r) * Ktot + (chunk ^ swz8(r)) * 16;
    }
    int nx_cs = 0, nx_tap = 0, nx_kh = 0, nx_kw = 0;
    auto issue_stage = [&](int s, int buf) {
        const int tap = nx_tap;
        const int64_t off = ((int64_t)nx_kh * a.W + nx_kw) * a.Cin + nx_cs * F8_BK;
        if (++nx_cs == csteps) {
            nx_cs = 0;
            ++nx_tap;
            if (++nx_kw == KW) { nx_kw = 0; ++nx_kh; }
        }
        char* A = smem + buf * F8_STAGE;
        char* B = A + BM * 128;
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            const void* src = ((a_tm[j] >> tap) & 1u) ? (const void*)(a_px[j] + off) : a.zero;
            __builtin_amdgcn_global_load_lds(src, (void*)(A + (wid * AR + j) * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < BR; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(wrow[j] + (int64_t)s * F8_BK), (void*)(B + (wid * BR + j) * 1024),
                                             16, 0, 0);
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    issue_stage(0, 0);
    // epilogue operands prefetched with stage 0: lane owns columns col..col+15 of rows it*16 + lane/4 of its tile
    // (16 e4m3 bytes per lane: one 16-byte store per row; 8-byte stores left the store tail issue-bound)
    const int ecg = lane & 3, erow = lane >> 2;
    const int ecol = n0 + wn * 64 + ecg * 16;
    uint4 rpre[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int m = m0 + wm * 64 + it * 16 + erow;
        rpre[it] = (a.res && m < a.M) ? *(const uint4*)(a.res + (int64_t)m * a.Cout + ecol) : uint4{0u, 0u, 0u, 0u};
    }
    f32x4 al[4], bi[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        al[g] = *(const f32x4*)(a.alpha + ecol + 4 * g);
        bi[g] = *(const f32x4*)(a.bias + ecol + 4 * g);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int fr = lane & 15, fq = lane >> 4;
    for (int s = 0; s < nsteps; ++s) {
        const int buf = s & 1;
        if (s + 1 < nsteps) issue_stage(s + 1, buf ^ 1);
        const char* A = smem + buf * F8_STAGE;
        const char* B = A + BM * 128;
        i32x8 av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = wm * 64 + i * 16 + fr;
            const i32x4 lo = *(const i32x4*)(A + r * 128 + (((2 * fq) ^ swz8(r)) * 16));
            const i32x4 hi = *(const i32x4*)(A + r * 128 + (((2 * fq + 1) ^ swz8(r)) * 16));
            av[i] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = wn * 64 + j * 16 + fr;
            const i32x4 lo = *(const i32x4*)(B + r * 128 + (((2 * fq) ^ swz8(r)) * 16));
            const i32x4 hi = *(const i32x4*)(B + r * 128 + (((2 * fq + 1) ^ swz8(r)) * 16));
            bv[j] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma_f8(av[i], bv[j], acc[i][j]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---- epilogue: wave-private fp32 image [64][F8_EPI_LD] ----
    float* E = (float*)smem + wid * 64 * F8_EPI_LD;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) E[(i * 16 + fq * 4 + q) * F8_EPI_LD + j * 16 + fr] = acc[i][j][q];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int r = it * 16 + erow;
        const int m = m0 + wm * 64 + r;
        if (m >= a.M) continue;
        float v[2][8];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 e = *(const f32x4*)(E + r * F8_EPI_LD + ecg * 16 + 4 * g);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[g >> 1][(g & 1) * 4 + q] = e[q] * al[g][q] + bi[g][q];
        }
        if (a.res) {
            float rv[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                unpack8_fp8(h ? uint2{rpre[it].z, rpre[it].w} : uint2{rpre[it].x, rpre[it].y}, a.res_scale, rv);
#pragma unroll
                for (int q = 0; q < 8; ++q) v[h][q] += rv[q];
            }
        }
        if (a.relu)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int q = 0; q < 8; ++q) v[h][q] = fmaxf(v[h][q], 0.f);
        if (a.out_bf16) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                bf16x8 o;
#pragma unroll
                for (int q = 0; q < 8; ++q) o[q] = f2bf(v[h][q]);
                *(bf16x8*)((bf16*)a.y + (int64_t)m * a.Cout + ecol + 8 * h) = o;
            }
        } else {
            const uint2 lo = pack8_fp8(v[0], a.y_inv_scale), hi = pack8_fp8(v[1], a.y_inv_scale);
            *(uint4*)((uint8_t*)a.y + (int64_t)m * a.Cout + ecol) = uint4{lo.x, lo.y, hi.x, hi.y};
        }
    }
}

// ---------------------------------------------------------------------------
// 8-wave ping-pong variant for Cout % 256 == 0 (stages 3-4): conv_igemm_p8's schedule (conv_igemm.hip) in bytes.
// BM = BN = 256, K-tile = 128 e4m3 channels (128 B rows, the same LDS image as p8's 64 bf16 channels), 8 waves as
// 2 groups x 4, each wave 128 pixels x 64 channels; a K-tile in four quadrant phases of 8 MFMAs 16x16x128 (the
// cycles of p8's 16 MFMAs 16x16x32 at twice the K), the next K-tile's four half-tiles DMA'd one per phase and
// retired by counted vmcnt(4); group 1 one barrier behind so one group's MFMAs overlap the other's LDS reads.
constexpr int F8P_BUF = (256 + 256) * 128;   // 64 KB per K-tile buffer
CBW_DEV int f8p_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

template <int KH, int KW>
__global__ __launch_bounds__(512, 1) void conv_fp8_p8(F8ConvArgs a) {
    static_assert(KH * KW <= 32, "tap mask");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;
    const int fr = lane & 15, fq = lane >> 4;
    const int nt_n = a.Cout / 256;
    const int nt_m = (a.M + 255) / 256;
    const int bid = xcd_remap(blockIdx.x, nt_m * nt_n);
    const int tm = bid / nt_n, tn = bid % nt_n;
    const int m0 = tm * 256, n0 = tn * 256;
    const int64_t Ktot = (int64_t)KH * KW * a.Cin;
    const int csteps = a.Cin / F8_BK;
    const int nk = KH * KW * csteps;
    const int HoWo = a.Ho * a.Wo;

    const int sub = lane >> 3, pch = lane & 7;
    const uint8_t* a_px[2][2];
    unsigned a_tm[2][2];
    const uint8_t* wrow[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int r = g * 128 + h * 64 + wid * 8 + sub;
            const int m = m0 + r;
            const bool okm = m < a.M;
            const int mm = okm ? m : 0;
            const int n = mm / HoWo, rem = mm - n * HoWo;
            const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
            const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
            unsigned tmask = 0;
#pragma unroll
            for (int kh = 0; kh < KH; ++kh)
#pragma unroll
                for (int kw = 0; kw < KW; ++kw) {
                    const int ih = ih0 + kh, iw = iw0 + kw;
                    if (okm && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) tmask |= 1u << (kh * KW + kw);
                }
            a_tm[h][g] = tmask;
            a_px[h][g] = a.x + (int64_t)n * a.H * a.W * a.Cin + ((int64_t)ih0 * a.W + iw0) * a.Cin +
                         ((pch ^ ((r >> 1) & 7)) * 16);
            const int rb = h * 128 + g * 64 + wid * 8 + sub;
            wrow[h][g] = a.w + (int64_t)(n0 + rb) * Ktot + ((pch ^ ((rb >> 1) & 7)) * 16);
        }
    int nx_cs = 0, nx_tap = 0, nx_kh = 0, nx_kw = 0;
    int nx_off = 0;   // (kh * W + kw) * Cin + channel offset: < 2^31 (the host checks the tap window)
    auto advance = [&]() {
        if (++nx_cs == csteps) {
            nx_cs = 0;
            ++nx_tap;
            if (++nx_kw == KW) { nx_kw = 0; ++nx_kh; }
        }
        nx_off = (nx_kh * a.W + nx_kw) * a.Cin + nx_cs * F8_BK;
    };
    // half-tile `which` (0 A0', 1 B0, 2 B1, 3 A1') of K-tile kt -> buffer kt & 1; two glds per lane in every case
    auto issue = [&](int kt, int which) {
        char* A = smem + (kt & 1) * F8P_BUF;
        if (which == 0 || which == 3) {
            const int h = which == 3;
            const int tap = nx_tap;
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const void* src = ((a_tm[h][g] >> tap) & 1u) ? (const void*)(a_px[h][g] + nx_off) : a.zero;
                __builtin_amdgcn_global_load_lds(src, (void*)(A + (g * 128 + h * 64 + wid * 8) * 128), 16, 0, 0);
            }
        } else {
            const int h = which - 1;
            char* B = A + 256 * 128;
#pragma unroll
            for (int g = 0; g < 2; ++g)
                __builtin_amdgcn_global_load_lds((const void*)(wrow[h][g] + (int64_t)kt * F8_BK),
                                                 (void*)(B + (h * 128 + g * 64 + wid * 8) * 128), 16, 0, 0);
        }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    i32x8 av[4], bv[2];

#pragma unroll
    for (int w = 0; w < 4; ++w) issue(0, w);
    advance();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind
    for (int kt = 0; kt < nk; ++kt) {
        const char* A = smem + (kt & 1) * F8P_BUF;
        const char* B = A + 256 * 128;
        const bool more = kt + 1 < nk;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int mi = q >> 1, ni = (q == 1 || q == 2) ? 1 : 0;
            __builtin_amdgcn_sched_barrier(0);
            if (more) {
                issue(kt + 1, q);
                if (q == 3) advance();
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            } else if (q == 0) {
                asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (q == 0 || q == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = wr * 128 + mi * 64 + i * 16 + fr;
                    const i32x4 lo = *(const i32x4*)(A + f8p_off(r, 2 * fq));
                    const i32x4 hi = *(const i32x4*)(A + f8p_off(r, 2 * fq + 1));
                    av[i] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
            }
            if (q != 2) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int r = ni * 128 + wc * 32 + j * 16 + fr;
                    const i32x4 lo = *(const i32x4*)(B + f8p_off(r, 2 * fq));
                    const i32x4 hi = *(const i32x4*)(B + f8p_off(r, 2 * fq + 1));
                    bv[j] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[mi * 4 + i][ni * 2 + j] = mfma_f8(bv[j], av[i], acc[mi * 4 + i][ni * 2 + j]);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
        }
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();   // equal barrier counts for both groups

    // epilogue: lane holds channels n0 + 128 ni + 32 wc + 16 j + 4 fq .. +3 of pixel m0 + 128 wr + 16 f + fr
#pragma unroll
    for (int nf = 0; nf < 4; ++nf) {
        const int col = n0 + (nf >> 1) * 128 + wc * 32 + (nf & 1) * 16 + fq * 4;
        const f32x4 al = *(const f32x4*)(a.alpha + col), bb = *(const f32x4*)(a.bias + col);
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const int m = m0 + wr * 128 + f * 16 + fr;
            if (m >= a.M) continue;
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = acc[f][nf][q] * al[q] + bb[q];
            if (a.res) {
                const unsigned r4 = *(const unsigned*)(a.res + (int64_t)m * a.Cout + col);
                const f32x2 r0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)r4, false);
                const f32x2 r1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)r4, true);
                v[0] += r0[0] * a.res_scale; v[1] += r0[1] * a.res_scale;
                v[2] += r1[0] * a.res_scale; v[3] += r1[1] * a.res_scale;
            }
            if (a.relu)
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
            if (a.out_bf16) {
                bf16x4 o;
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
                *(bf16x4*)((bf16*)a.y + (int64_t)m * a.Cout + col) = o;
            } else {
                float qv[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) qv[q] = fminf(fmaxf(v[q] * a.y_inv_scale, -F8_MAX), F8_MAX);
                int pk = __builtin_amdgcn_cvt_pk_fp8_f32(qv[0], qv[1], 0, false);
                pk = __builtin_amdgcn_cvt_pk_fp8_f32(qv[2], qv[3], pk, true);
                *(int*)((uint8_t*)a.y + (int64_t)m * a.Cout + col) = pk;
            }
        }
    }
}

// bf16 NHWC -> e4m3 (value * inv_scale, saturated); 8 elements per thread and step, QU steps' loads in flight
constexpr int QU = 4;
__global__ void quant_fp8_kernel(const bf16* x, uint8_t* y, int64_t n8, float inv) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < n8; i0 += QU * stride) {
        bf16x8 v[QU];
#pragma unroll
        for (int u = 0; u < QU; ++u) {
            const int64_t i = i0 + u * stride;
            v[u] = i < n8 ? *(const bf16x8*)(x + i * 8) : bf16x8{};
        }
#pragma unroll
        for (int u = 0; u < QU; ++u) {
            const int64_t i = i0 + u * stride;
            if (i >= n8) break;
            float f[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] = bf2f(v[u][q]);
            *(uint2*)(y + i * 8) = pack8_fp8(f, inv);
        }
    }
}

// per-workgroup absolute maxima of an fp32 tensor (calibration; the host takes the max of the partials)
constexpr int ABSMAX_GROUPS = 256;
__global__ __launch_bounds__(256) void absmax_f32_kernel(const float* x, int64_t n, float* part) {
    __shared__ float red[4];
    float m = 0.f;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(x[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// ---- probes for tests/test_gpu_fp8.py: the MFMA operand lane map and the conversions ----
// mode 0: lane l holds A[l & 15][32 (l >> 4) + j]; 1: k = 16 (l >> 4) + (j & 15) + 64 (j >> 4);
// 2: k = 8 (l >> 4) + (j & 7) + 32 (j >> 3); 3: k = 4 (l >> 4) + (j & 3) + 16 (j >> 2).  B the same with its column.
__global__ void mfma_fp8_probe_kernel(const uint8_t* A, const uint8_t* Bt, float* C, int mode) {
    const int l = threadIdx.x, r = l & 15, g = l >> 4;
    uint8_t ab[32], bb[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        int k;
        if (mode == 0) k = 32 * g + j;
        else if (mode == 1) k = 16 * g + (j & 15) + 64 * (j >> 4);
        else if (mode == 2) k = 8 * g + (j & 7) + 32 * (j >> 3);
        else k = 4 * g + (j & 3) + 16 * (j >> 2);
        ab[j] = A[r * 128 + k];
        bb[j] = Bt[r * 128 + k];
    }
    i32x8 av, bv;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        av[w] = ab[4 * w] | (ab[4 * w + 1] << 8) | (ab[4 * w + 2] << 16) | (ab[4 * w + 3] << 24);
        bv[w] = bb[4 * w] | (bb[4 * w + 1] << 8) | (bb[4 * w + 2] << 16) | (bb[4 * w + 3] << 24);
    }
    const f32x4 c = mfma_f8(av, bv, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int q = 0; q < 4; ++q) C[(4 * g + q) * 16 + r] = c[q];
}

__global__ void cvt_fp8_probe_kernel(const float* x, uint8_t* q, float* back, int n) {
    const int i = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i + 8 > n) return;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = x[i + k];
    const uint2 p = pack8_fp8(v, 1.f);
    *(uint2*)(q + i) = p;
    float b[8];
    unpack8_fp8(p, 1.f, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) back[i + k] = b[k];
}

// CBW_FP8_P8=1 runs the >= 8 K-tile shapes (Cout % 256) on the 8-wave schedule.  Off by default: at the realistic
// operating point with the streaming 1x1 kernel the fp8 pass took 128.3 ms per clip with it vs 120.1 ms on the
// 4-wave kernel (r03h; stage 4's 3x3 is 352 tiles of 256 x 256 = 1.4 rounds of one workgroup per CU)
int fp8_p8_mode() {
    static const int m = [] {
        const char* e = getenv("CBW_FP8_P8");
        return e ? atoi(e) : 0;
    }();
    return m;
}

template <int KH, int KW>
hipError_t launch_f8(const F8ConvArgs& a, hipStream_t st) {
    // the 8-wave schedule pays on the MFMA-bound shapes (>= 8 K-tiles: 3x3 of stages 3-4, the deep 1x1 reduces);
    // on 1-4 K-tiles its 256 x 256 tiles and one workgroup per CU leave the HBM idle (r03g: fp8 pass 138 -> 184 ms)
    if (a.Cout % 256 == 0 && KH * KW * (a.Cin / F8_BK) >= 8 && fp8_p8_mode()) {
        const int nt = ((a.M + 255) / 256) * (a.Cout / 256);
        static const std::string nm = kernel_name("conv_fp8_p8", {KH, KW});
        cbw_last_conv_kernel = nm.c_str();
        hipLaunchKernelGGL((conv_fp8_p8<KH, KW>), dim3(nt), dim3(512), 2 * F8P_BUF, st, a);
        return hipGetLastError();
    }
    const int nt = ((a.M + 127) / 128) * (a.Cout / 128);
    static const std::string nm = kernel_name("conv_fp8_kernel", {KH, KW});
    cbw_last_conv_kernel = nm.c_str();
    hipLaunchKernelGGL((conv_fp8_kernel<KH, KW>), dim3(nt), dim3(256), F8_LDS, st, a);
    return hipGetLastError();
}

}  // namespace

bool cbw_conv_fp8_supported(const F8ConvArgs& a) {
    return a.x && a.w && a.alpha && a.bias && a.y && a.zero && a.Cin > 0 && a.Cin % F8_BK == 0 && a.Cout > 0 &&
           a.Cout % 128 == 0 && a.M > 0 && a.M == a.N * a.Ho * a.Wo && a.sh >= 1 && a.sw >= 1 &&
           ((a.KH == 1 && a.KW == 1) || (a.KH == 3 && a.KW == 3)) &&
           ((int64_t)a.N * a.H * a.W * a.Cin < (1ll << 40)) &&
           ((int64_t)((a.KH - 1) * a.W + a.KW) * a.Cin < (1ll << 31));   // the in-kernel tap offset is 32-bit
}

hipError_t cbw_conv_fp8(const F8ConvArgs& a, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)conv_fp8_kernel<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, F8_LDS);
        (void)hipFuncSetAttribute((const void*)conv_fp8_kernel<3, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, F8_LDS);
        (void)hipFuncSetAttribute((const void*)conv_fp8_p8<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * F8P_BUF);
        (void)hipFuncSetAttribute((const void*)conv_fp8_p8<3, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * F8P_BUF);
        attr = true;
    }
    if (!cbw_conv_fp8_supported(a)) return hipErrorInvalidValue;
    if (cbw_conv_fp8_stream_supported(a)) return cbw_conv_fp8_stream(a, st);   // HBM-bound stride-1 1x1
    if (a.KH == 1) return launch_f8<1, 1>(a, st);
    return launch_f8<3, 3>(a, st);
}

hipError_t cbw_quant_fp8(const uint16_t* x, uint8_t* y, int64_t n, float inv_scale, hipStream_t st) {
    if (n % 8) return hipErrorInvalidValue;
    const int64_t n8 = n / 8;
    if (n8 == 0) return hipSuccess;
    const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 8192);
    hipLaunchKernelGGL(quant_fp8_kernel, dim3(blocks), dim3(256), 0, st, (const bf16*)x, y, n8, inv_scale);
    return hipGetLastError();
}

int cbw_absmax_groups() { return ABSMAX_GROUPS; }

hipError_t cbw_absmax_f32(const float* x, int64_t n, float* part, hipStream_t st) {
    hipLaunchKernelGGL(absmax_f32_kernel, dim3(ABSMAX_GROUPS), dim3(256), 0, st, x, n, part);
    return hipGetLastError();
}

hipError_t cbw_mfma_fp8_probe(const uint8_t* A, const uint8_t* Bt, float* C, int mode, hipStream_t st) {
    if (mode < 0 || mode > 3) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mfma_fp8_probe_kernel, dim3(1), dim3(64), 0, st, A, Bt, C, mode);
    return hipGetLastError();
}

hipError_t cbw_cvt_fp8_probe(const float* x, uint8_t* q, float* back, int n, hipStream_t st) {
    if (n % 8 || n <= 0) return hipErrorInvalidValue;
    const int thr = n / 8;
    hipLaunchKernelGGL(cvt_fp8_probe_kernel, dim3((thr + 255) / 256), dim3(256), 0, st, x, q, back, n);
    return hipGetLastError();
}
