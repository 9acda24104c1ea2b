// Fused ResNet-50 identity bottleneck for small maps (stage 3 at LEF sizes: 5 x 47 pixels, 1024 -> 256 -> 256
// -> 1024): reduce 1x1 + BN + ReLU, 3x3 + BN + ReLU, expand 1x1 + BN + residual + ReLU in one persistent launch,
// one workgroup per pair image -- the whole image's two 256-channel intermediates live in LDS, so the block
// reads its input from HBM twice (reduce operand, residual) and writes its output once, with no launch tails
// between its three convs.
//
// Reference: HF ResNetBottleNeckLayer as instantiated by efficient_kws/resnet.py:22-38 (ResNet-50 stage 3,
// layers 2-6) and run by Resnet.forward (resnet.py:51-58).  Same rounding points as the three-conv path
// (bf16 T1 / T2 after bias + ReLU, fp32 accumulation); the biases seed the accumulators.
//
// Workgroup: 8 waves (two per SIMD), wave (wh, wq) owns a channel quarter (CM / 4; CM / 8 in phase E) of the
// pixel fragments of half of the image (16 F rows over the two halves; rows >= H W are dummies whose results
// are dropped).  MFMAs run transposed (C^T = W . X^T): a lane ends with 4 consecutive channels of one pixel.
//   phase R  T1 = relu(X . Wr^T + br): X streamed through LDS in 128-channel chunks (buffer DMA, double-
//            buffered, rows past the image read 0), Wr fragments straight from L2 into registers.
//   phase M  T2 = relu(conv3x3(T1) . Wm^T + bm): T1 (bf16, 16-byte chunks XOR-swizzled by row) in LDS with
//            one zero row that every out-of-image tap reads; no barriers inside the phase.
//   phase E  y = relu(T2 . We^T + be + x) in CIN / (CM / 2) passes of CM / 2 output channels (the narrower
//            pass leaves registers for the residual, which comes from HBM / L2 during the pass).
// The weight fragments of every k-step (168 per pair at stage 3; the two pixel halves read the same ones) form one stream, prefetched two k-steps
// ahead across phase and pair boundaries (all pairs share the weights).
#include <algorithm>

#include "cbw_common.h"
#include "cbw_kernels.h"
#ifndef BI_WAVES
#define BI_WAVES 8
#endif
#ifndef BI_RING
#define BI_RING 2   // weight-fragment ring slots: prefetch distance BI_RING - 1 k-steps
#endif

typedef int bi_i32x4 __attribute__((ext_vector_type(4)));
typedef short bi_s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int bi_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int bi_u32x4 __attribute__((ext_vector_type(4)));
__device__ bi_i32x4 bi_raw_load4(bi_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ bi_u32x2 bi_raw_load2(bi_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v2i32");
__device__ void bi_raw_store2(bi_u32x2 vdata, bi_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v2i32");
__device__ void bi_raw_buffer_load_lds(bi_i32x4 rsrc, __attribute__((address_space(3))) void* lds, int size,
                                       int voffset, int soffset, int offset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.lds");

namespace {

template <int CIN, int CM, int F>
struct BiL {
    static constexpr int ROWS = 16 * F;              // pixel rows incl. dummies
    static constexpr int ZROW = ROWS;                // T1's zero row (out-of-image 3x3 taps)
    static constexpr int PITCH = CM * 2;             // T1 / T2 bytes per pixel
    static constexpr int T_BYTES = (ROWS + 1) * PITCH;
    static constexpr int XK = 128;                   // phase-R channels per DMA chunk
    static constexpr int XPITCH = XK * 2;            // 256 B: 16 chunks of 16 B, swizzled by row & 15
    static constexpr int XBUF = ROWS * XPITCH;
    static constexpr int XG = ROWS / 4;              // DMA instructions (4 rows of 256 B) per chunk
    static constexpr int LDS = T_BYTES > 2 * XBUF ? T_BYTES : 2 * XBUF;
    static constexpr int NW = BI_WAVES;              // waves: 4 (one per SIMD, every fragment) or 8 (two pixel halves)
    static constexpr int FW = NW == 4 ? F : (F + 1) / 2;   // pixel fragments per wave
    static constexpr int CW = CM / 4;                // channels per wave in phases R / M (four channel quarters)
    static constexpr int NJ = CW / 16;               // channel tiles per wave
    static constexpr int CE = CM / 2;                // phase-E output channels per pass
    static constexpr int NJE = CE / 64;              // phase-E channel tiles per wave
    static constexpr int NR = CIN / 32, NM = 9 * CM / 32, NE = CM / 32;   // k-steps per phase (pass)
    static constexpr int NPASS = CIN / CE;
    static constexpr int NU = NR + NM + NPASS * NE;  // k-steps per pair
    static constexpr int NCH = CIN / XK;
    static_assert(CIN % XK == 0 && CM % 128 == 0 && CIN % CE == 0, "shape");
    static_assert(NR % 4 == 0 && NM % 4 == 0 && NE % 4 == 0, "the A ring slot is a compile-time k-step % ring (2 or 4)");
    static_assert(LDS <= 163840, "LDS budget");
};

CBW_DEV bi_i32x4 bi_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    return bi_i32x4{(int)(uint32_t)a, (int)(uint32_t)(a >> 32), (int)bytes, 0x00020000};
}

CBW_DEV uint32_t bi_relu_pk(float a, float b) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    bi_s16x2 v = __builtin_bit_cast(bi_s16x2, __builtin_convertvector((f32x2{a, b}), bf16x2));
    v = __builtin_elementwise_max(v, bi_s16x2{0, 0});
    return __builtin_bit_cast(uint32_t, v);
}
CBW_DEV float bi_lo(uint32_t u) { return __builtin_bit_cast(float, u << 16); }
CBW_DEV float bi_hi(uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); }

template <int CIN, int CM, int F>
__global__ __launch_bounds__(BI_WAVES * 64, 1) void bottleneck_img_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                                const bf16* __restrict__ wr, const float* __restrict__ br,
                                                                const bf16* __restrict__ wm, const float* __restrict__ bm,
                                                                const bf16* __restrict__ we, const float* __restrict__ be,
                                                                int N, int H, int W) {
    using L = BiL<CIN, CM, F>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar loops and branches
    const int wh = w >> 2, wq = w & 3;   // pixel half (fragments FW wh ..; 0 with 4 waves), channel quarter
    const int fr = lane & 15, fq = lane >> 4;
    const int nt = wh == 0 ? L::FW : F - L::FW;   // this wave's real fragments (wave-uniform)
    const int P = H * W;
    const int G = gridDim.x;

    // ---- the weight stream: k-step u of a pair (phase R: Wr, M: Wm, E: We of pass (u - NR - NM) / NE); the
    // lane's A row: channel wq CW + 16 j + fr (R, M), g CE + wq CE / 4 + 16 j + fr (E, j < NJE).  Buffer loads:
    // one descriptor per matrix, the lane's row offsets in VGPRs, the k-step as the scalar offset
    const bi_i32x4 rs_r = bi_rsrc(wr, (uint32_t)CM * CIN * 2), rs_m = bi_rsrc(wm, (uint32_t)CM * 9 * CM * 2),
                   rs_e = bi_rsrc(we, (uint32_t)CIN * CM * 2);
    int vo_r[L::NJ], vo_m[L::NJ], vo_e[L::NJE];
#pragma unroll
    for (int j = 0; j < L::NJ; ++j) {
        vo_r[j] = ((wq * L::CW + 16 * j + fr) * CIN + fq * 8) * 2;
        vo_m[j] = ((wq * L::CW + 16 * j + fr) * 9 * CM + fq * 8) * 2;
    }
#pragma unroll
    for (int j = 0; j < L::NJE; ++j) vo_e[j] = ((wq * (L::CE / 4) + 16 * j + fr) * CM + fq * 8) * 2;
    auto load_a = [&](int u, bf16x8 (&dst)[L::NJ]) {
        if (u < L::NR) {
#pragma unroll
            for (int j = 0; j < L::NJ; ++j) dst[j] = __builtin_bit_cast(bf16x8, bi_raw_load4(rs_r, vo_r[j], u * 64, 0));
        } else if (u < L::NR + L::NM) {
#pragma unroll
            for (int j = 0; j < L::NJ; ++j)
                dst[j] = __builtin_bit_cast(bf16x8, bi_raw_load4(rs_m, vo_m[j], (u - L::NR) * 64, 0));
        } else {
            const int e = u - L::NR - L::NM, g = e / L::NE;
            const int so = g * L::CE * CM * 2 + (e - g * L::NE) * 64;
#pragma unroll
            for (int j = 0; j < L::NJE; ++j) dst[j] = __builtin_bit_cast(bf16x8, bi_raw_load4(rs_e, vo_e[j], so, 0));
        }
    };
    constexpr int RG = BI_RING, RD = BI_RING - 1;   // ring: k-step u in slot u % RG, requested RD k-steps ahead
    bf16x8 ar[RG][L::NJ];

    // ---- per-lane constants
    // phase R: B fragment = X chunk row 16 (FW wh + i) + fr, chunk 4 ks + fq, physical chunk ^ fr
    int xoff[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) xoff[ks] = (L::FW * wh * 16 + fr) * L::XPITCH + (((ks * 4 + fq) ^ fr) << 4);
    // T1 / T2 write: channels ch0 = wq CW + 16 j + 4 fq of pixel 16 (FW wh + i) + fr
    int twr[L::NJ];
#pragma unroll
    for (int j = 0; j < L::NJ; ++j) {
        const int ch0 = wq * L::CW + 16 * j + 4 * fq;
        twr[j] = (L::FW * wh * 16 + fr) * L::PITCH + (((ch0 >> 3) ^ fr) << 4) + (ch0 & 4) * 2;
    }
    // LDS reads of T1 / T2 with the swizzle folded into the address: row q's k-chunk (4 cs + fq) sits at
    // q PITCH + (((4 cs + fq) ^ (q & 15)) << 4) = (q PITCH | ((fq ^ (q & 15)) << 4)) ^ ((cs & 3) << 6) + (cs >> 2) 256
    const float rcp_w = 1.0f / (float)W;
    const int t2rd = ((L::FW * wh * 16 + fr) * L::PITCH) | ((fq ^ fr) << 4);
    // phase E: byte offset of the lane's pixel row in x / y (rows past the image: past num_records)
    int pvo[L::FW];
#pragma unroll
    for (int i = 0; i < L::FW; ++i) {
        const int p = 16 * (L::FW * wh + i) + fr;
        pvo[i] = p < P ? p * CIN * 2 : 0x40000000;
    }

#pragma unroll
    for (int u = 0; u < RD; ++u) load_a(u, ar[u]);
    for (int n = blockIdx.x; n < N; n += G) {
        const bi_i32x4 xr = bi_rsrc(x + (int64_t)n * P * CIN, (uint32_t)P * CIN * 2);
        const bi_i32x4 yr = bi_rsrc(y + (int64_t)n * P * CIN, (uint32_t)P * CIN * 2);
        // chunk ch of X -> buffer buf: instruction gi (of XG) = rows 4 gi + lane / 16, physical chunk lane & 15
        // holding logical chunk (lane & 15) ^ (row & 15); rows past the image read 0
        auto issue_x = [&](int ch, int buf) {
            for (int gi = w; gi < L::XG; gi += L::NW) {
                const int row = 4 * gi + (lane >> 4), c = (lane & 15) ^ (row & 15);
                bi_raw_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(smem + buf * L::XBUF + gi * 1024),
                                       16, (row * CIN + ch * L::XK + c * 8) * 2, 0, 0, 0);
            }
        };
        f32x4 acc[L::FW][L::NJ];

        // ================= phase R: T1 = relu(X . Wr^T + br)
        __builtin_amdgcn_s_barrier();   // the previous pair's phase E is done with T2 (the X buffers alias it)
        issue_x(0, 0);
#pragma unroll
        for (int j = 0; j < L::NJ; ++j) {
            const f32x4 b = *(const f32x4*)(br + wq * L::CW + 16 * j + 4 * fq);
#pragma unroll
            for (int i = 0; i < L::FW; ++i) acc[i][j] = b;
        }
        for (int ch = 0; ch < L::NCH; ++ch) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of chunk ch has landed
            __builtin_amdgcn_s_barrier();                       // ... every wave's, and chunk ch - 1 is consumed
            if (ch + 1 < L::NCH) issue_x(ch + 1, (ch + 1) & 1);
            const int xb = (ch & 1) * L::XBUF;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                __builtin_amdgcn_sched_barrier(0);   // k-steps do not interleave: bounds the live B fragments
                load_a(ch * 4 + ks + RD, ar[(ks + RD) % RG]);
#pragma unroll
                for (int i = 0; i < L::FW; ++i) {
                    if (i >= nt) continue;
                    const bf16x8 bv = *(const bf16x8*)(smem + xb + i * 16 * L::XPITCH + xoff[ks]);
#pragma unroll
                    for (int j = 0; j < L::NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[ks % RG][j], bv, acc[i][j], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every wave is done with the X buffers: T1 overwrites them
#pragma unroll
        for (int i = 0; i < L::FW; ++i) {
            if (i >= nt) continue;
            const bool ok = 16 * (L::FW * wh + i) + fr < P;
#pragma unroll
            for (int j = 0; j < L::NJ; ++j) {
                bi_u32x2 o = {bi_relu_pk(acc[i][j][0], acc[i][j][1]), bi_relu_pk(acc[i][j][2], acc[i][j][3])};
                if (!ok) o = bi_u32x2{0u, 0u};
                *(bi_u32x2*)(smem + i * 16 * L::PITCH + twr[j]) = o;
            }
        }
        if (w == 0 && lane < CM / 8) *(bi_u32x4*)(smem + L::ZROW * L::PITCH + lane * 16) = bi_u32x4{0u, 0u, 0u, 0u};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();

        // ================= phase M: T2 = relu(conv3x3(T1) . Wm^T + bm)
#pragma unroll
        for (int j = 0; j < L::NJ; ++j) {
            const f32x4 b = *(const f32x4*)(bm + wq * L::CW + 16 * j + 4 * fq);
#pragma unroll
            for (int i = 0; i < L::FW; ++i) acc[i][j] = b;
        }
        for (int tap = 0; tap < 9; ++tap) {
            const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
            int tq[L::FW];   // this tap's T1 row of the lane's pixel in fragment i, swizzle folded in
#pragma unroll
            for (int i = 0; i < L::FW; ++i) {
                const int p = 16 * (L::FW * wh + i) + fr;
                int py = (int)(((float)p + 0.5f) * rcp_w);
                int px = p - py * W;
                if (px < 0) { --py; px += W; } else if (px >= W) { ++py; px -= W; }
                const bool ok = p < P && (unsigned)(py + dy) < (unsigned)H && (unsigned)(px + dx) < (unsigned)W;
                const int q = ok ? p + dy * W + dx : L::ZROW;
                tq[i] = (q * L::PITCH) | ((fq ^ (q & 15)) << 4);
            }
#pragma unroll
            for (int cs = 0; cs < CM / 32; ++cs) {
                __builtin_amdgcn_sched_barrier(0);   // k-steps do not interleave: bounds the live B fragments
                load_a(L::NR + tap * (CM / 32) + cs + RD, ar[(cs + RD) % RG]);
#pragma unroll
                for (int i = 0; i < L::FW; ++i) {
                    if (i >= nt) continue;
                    const bf16x8 bv = *(const bf16x8*)(smem + ((tq[i] ^ ((cs & 3) << 6)) + (cs >> 2) * 256));
#pragma unroll
                    for (int j = 0; j < L::NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[cs % RG][j], bv, acc[i][j], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every wave is done with T1: T2 overwrites it
#pragma unroll
        for (int i = 0; i < L::FW; ++i) {
            if (i >= nt) continue;
#pragma unroll
            for (int j = 0; j < L::NJ; ++j)
                *(bi_u32x2*)(smem + i * 16 * L::PITCH + twr[j]) =
                    bi_u32x2{bi_relu_pk(acc[i][j][0], acc[i][j][1]), bi_relu_pk(acc[i][j][2], acc[i][j][3])};
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();

        // ================= phase E: y = relu(T2 . We^T + be + x), CIN / CE passes of CE channels
        for (int g = 0; g < L::NPASS; ++g) {
            const int cg = g * L::CE + wq * (L::CE / 4) + 4 * fq;   // + 16 j: this lane's 4 output channels
#pragma unroll
            for (int j = 0; j < L::NJE; ++j) {   // the first NJE channel tiles of acc hold the pass
                const f32x4 b = *(const f32x4*)(be + cg + 16 * j);
#pragma unroll
                for (int i = 0; i < L::FW; ++i) acc[i][j] = b;
            }
            bi_u32x2 res[L::FW][L::NJE];   // the pass's residual, in flight during its k-steps (rows past the image: 0)
#pragma unroll
            for (int i = 0; i < L::FW; ++i)
#pragma unroll
                for (int j = 0; j < L::NJE; ++j) res[i][j] = bi_raw_load2(xr, pvo[i], (cg + 16 * j) * 2, 0);
#pragma unroll
            for (int s = 0; s < L::NE; ++s) {
                const int u = L::NR + L::NM + g * L::NE + s;
                __builtin_amdgcn_sched_barrier(0);   // k-steps do not interleave: bounds the live B fragments
                load_a(u + RD >= L::NU ? u + RD - L::NU : u + RD, ar[(s + RD) % RG]);   // past the pair: the next pair's Wr
#pragma unroll
                for (int i = 0; i < L::FW; ++i) {
                    if (i >= nt) continue;
                    const bf16x8 bv = *(const bf16x8*)(smem + i * 16 * L::PITCH + ((t2rd ^ ((s & 3) << 6)) + (s >> 2) * 256));
#pragma unroll
                    for (int j = 0; j < L::NJE; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[s % RG][j], bv, acc[i][j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int i = 0; i < L::FW; ++i) {
                if (i >= nt) continue;
#pragma unroll
                for (int j = 0; j < L::NJE; ++j) {   // rows past the image fall past num_records: dropped
                    const f32x4 v = acc[i][j];
                    const bi_u32x2 rv = res[i][j];
                    const bi_u32x2 o = {bi_relu_pk(v[0] + bi_lo(rv[0]), v[1] + bi_hi(rv[0])),
                                        bi_relu_pk(v[2] + bi_lo(rv[1]), v[3] + bi_hi(rv[1]))};
                    bi_raw_store2(o, yr, pvo[i], (cg + 16 * j) * 2, 0);
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing weight prefetch drains before exit
}

int num_cus_bi() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

}  // namespace

bool cbw_bottleneck_img_fits(int cin, int cm, int H, int W) {
    return cin == 1024 && cm == 256 && H > 0 && W > 0 && H * W <= BiL<1024, 256, 15>::ROWS;
}

hipError_t cbw_bottleneck_img(const uint16_t* x, uint16_t* y, const uint16_t* wr, const float* br, const uint16_t* wm,
                              const float* bm, const uint16_t* we, const float* be, int N, int H, int W, int cin,
                              int cm, hipStream_t st) {
    if (N <= 0) return hipSuccess;
    if (!cbw_bottleneck_img_fits(cin, cm, H, W)) return hipErrorInvalidValue;
    using L = BiL<1024, 256, 15>;
    const int G = std::min(N, num_cus_bi());
    hipLaunchKernelGGL((bottleneck_img_kernel<1024, 256, 15>), dim3(G), dim3(BI_WAVES * 64), L::LDS, st, (const bf16*)x,
                       (bf16*)y, (const bf16*)wr, br, (const bf16*)wm, bm, (const bf16*)we, be, N, H, W);
    return hipGetLastError();
}
